// Host side of the RBF interpolating skins around the GPU pass
// (src/Flash.jl:143-213: SpatialFields.InterpolatingSurface(points, values,
// XCubed(), true) over the posed surface points, value 0, and skeleton
// points, value -1):
//   fsdf_rbf_solve    the per-pass weight solve [A P; Pᵀ 0][w; a; b] = [v; 0],
//                     A_ij = |c_i - c_j|^3, P_i = (1, c_iᵀ), by LU with partial
//                     pivoting (kept for the adjoint);
//   fsdf_rbf_adjoint  the pass's RBF accumulator block (λ = Σ 2s ∂s/∂(w,a,b),
//                     E_j = Σ 2s ∂s/∂c_j) -> G_j = ∂c/∂c_j through the solve:
//                     μ = M⁻ᵀλ (M is symmetric), ∂(w,a,b)/∂c_j by implicit
//                     differentiation of M u = rhs.
// flash/rbf.py solve / chain are the numpy twins the tests compare with.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "flashsdf.h"

namespace {

// In-place LU with partial pivoting of the row-major m x m matrix A
// (PA = LU, unit lower L below the diagonal, U on and above it).
int lu_factor(int m, double* A, int32_t* piv) {
  for (int k = 0; k < m; ++k) {
    int p = k;
    double best = std::fabs(A[k * m + k]);
    for (int i = k + 1; i < m; ++i) {
      const double v = std::fabs(A[i * m + k]);
      if (v > best) { best = v; p = i; }
    }
    if (!(best > 0.0) || !std::isfinite(best)) return FSDF_ERR_DEGENERATE;
    piv[k] = p;
    if (p != k)
      for (int j = 0; j < m; ++j) {
        const double t = A[k * m + j];
        A[k * m + j] = A[p * m + j];
        A[p * m + j] = t;
      }
    const double inv = 1.0 / A[k * m + k];
    for (int i = k + 1; i < m; ++i) {
      const double l = A[i * m + k] * inv;
      A[i * m + k] = l;
      if (l != 0.0)
        for (int j = k + 1; j < m; ++j) A[i * m + j] -= l * A[k * m + j];
    }
  }
  return FSDF_OK;
}

// Solves A x = b in place with the factorization of lu_factor.
void lu_solve(int m, const double* LU, const int32_t* piv, double* b) {
  for (int k = 0; k < m; ++k)
    if (piv[k] != k) {
      const double t = b[k];
      b[k] = b[piv[k]];
      b[piv[k]] = t;
    }
  for (int i = 1; i < m; ++i) {
    double s = b[i];
    for (int j = 0; j < i; ++j) s -= LU[i * m + j] * b[j];
    b[i] = s;
  }
  for (int i = m - 1; i >= 0; --i) {
    double s = b[i];
    for (int j = i + 1; j < m; ++j) s -= LU[i * m + j] * b[j];
    b[i] = s / LU[i * m + i];
  }
}

}  // namespace

extern "C" int fsdf_rbf_solve(int32_t n, const double* centres, const double* values, double* u, double* lu,
                              int32_t* piv) {
  if (n < 1 || !centres || !values || !u || !lu || !piv) return FSDF_ERR_ARG;
  const int m = n + 4;
  for (int i = 0; i < n; ++i) {
    const double* ci = centres + 3 * i;
    for (int j = 0; j < n; ++j) {
      const double* cj = centres + 3 * j;
      const double dx = ci[0] - cj[0], dy = ci[1] - cj[1], dz = ci[2] - cj[2];
      const double r = std::sqrt(dx * dx + dy * dy + dz * dz);
      lu[i * m + j] = r * r * r;
    }
    double* row = lu + i * m + n;
    row[0] = 1.0;
    row[1] = ci[0];
    row[2] = ci[1];
    row[3] = ci[2];
    for (int c = 0; c < 4; ++c) lu[(n + c) * m + i] = row[c];
  }
  for (int a = n; a < m; ++a)
    for (int b = n; b < m; ++b) lu[a * m + b] = 0.0;
  const int rc = lu_factor(m, lu, piv);
  if (rc) return rc;
  for (int i = 0; i < n; ++i) u[i] = values[i];
  for (int c = 0; c < 4; ++c) u[n + c] = 0.0;
  lu_solve(m, lu, piv, u);
  for (int i = 0; i < m; ++i)
    if (!std::isfinite(u[i])) return FSDF_ERR_DEGENERATE;
  return FSDF_OK;
}

extern "C" int fsdf_rbf_adjoint(int32_t n, const double* centres, const double* u, const double* lu,
                                const int32_t* piv, const double* block, double* G, double* work) {
  if (n < 1 || !centres || !u || !lu || !piv || !block || !G || !work) return FSDF_ERR_ARG;
  const int m = n + 4;
  double* mu = work;  // μ = M⁻ᵀ λ = M⁻¹ λ (M symmetric)
  std::memcpy(mu, block, (size_t)m * sizeof(double));
  lu_solve(m, lu, piv, mu);
  const double* E = block + m;
  const double *w = u, *b = u + n + 1, *mw = mu, *mb = mu + n + 1;
  for (int j = 0; j < n; ++j) {
    const double* cj = centres + 3 * j;
    // Σ_i mw_i ∇φ(c_j - c_i) and Σ_i w_i ∇φ(c_j - c_i), ∇φ(d) = 3 |d| d
    double sm[3] = {0.0, 0.0, 0.0}, sw[3] = {0.0, 0.0, 0.0};
    for (int i = 0; i < n; ++i) {
      const double* ci = centres + 3 * i;
      const double d[3] = {cj[0] - ci[0], cj[1] - ci[1], cj[2] - ci[2]};
      const double r3 = 3.0 * std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
      for (int c = 0; c < 3; ++c) {
        const double g = r3 * d[c];
        sm[c] += mw[i] * g;
        sw[c] += w[i] * g;
      }
    }
    for (int c = 0; c < 3; ++c) {
      const double term = w[j] * sm[c] + mw[j] * sw[c] + mw[j] * b[c] + w[j] * mb[c];
      G[3 * j + c] = E[3 * j + c] - term;
    }
  }
  return FSDF_OK;
}
