/*
 * flash_oracle.c — CPU restatement of the Flash.jl residual pass.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed
 * CPU baseline — never as the product path.
 *
 * What it restates (reference file:line):
 *   skin(state)(x) = minimum(s(x) for s in all_surfaces)      src/Flash.jl:265-268
 *       first surface wins ties (Julia left-fold `minimum`)    -> oracle_skin
 *   s(x) for ConvexGeometry = gjk!(cache, pose, Translation(x)).signed_distance
 *                                                              src/Flash.jl:233-250
 *       restated as the exact signed distance to conv(V):      -> oracle_hull_sdf
 *         inside:  max_f (n_f·x − d_f);  outside: distance to the closest
 *         boundary point (EnhancedGJK @404de6a9 is un-vendored: outside it
 *         converges to this value; inside it returns a termination-simplex
 *         estimate, replaced here by the exact value — DESIGN.md §2).
 *   pose of a surface = transform_to_root(state, frame)       src/Flash.jl:248
 *       given as R|t per hull; world planes/vertices          -> oracle_pose_model
 *   s(x) for InterpolatingGeometry = SpatialFields surface     src/Flash.jl:207-213
 *       restated as f/|∇f| of the XCubed + affine RBF fit    -> oracle_rbf_skin
 *       (KAT test/runtests.jl:17 holds; the notebook costs do not: DESIGN.md §2)
 *   cost = Σ_p skin(p)^2                                      src/gradientdescent.jl:32
 *       plus the per-hull wrench sums that carry ∂cost/∂pose   -> oracle_cost_accum
 *
 * Arithmetic is written operation-for-operation like the gfx950 kernel
 * (point-cloud-signed-distance_amd/csrc/sdf_kernels.hip): explicit fma(),
 * -ffp-contract=off, correctly rounded sqrt and division, so per-hull values
 * and the argmin k* agree bit for bit. Parity of the SDF values themselves
 * against the Julia reference is UNPINNED for convex hulls (no reference test
 * touches ConvexGeometry); they are pinned by closed forms and
 * an independent numpy formulation in tests/.
 *
 * fp32 contexts: skin_impl.h holds the per-surface restatement once for a
 * working precision and is instantiated for fp64 and for fp32 (oracle_*_f32:
 * the kernel's hull_sdf<float> / rbf_field<float> operation for operation,
 * world rows rounded once from the fp64 pose as pose_body<float> does), so
 * fp32 k*, d* and ∇d* are checked bit for bit as well.
 *
 * Build: oracle/Makefile (gcc -O2 -mfma -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define FX 24 /* stride of the per-face extra record, as in the kernel */

static inline void xf_point(const double* P, const double* v, double* o) {
  o[0] = fma(P[0], v[0], fma(P[1], v[1], fma(P[2], v[2], P[9])));
  o[1] = fma(P[3], v[0], fma(P[4], v[1], fma(P[5], v[2], P[10])));
  o[2] = fma(P[6], v[0], fma(P[7], v[1], fma(P[8], v[2], P[11])));
}
static inline void rot_vec(const double* P, const double* v, double* o) {
  o[0] = fma(P[0], v[0], fma(P[1], v[1], P[2] * v[2]));
  o[1] = fma(P[3], v[0], fma(P[4], v[1], P[5] * v[2]));
  o[2] = fma(P[6], v[0], fma(P[7], v[1], P[8] * v[2]));
}
/* The per-surface restatement (world pose, hull SDF, RBF skin, scene minimum),
 * once for fp64 contexts and once for fp32 contexts (names suffixed _f32). */
#define R double
#define RF(x) x
#define RFMA fma
#define RSQRT sqrt
#define RFABS fabs
#define R_CERT_EPS 1e-13
#include "skin_impl.h"
#undef R
#undef RF
#undef RFMA
#undef RSQRT
#undef RFABS
#undef R_CERT_EPS
#define R float
#define RF(x) x##_f32
#define RFMA fmaf
#define RSQRT sqrtf
#define RFABS fabsf
#define R_CERT_EPS 4e-6f
#include "skin_impl.h"
#undef R
#undef RF
#undef RFMA
#undef RSQRT
#undef RFABS
#undef R_CERT_EPS


/* adds 2s ∂s/∂(w, a, b) and 2s ∂s/∂c_i (coefficients fixed) into acc:
 * acc[0..n) λ_w, acc[n] λ_a, acc[n+1..n+4) λ_b, acc[n+4+3i..] E_i */
static void rbf_adjoint(const double* rows, int nc, const double* p, double* acc) {
  double F[10], s, g[3], c, invG;
  rbf_field(rows, nc, p, F);
  rbf_skin_from_field(F, &s, g, &c, &invG);
  const double two_s = 2.0 * s, dsdf = invG;
  const double ux = -c * F[1], uy = -c * F[2], uz = -c * F[3];
  for (int i = 0; i < nc; ++i) {
    const double* cw = rows + 4 * i;
    const double dx = p[0] - cw[0], dy = p[1] - cw[1], dz = p[2] - cw[2];
    const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
    const double r = sqrt(r2);
    const double e = fma(dx, ux, fma(dy, uy, dz * uz));
    acc[i] += two_s * fma(dsdf * r2, r, 3.0 * r * e);
    const double k1 = fma(3.0 * r, dsdf, r2 > 0 ? (3.0 * e) / r : 0.0);
    const double k2 = 3.0 * r;
    const double sc = -two_s * cw[3];
    double* E = acc + nc + 4 + 3 * i;
    E[0] += sc * fma(k1, dx, k2 * ux);
    E[1] += sc * fma(k1, dy, k2 * uy);
    E[2] += sc * fma(k1, dz, k2 * uz);
  }
  acc[nc] += two_s * dsdf;
  acc[nc + 1] += two_s * fma(dsdf, p[0], ux);
  acc[nc + 2] += two_s * fma(dsdf, p[1], uy);
  acc[nc + 3] += two_s * fma(dsdf, p[2], uz);
}


/* Culled scene SDF (the CPU baseline's second leg, BASELINE.md §2 / SURVEY.md
 * §8d "culling disabled and enabled"): the same per-surface values as
 * skin_one, visited in order of a bounding-sphere lower bound
 * d_k(p) >= |p − c_k| − r_k (c_k the world vertex centroid, r_k the largest
 * vertex distance, padded), stopping once the bound exceeds the best value by
 * a rounding margin; ties keep the smaller k whatever the visiting order, so
 * the result equals the brute-force minimum bit for bit. RBF skins have no
 * cheap bound and are always evaluated. */
static void hull_spheres(const oracle_posed* m, double* sph) {
  for (int32_t k = 0; k < m->K; ++k) {
    double c[3] = {0, 0, 0}, r2 = 0;
    const int v0 = m->vert_off[k], v1 = m->vert_off[k + 1];
    for (int v = v0; v < v1; ++v)
      for (int j = 0; j < 3; ++j) c[j] += m->verts_w[4 * v + j];
    for (int j = 0; j < 3; ++j) c[j] /= (double)(v1 - v0);
    for (int v = v0; v < v1; ++v) {
      const double e2 = dist2_to(m->verts_w + 4 * v, c);
      r2 = e2 > r2 ? e2 : r2;
    }
    sph[4 * k] = c[0]; sph[4 * k + 1] = c[1]; sph[4 * k + 2] = c[2];
    sph[4 * k + 3] = sqrt(r2) * (1.0 + 1e-12) + 1e-12;
  }
}

static void skin_one_culled(const oracle_posed* m, const double* sph, const double* p, double* d, int32_t* k,
                            double* g) {
  double best = INFINITY, gb[3] = {0, 0, 0};
  int32_t bk = 0x7fffffff;
  double lb[1024];
  int32_t ord[1024], nh = 0;
  for (int32_t kk = 0; kk < m->S; ++kk) {
    const int32_t si = m->surf_index[kk];
    double dk, gk[3];
    if (si < 0) {
      const int r = -si - 1, r0 = m->rbf_row_off[r];
      oracle_rbf_skin(m->rbf_rows + 4 * r0, m->rbf_row_off[r + 1] - r0 - 1, p, &dk, gk);
      if (dk < best || (dk == best && kk < bk)) { best = dk; bk = kk; gb[0] = gk[0]; gb[1] = gk[1]; gb[2] = gk[2]; }
      continue;
    }
    const double* c = sph + 4 * si;
    const double l = sqrt(dist2_to(p, c)) - c[3];
    int32_t j = nh++;  /* insertion by lower bound */
    while (j > 0 && lb[j - 1] > l) { lb[j] = lb[j - 1]; ord[j] = ord[j - 1]; --j; }
    lb[j] = l;
    ord[j] = kk;
  }
  const double mrg = 1e-9 * (1.0 + fabs(p[0]) + fabs(p[1]) + fabs(p[2]));
  for (int32_t j = 0; j < nh; ++j) {
    if (lb[j] - mrg > best) break;
    const int32_t kk = ord[j];
    double dk, gk[3];
    oracle_hull_sdf(m, m->surf_index[kk], p, &dk, gk);
    if (dk < best || (dk == best && kk < bk)) { best = dk; bk = kk; gb[0] = gk[0]; gb[1] = gk[1]; gb[2] = gk[2]; }
  }
  *d = best;
  *k = bk == 0x7fffffff ? 0 : bk;
  g[0] = gb[0]; g[1] = gb[1]; g[2] = gb[2];
}

/* oracle_skin with lower-bound culling (identical results; <= 1024 surfaces). */
int32_t oracle_skin_culled(const oracle_posed* m, const double* pts, int64_t n, double* d_out, int32_t* k_out,
                           double* g_out, int32_t threads) {
  if (m->S > 1024) return -1;
  double sph[4 * 1024];
  hull_spheres(m, sph);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 256)
#endif
  for (int64_t i = 0; i < n; ++i) {
    double d, g[3];
    int32_t k;
    skin_one_culled(m, sph, pts + 3 * i, &d, &k, g);
    if (d_out) d_out[i] = d;
    if (k_out) k_out[i] = k;
    if (g_out) { g_out[3 * i] = g[0]; g_out[3 * i + 1] = g[1]; g_out[3 * i + 2] = g[2]; }
  }
  (void)threads;
  return 0;
}


/* cost = Σ d*² and the per-hull wrench sums (layout of include/flashsdf.h):
 * accum[0] = Σ d², accum[1+6k..] = Σ 2d∇d, Σ 2d (p×∇d) over points with k*=k.
 * Serial in point order (the reference's `sum` is pairwise; both agree to
 * rounding, compared at 1e-9 relative). */
void oracle_cost_accum(const oracle_posed* m, const double* pts, int64_t n, double* accum) {
  int32_t R = 0;
  for (int32_t kk = 0; kk < m->S; ++kk) R += m->surf_index[kk] < 0;
  const int32_t len = 1 + 6 * m->S + (R ? m->rbf_acc_off[R] : 0);
  memset(accum, 0, sizeof(double) * (size_t)len);
  for (int64_t i = 0; i < n; ++i) {
    const double* p = pts + 3 * i;
    double d, g[3];
    int32_t k;
    skin_one(m, p, &d, &k, g);
    accum[0] = fma(d, d, accum[0]);
    const int32_t si = m->surf_index[k];
    if (si < 0) {
      const int r = -si - 1, r0 = m->rbf_row_off[r];
      rbf_adjoint(m->rbf_rows + 4 * r0, m->rbf_row_off[r + 1] - r0 - 1, p,
                  accum + 1 + 6 * m->S + m->rbf_acc_off[r]);
      continue;
    }
    const double w = 2.0 * d;
    double* a = accum + 1 + 6 * k;
    a[0] += w * g[0];
    a[1] += w * g[1];
    a[2] += w * g[2];
    a[3] += w * fma(p[1], g[2], -(p[2] * g[1]));
    a[4] += w * fma(p[2], g[0], -(p[0] * g[2]));
    a[5] += w * fma(p[0], g[1], -(p[1] * g[0]));
  }
}

/* doRaycast (src/depthsensors.jl:56-81) for every ray on the scene SDF:
 * secant march, |step| <= 0.4, EPS 1e-5, <= 60 steps, NaN if the final
 * |SDF| > 1000·EPS. Same operation order as raycast_kernel. */
void oracle_raycast(const oracle_posed* m, const double* o, const double* rays, int64_t n, double* depth,
                    int32_t threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
  for (int64_t i = 0; i < n; ++i) {
    const double* r = rays + 3 * i;
    double dist = 0.0, est = -1.0, last, g[3], p[3];
    int32_t kk, k = 0;
    p[0] = o[0] + dist * r[0]; p[1] = o[1] + dist * r[1]; p[2] = o[2] + dist * r[2];
    skin_one(m, p, &last, &kk, g);
    while (fabs(last) > 1e-5 && k < 60) {
      double step = -last / est;
      const double a = fabs(step);
      step = copysign(a < 0.4 ? a : 0.4, step);
      dist += step;
      p[0] = o[0] + dist * r[0]; p[1] = o[1] + dist * r[1]; p[2] = o[2] + dist * r[2];
      double v;
      skin_one(m, p, &v, &kk, g);
      est = (v - last) / step;
      last = v;
      ++k;
    }
    depth[i] = fabs(last) > 1000.0 * 1e-5 ? NAN : dist;
  }
  (void)threads;
}

/* Threads the oracle would use (for the bench's cpu_baseline "cores"). */
int32_t oracle_max_threads(void) {
#ifdef _OPENMP
  return (int32_t)omp_get_max_threads();
#else
  return 1;
#endif
}