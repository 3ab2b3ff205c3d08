// solver.hip — estimate_state's solver iteration on the device, for rigid
// (hull-only) scenes: after a residual pass and its reduce, one small
// workgroup turns the accumulator into the next configuration and the next
// surface poses, so a whole frame of iterations is enqueued with no host
// round trip (fsdf_descend, capi.hip descend_device).
//
// Per iteration, the arithmetic of the host loop (capi.hip fsdf_descend around
// fsdf_value_and_gradient) in the same order, from kin_impl.h:
//   chain rule  surface wrenches -> body sums (surfaces in index order) ->
//               subtree sums (children in descending index, as the host's
//               reverse topological loop adds them) -> per joint ∂c/∂q
//               (src/gradientdescent.jl:28-39 through ForwardDiff in the
//               reference; src/tracking.jl:16-21 divides by N)
//   NaiveSolver g = (∂c/∂x / N) ./ divisors, stop at |g| < tolerance, else
//               x += clamp(-rate g, ±max_step) (flash/tracking.py; the
//               un-vendored SimpleGradientDescent.jl, src/tracking.jl:12-15)
//   FK          joint motions in parallel, then composition level by level
//               (each body's product as the host computes it), surface poses
// so x, f and the iteration count equal the host loop's bit for bit.
//
// The pose / pass / reduce launches of later iterations read `flags[0]`
// (SolverState::flags) and return at once after convergence; the remaining
// iterations of the frame cost their (empty) launches only.
#include <hip/hip_runtime.h>

#include "fsdf_internal.h"
#include "kin_impl.h"

namespace fsdf {

namespace {

constexpr int kSolverBlock = 256;

// LDS carve of one step: sub [6 nb] | LR [9 nb] | Lt [3 nb] | R [9 nb] | t [3 nb]
// | Rb [9 nb] | tb [3 nb] | x [nx] | g [nx]
__device__ __forceinline__ void carve(double* lds, int nb, int nx, double** sub, double** LR, double** Lt, double** R,
                                      double** t, double** Rb, double** tb, double** x, double** g) {
  *sub = lds;
  *LR = *sub + 6 * nb;
  *Lt = *LR + 9 * nb;
  *R = *Lt + 3 * nb;
  *t = *R + 9 * nb;
  *Rb = *t + 3 * nb;
  *tb = *Rb + 9 * nb;
  *x = *tb + 3 * nb;
  *g = *x + nx;
}

// FK of the LDS configuration x into LDS R, t, Rb, tb; then the surface poses
// (global) and Rb, tb (global, for the next chain rule). Returns through
// *bad: 1 a zero quaternion / unknown joint, 2 a non-finite pose.
__device__ void fk_and_poses(const SolverTree& T, const SolverState& st, const double* x, double* LR, double* Lt,
                             double* R, double* t, double* Rb, double* tb, int* bad) {
  const int tid = threadIdx.x;
  for (int b = 1 + tid; b < T.nb; b += kSolverBlock) {
    const int k = T.kind[b];
    if (!kin::joint_local(k, T.axis + 3 * b, T.AR + 9 * b, T.At + 3 * b, T.BR + 9 * b, T.Bt + 3 * b,
                          k ? x + T.qoff[b] : x, LR + 9 * b, Lt + 3 * b))
      atomicOr(bad, 1);
  }
  if (tid < 9) {
    const double v = (tid % 4 == 0) ? 1.0 : 0.0;
    R[tid] = v;
    Rb[tid] = v;
  } else if (tid < 12) {
    t[tid - 9] = 0.0;
    tb[tid - 9] = 0.0;
  }
  __syncthreads();
  for (int d = 0; d < T.D; ++d) {
    const int a = T.depth_off[d], e = T.depth_off[d + 1];
    for (int i = a + tid; i < e; i += kSolverBlock) {
      const int b = T.depth_order[i], p = T.parent[b];
      kin::compose(R + 9 * p, t + 3 * p, LR + 9 * b, Lt + 3 * b, T.AR + 9 * b, T.At + 3 * b, R + 9 * b, t + 3 * b,
                   Rb + 9 * b, tb + 3 * b);
    }
    __syncthreads();
  }
  for (int k = tid; k < T.S; k += kSolverBlock) {
    double P[12];
    const int b = T.surface_body[k];
    if (b < 0) {
      for (int i = 0; i < 12; ++i) P[i] = (i % 4 == 0 && i < 9) ? 1.0 : 0.0;
    } else {
      kin::surface_pose(R + 9 * b, t + 3 * b, T.frame_R + 9 * k, T.frame_t + 3 * k, P);
    }
    bool fin = true;
    for (int i = 0; i < 12; ++i) {
      fin = fin && isfinite(P[i]);
      st.poses[12 * k + i] = P[i];
    }
    if (!fin) atomicOr(bad, 2);
  }
  for (int i = tid; i < 9 * T.nb; i += kSolverBlock) st.Rb[i] = Rb[i];
  for (int i = tid; i < 3 * T.nb; i += kSolverBlock) st.tb[i] = tb[i];
}

__global__ __launch_bounds__(kSolverBlock) void solver_init_kernel(SolverTree T, SolverState st) {
  extern __shared__ double lds[];
  __shared__ int bad;
  double *sub, *LR, *Lt, *R, *t, *Rb, *tb, *x, *g;
  carve(lds, T.nb, T.nx, &sub, &LR, &Lt, &R, &t, &Rb, &tb, &x, &g);
  const int tid = threadIdx.x;
  if (tid == 0) bad = 0;
  for (int i = tid; i < T.nx; i += kSolverBlock) x[i] = st.x[i];
  __syncthreads();
  fk_and_poses(T, st, x, LR, Lt, R, t, Rb, tb, &bad);
  __syncthreads();
  if (tid == 0) {
    st.flags[1] = 0;
    st.flags[2] = bad;
    st.flags[0] = bad ? 1 : 0;
    *st.f = 0.0;
  }
}

__global__ __launch_bounds__(kSolverBlock) void solver_step_kernel(SolverTree T, SolverState st,
                                                                   const double* __restrict__ accum) {
  if (st.flags[0]) return;  // converged (or failed): the frame's remaining steps are no-ops
  extern __shared__ double lds[];
  __shared__ int bad, verdict;
  double *sub, *LR, *Lt, *R, *t, *Rb, *tb, *x, *g;
  carve(lds, T.nb, T.nx, &sub, &LR, &Lt, &R, &t, &Rb, &tb, &x, &g);
  const int tid = threadIdx.x;
  if (tid == 0) bad = 0;
  for (int i = tid; i < T.nx; i += kSolverBlock) {
    x[i] = st.x[i];
    g[i] = 0.0;
  }
  // body wrenches: each body's surfaces in index order (fsdf_config_gradient)
  for (int i = tid; i < 6 * T.nb; i += kSolverBlock) {
    const int b = i / 6, j = i - 6 * b;
    double s = 0.0;
    for (int q = T.surf_off[b]; q < T.surf_off[b + 1]; ++q) s += accum[1 + 6 * T.surf_list[q] + j];
    sub[i] = s;
  }
  __syncthreads();
  // subtree sums: parents by height, each adding its children in descending index
  for (int h = 0; h < T.H; ++h) {
    const int a = T.height_off[h], e = T.height_off[h + 1];
    for (int i = tid; i < 6 * (e - a); i += kSolverBlock) {
      const int p = T.height_order[a + i / 6], j = i % 6;
      double s = sub[6 * p + j];
      for (int q = T.child_off[p]; q < T.child_off[p + 1]; ++q) s += sub[6 * T.child_list[q] + j];
      sub[6 * p + j] = s;
    }
    __syncthreads();
  }
  for (int b = 1 + tid; b < T.nb; b += kSolverBlock) {
    const int k = T.kind[b];
    if (k && !kin::joint_gradient(k, T.axis + 3 * b, st.Rb + 9 * b, st.tb + 3 * b, x + T.qoff[b], sub + 6 * b,
                                  g + T.qoff[b]))
      atomicOr(&bad, 1);
  }
  __syncthreads();
  for (int i = tid; i < T.nx; i += kSolverBlock) {
    double gi = g[i] / st.n_points;
    if (st.div) gi = gi / st.div[i];
    g[i] = gi;
  }
  __syncthreads();
  if (tid == 0) {
    double nrm2 = 0.0;  // in index order, as the host sums it
    for (int i = 0; i < T.nx; ++i) nrm2 += g[i] * g[i];
    const double cost = accum[0] + st.weight * 0.0;  // (rigid: the regularizer's sum is 0.0)
    const int it = st.flags[1] + 1;
    st.flags[1] = it;
    *st.f = cost / st.n_points;
    verdict = bad ? 3 : (sqrt(nrm2) < st.tol ? 1 : (it >= st.limit ? 2 : 0));
  }
  __syncthreads();
  const int v = verdict;
  if (v == 3 || v == 1) {  // failed / converged: x stays
    if (tid == 0) {
      st.flags[2] = v == 3 ? 1 : 0;
      st.flags[0] = 1;
    }
    return;
  }
  for (int i = tid; i < T.nx; i += kSolverBlock) {
    const double xi = x[i] + kin::clipped_step(st.rate, g[i], st.max_step);
    x[i] = xi;
    st.x[i] = xi;
  }
  if (v == 2) {  // the last iteration: no pass follows
    if (tid == 0) st.flags[0] = 1;
    return;
  }
  __syncthreads();
  fk_and_poses(T, st, x, LR, Lt, R, t, Rb, tb, &bad);
  __syncthreads();
  if (tid == 0 && bad) {
    st.flags[2] = bad;
    st.flags[0] = 1;
  }
}

size_t solver_lds_bytes(const SolverTree& T) { return (size_t)(42 * T.nb + 2 * T.nx) * sizeof(double); }

}  // namespace

bool solver_fits(int nb, int nx) { return nb >= 1 && (size_t)(42 * nb + 2 * nx) * sizeof(double) <= 65536; }

hipError_t launch_solver_init(const SolverTree& T, const SolverState& st, hipStream_t s) {
  hipLaunchKernelGGL(solver_init_kernel, dim3(1), dim3(kSolverBlock), solver_lds_bytes(T), s, T, st);
  return hipGetLastError();
}

hipError_t launch_solver_step(const SolverTree& T, const SolverState& st, const double* d_accum, hipStream_t s) {
  hipLaunchKernelGGL(solver_step_kernel, dim3(1), dim3(kSolverBlock), solver_lds_bytes(T), s, T, st, d_accum);
  return hipGetLastError();
}

}  // namespace fsdf
