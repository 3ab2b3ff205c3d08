// solver.hip — estimate_state's solver iteration on the device, for rigid
// (hull-only) scenes: after a residual pass and its reduce, one launch turns
// the accumulator into the next configuration, the next surface poses and the
// next pass's posed model, so a whole frame of iterations is enqueued with no
// host round trip (fsdf_descend, capi.hip descend_device; the default for
// rigid scenes, fsdf_set_solver).
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
//   FK          joint motions in parallel, then each body's chain from the
//               root composed in registers (each product as the host's level
//               order computes it), surface poses
// so x, f and the iteration count equal the host loop's bit for bit. Every
// workgroup of the launch runs the whole step on the same inputs (the same
// values) and then poses its 1,024 of the model's pose items (pose_impl.h);
// workgroup 0 alone writes the state, double-buffered by iteration parity.
//
// The pass / reduce / step launches of later iterations read `flags[0]`
// (SolverState::flags) and return at once after convergence; the remaining
// iterations of the frame cost their (empty) launches only.
#include <hip/hip_runtime.h>

#include "fsdf_internal.h"
#include "kin_impl.h"
#include "pose_impl.h"

#ifndef FSDF_SOLVER_TIMES
#define FSDF_SOLVER_TIMES 0  // diagnostic builds: per-phase clocks of the step (capi.hip prints them)
#endif

namespace fsdf {

namespace {

// kSolverBlock: the unit the staging capacities are counted in (kBlobPer /
// kDynPer per thread of a 256-thread group); kStepThreads: the kernels'
// width. 16 waves run the step's per-(body, component) loops in one round
// (6 (nb - 1) = 384 for M64) and publish the 12 S pose entries in one round:
// the M64 step 15.8 -> 12.6 us against 4 waves (profiles/r06/solver_nt/)
constexpr int kSolverBlock = 256;
constexpr int kStepThreads = 1024;

#if FSDF_SOLVER_TIMES
__device__ unsigned long long g_solver_times[64];
#define STAMP(i) \
  if (threadIdx.x == 0 && blockIdx.x == 0 && it0 == 5) g_solver_times[i] = wall_clock64()
#else
#define STAMP(i)
#endif

// The step's LDS: the tree blob (doubles [nd], ints [ni], padded to 16 B) |
// the accumulator [1+6S] | Rb [9nb] | tb [3nb] (the last FK's joint frames:
// read by the chain rule, then overwritten by this step's FK) | x [nx] |
// div [nx] | sub [6nb] | LR [9nb] | Lt [3nb] | R [9nb] | t [3nb] | g [nx] |
// P [12S] (the surface poses the pose items read).
// Every array the level loops touch is here: a level costs LDS latency and a
// barrier, not a global-memory round trip.
struct Lds {
  const double *axis, *AR, *At, *BR, *Bt, *FR, *Ft;
  double *acc, *Rb, *tb, *sub, *LR, *Lt, *R, *t, *x, *g, *div, *P;
  const int32_t *parent, *kind, *qoff, *plist, *poff, *hord, *hoff, *coff, *clist, *soff, *slist, *sbody;
  const int32_t *chlist, *choff;
};

// the doubles after the blob: acc | Rb | tb | x | div | sub | LR | Lt | R | t | g | P (the surface poses)
__host__ __device__ inline size_t work_doubles(int nb, int nx, int S) {
  return 1 + 18 * (size_t)S + 42 * (size_t)nb + 3 * (size_t)nx;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)b, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// The tree blob, the accumulator (optional), Rb / tb and x (+ divisors) into
// LDS: every thread issues all of its loads before its first store, so the
// staging costs one memory latency (the blob is ~23 KB for M64: 6 16-B chunks
// per thread). A copy loop that stores each load before the next one waits a
// full memory round trip (~1-2 us) per element per thread — measured 28 us per
// step that way.
constexpr int kBlobPer = 12;  // 16-B blob chunks per thread: blobs up to 48 KB
constexpr int kDynPer = 8;    // dynamic doubles per thread (accum, Rb|tb, x, div): up to 2,048

template <int NT>
__device__ Lds stage(const SolverTree& T, const SolverState& st, double* lds, const double* accum, int slot) {
  // (per-thread load counts for NT threads: the same totals as kBlobPer / kDynPer at kSolverBlock)
  constexpr int BP = (kBlobPer * kSolverBlock + NT - 1) / NT, DP = (kDynPer * kSolverBlock + NT - 1) / NT;
  const int tid = threadIdx.x, nb = T.nb, nx = T.nx, S = T.S;
  typedef double D2 __attribute__((ext_vector_type(2)));
  // loads: blob chunks, then the dynamic doubles (a flat index over accum | Rb tb | x | div)
  const D2* blob = (const D2*)T.blob;
  D2 bv[BP];
#pragma unroll
  for (int u = 0; u < BP; ++u) {
    const int i = tid + u * NT;
    bv[u] = i < T.chunks16 ? blob[i] : D2{0.0, 0.0};
  }
  const int na = accum ? 1 + 6 * S : 0, nr = accum ? 12 * nb : 0, nd_ = st.div ? nx : 0;
  const int ndyn = na + nr + nx + nd_;
  double dv[DP];
#pragma unroll
  for (int u = 0; u < DP; ++u) {
    const int i = tid + u * NT;
    double v = 0.0;
    if (i < na) v = accum[i];
    else if (i < na + nr) v = st.Rb[(size_t)slot * 12 * nb + (i - na)];  // (Rb | tb adjacent in a slot)
    else if (i < na + nr + nx) v = st.x[(size_t)slot * nx + (i - na - nr)];
    else if (i < ndyn) v = st.div[i - na - nr - nx];
    dv[u] = v;
  }
  Lds L;
  double* d = lds;
  D2* l2 = (D2*)lds;
#pragma unroll
  for (int u = 0; u < BP; ++u) {
    const int i = tid + u * NT;
    if (i < T.chunks16) l2[i] = bv[u];
  }
  L.axis = d + T.axis;
  L.AR = d + T.AR;
  L.At = d + T.At;
  L.BR = d + T.BR;
  L.Bt = d + T.Bt;
  L.FR = d + T.frame_R;
  L.Ft = d + T.frame_t;
  const int32_t* iv = (const int32_t*)(d + T.nd);
  L.parent = iv + T.parent;
  L.kind = iv + T.kind;
  L.qoff = iv + T.qoff;
  L.plist = iv + T.path_list;
  L.poff = iv + T.path_off;
  L.hord = iv + T.height_order;
  L.hoff = iv + T.height_off;
  L.coff = iv + T.child_off;
  L.clist = iv + T.child_list;
  L.soff = iv + T.surf_off;
  L.slist = iv + T.surf_list;
  L.sbody = iv + T.surface_body;
  L.chlist = iv + T.chain_list;
  L.choff = iv + T.chain_off;
  d += 2 * T.chunks16;  // (the blob, padded to 16 B)
  L.acc = d;
  d += 1 + 6 * S;
  L.Rb = d;
  d += 9 * nb;
  L.tb = d;
  d += 3 * nb;
  L.x = d;
  d += nx;
  L.div = st.div ? d : nullptr;
  d += nx;
  L.sub = d;
  d += 6 * nb;
  L.LR = d;
  d += 9 * nb;
  L.Lt = d;
  d += 3 * nb;
  L.R = d;
  d += 9 * nb;
  L.t = d;
  d += 3 * nb;
  L.g = d;
  d += nx;
  L.P = d;
  // the dynamic doubles land at acc (accum | Rb tb | x | div are contiguous
  // there too; without an accumulator x lands at L.x)
#pragma unroll
  for (int u = 0; u < DP; ++u) {
    const int i = tid + u * NT;
    if (i < na + nr) L.acc[i] = dv[u];
    else if (i < ndyn) L.x[i - na - nr] = dv[u];
  }
  for (int i = tid; i < nx; i += NT) L.g[i] = 0.0;
  return L;
}

// FK of L.x into L.R, t, Rb, tb (LDS; *bad |= 1 for a zero quaternion /
// unknown joint). Global memory is not touched: a workgroup barrier after a
// global store waits for the store to complete (its release fence), so every
// store of the step is issued after the last barrier (publish()).
template <int NT>
__device__ void fk(const SolverTree& T, const Lds& L, int* bad, int it0 = -1) {
  (void)it0;  // (FSDF_SOLVER_TIMES: the iteration whose phases are clocked)
  const int tid = threadIdx.x, nb = T.nb;
  for (int b = 1 + tid; b < nb; b += NT) {
    const int k = L.kind[b];
    if (!kin::joint_local(k, L.axis + 3 * b, L.AR + 9 * b, L.At + 3 * b, L.BR + 9 * b, L.Bt + 3 * b,
                          L.x + (k ? L.qoff[b] : 0), L.LR + 9 * b, L.Lt + 3 * b))
      atomicOr(bad, 1);
  }
  if (tid == 0) {  // the root: identity (one thread: no per-lane choice of the destination array)
    for (int i = 0; i < 9; ++i) {
      const double v = (i % 4 == 0) ? 1.0 : 0.0;
      L.R[i] = v;
      L.Rb[i] = v;
    }
    for (int i = 0; i < 3; ++i) {
      L.t[i] = 0.0;
      L.tb[i] = 0.0;
    }
  }
  __syncthreads();
  STAMP(5);
  // one thread per body composes its chain from the root in registers (every
  // ancestor's product as the host's level order computes it: the same bits,
  // no barrier per level); the ancestors' R, t only, and the joint frame
  // Rb, tb = R_parent · joint_to_parent for b itself
  for (int b = 1 + tid; b < nb; b += NT) {
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t[3] = {0, 0, 0}, v[12], w[12], Rp[9], tp[3];
    const int q0 = L.poff[b], q1 = L.poff[b + 1];
    // the next ancestor's joint motion is loaded while this one composes
    double nLR[9], nLt[3];
    int an = L.plist[q0];
    kin::load(L.LR + 9 * an, nLR, 9);
    kin::load(L.Lt + 3 * an, nLt, 3);
    for (int q = q0; q < q1; ++q) {
      const int a = an;
      double LR[9], Lt[3];
#pragma unroll
      for (int e = 0; e < 9; ++e) LR[e] = nLR[e];
#pragma unroll
      for (int e = 0; e < 3; ++e) Lt[e] = nLt[e];
      if (q + 1 < q1) {
        an = L.plist[q + 1];
        kin::load(L.LR + 9 * an, nLR, 9);
        kin::load(L.Lt + 3 * an, nLt, 3);
      }
      (void)a;
#pragma unroll
      for (int e = 0; e < 9; ++e) Rp[e] = R[e];  // (the parent's frame, for b's joint frame below)
#pragma unroll
      for (int e = 0; e < 3; ++e) tp[e] = t[e];
#pragma unroll
      for (int e = 0; e < 12; ++e) v[e] = kin::compose_entry(e, R, t, LR, Lt, nullptr, nullptr);
#pragma unroll
      for (int e = 0; e < 9; ++e) R[e] = v[e];
#pragma unroll
      for (int e = 0; e < 3; ++e) t[e] = v[9 + e];
    }
    // b's joint frame Tb_b = T_parent · joint_to_parent, after the walk (not a
    // branch on the last level inside it: lanes of different depths would run
    // that branch at every level between them)
    {
      double AR[9], At[3];
      kin::load(L.AR + 9 * b, AR, 9);
      kin::load(L.At + 3 * b, At, 3);
#pragma unroll
      for (int e = 0; e < 12; ++e) w[e] = kin::compose_entry(12 + e, Rp, tp, nullptr, nullptr, AR, At);
    }
    kin::store(L.R + 9 * b, v, 9);
    kin::store(L.t + 3 * b, v + 9, 3);
    kin::store(L.Rb + 9 * b, w, 9);
    kin::store(L.tb + 3 * b, w + 9, 3);
  }
  __syncthreads();
}

// The end of a step (and of the init): the surface poses into LDS (a
// non-finite entry marks the frame failed, error 2), then — the next pass's
// pose, in this launch instead of a pose kernel of its own — every work item
// of the model's pose from them (pose_impl.h: world planes, screening pairs,
// stage images, vertices, spheres and scales into the posed model the pass
// reads), the joint frames for the next chain rule, x and — thread 0 — f, the
// iteration count and the done / error flags. Every global store is issued
// after the last barrier (a barrier's release fence would wait for them).
// pose = false: the last iteration (no pass follows) publishes x and the flags only.
template <typename TP, int NT>
__device__ void publish(const SolverTree& T, const SolverState& st, const Lds& L, bool pose, int bad, double f,
                        int it, int done, const LocalModel& lm, const PosedModel& pm) {
  const int tid = threadIdx.x, nb = T.nb, wg = blockIdx.x;
  const int slot = it & 1;  // (the state the next step reads: x, Rb, tb of iteration it)
  __shared__ int nonfinite;
  if (pose) {
    if (tid == 0) nonfinite = 0;
    __syncthreads();
    for (int i = tid; i < 12 * T.S; i += NT) {
      const int k = i / 12, q = i % 12, b = L.sbody[k];
      const double v = b < 0 ? ((q % 4 == 0 && q < 9) ? 1.0 : 0.0)
                             : kin::surface_pose_entry(q, L.R + 9 * b, L.t + 3 * b, L.FR + 9 * k, L.Ft + 3 * k);
      L.P[i] = v;
      if (!isfinite(v)) nonfinite = 1;  // (every writer writes the same value)
    }
    __syncthreads();
    // this workgroup's NT consecutive work items of the pose (whole waves: the
    // total is a multiple of 64, as NT)
    const int item = wg * NT + tid;
    if (item < pose_items(lm))
      pose_item<TP>(lm, L.P, (TP*)pm.planes_w, pm.spheres_w, (TP*)pm.verts_w, (TP*)pm.hscale_w,
                    sizeof(TP) == 8 ? pm.screen_w : nullptr, sizeof(TP) == 8 ? (I4*)pm.image_w : nullptr, item);
  }
  if (wg != 0) return;  // (the state: workgroup 0; every workgroup computed the same values)
  if (pose) {
    double* Rb = st.Rb + (size_t)slot * 12 * nb;
    for (int i = tid; i < 9 * nb; i += NT) Rb[i] = L.Rb[i];
    for (int i = tid; i < 3 * nb; i += NT) Rb[9 * nb + i] = L.tb[i];
  }
  if (it > 0)  // (the init's x is slot 0's own, which its workgroups are reading)
    for (int i = tid; i < T.nx; i += NT) st.x[(size_t)slot * T.nx + i] = L.x[i];
  if (tid == 0) {
    *st.f = f;
    st.flags[1] = it;
    if (pose && nonfinite) {
      st.flags[2] = 2;
      st.flags[0] = 1;
    } else if (bad || done) {
      st.flags[2] = bad ? 1 : 0;
      st.flags[0] = 1;
    }
  }
}

template <typename TP>
__global__ __launch_bounds__(kStepThreads) void solver_init_kernel(SolverTree T, SolverState st, LocalModel lm,
                                                                   PosedModel pm) {
  extern __shared__ double lds[];
  __shared__ int bad;
  const int tid = threadIdx.x;
  if (tid == 0) bad = 0;
  const Lds L = stage<kStepThreads>(T, st, lds, nullptr, 0);  // (x0 in slot 0)
  __syncthreads();
  fk<kStepThreads>(T, L, &bad);  // (ends with a barrier; the host zeroed the flags before this launch)
  publish<TP, kStepThreads>(T, st, L, true, bad, 0.0, 0, 0, lm, pm);
}

// One step over NT threads (solver_step_kernel: kStepThreads). (A launch
// that also did the pass's final reduce — its last workgroup running the step
// — measured no faster: the hand-off between workgroups costs what the launch
// saves; branch archive/fused-reduce-step)
template <typename TP, int NT>
__device__ void step_body(const SolverTree& T, const SolverState& st, const double* __restrict__ accum,
                          double* __restrict__ lds, const LocalModel& lm, const PosedModel& pm, int it_before) {
  // (the frame's done flag loads with the stage's loads; the check waits for it.
  // Workgroup 0 of this launch may set it at its end: a workgroup that reads it
  // set returns — no pass follows a converged step)
  const int done = __builtin_nontemporal_load(st.flags);
  __shared__ int bad, verdict;
  __shared__ double s_f;
  const int tid = threadIdx.x, nb = T.nb, nx = T.nx;
#if FSDF_SOLVER_TIMES
  const int it0 = it_before;
#endif
  STAMP(0);
  if (tid == 0) bad = 0;
  const Lds L = stage<NT>(T, st, lds, accum, it_before & 1);
  if (done) return;  // converged (or failed): the frame's remaining steps are no-ops (uniform)
  __syncthreads();
  STAMP(1);
  if (T.chains) {
    // chains (every non-root body has <= 1 child): body b's subtree sum along
    // its chain, deepest first — sub[a] = own[a] + sub[child], own[a] the body's
    // surfaces summed in index order from 0.0: fsdf_config_gradient's additions
    // in its order, no level barriers. First every own[a] (one thread per (a,
    // component); into L.LR, free until the FK), then one thread per (b,
    // component) walks its chain, the next four own[] loads issued before
    // their additions (a chain level costs an addition, not a chain of
    // dependent LDS loads)
    double* own = L.LR;
    for (int i = tid; i < 6 * (nb - 1); i += NT) {
      const int a = 1 + i / 6, j = i % 6;
      double o = 0.0;
      for (int u = L.soff[a]; u < L.soff[a + 1]; ++u) o += L.acc[1 + 6 * L.slist[u] + j];
      own[6 * a + j] = o;
    }
    __syncthreads();
    for (int i = tid; i < 6 * (nb - 1); i += NT) {
      const int b = 1 + i / 6, j = i % 6;
      const int q0 = L.choff[b];
      int q = L.choff[b + 1] - 1;
      double s = own[6 * L.chlist[q] + j];
      for (--q; q >= q0; q -= 4) {
        double v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = q - k >= q0 ? own[6 * L.chlist[q - k] + j] : 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (q - k >= q0) s = v[k] + s;
      }
      L.sub[6 * b + j] = s;
    }
    __syncthreads();
  } else {
    // body wrenches: each body's surfaces in index order (fsdf_config_gradient)
    for (int i = tid; i < 6 * nb; i += NT) {
      const int b = i / 6, j = i - 6 * b;
      double s = 0.0;
      for (int q = L.soff[b]; q < L.soff[b + 1]; ++q) s += L.acc[1 + 6 * L.slist[q] + j];
      L.sub[i] = s;
    }
    __syncthreads();
    // subtree sums: parents by height, each adding its children in descending
    // index; a narrow tree (<= 10 parents per height) in one wave, its levels
    // ordered by wave-local fences instead of workgroup barriers
    if (T.narrow) {
      if (tid < 64) {
        for (int h = 0; h < T.H; ++h) {
          const int a = L.hoff[h], e = L.hoff[h + 1];
          if (tid < 6 * (e - a)) {
            const int p = L.hord[a + tid / 6], j = tid % 6;
            double s = L.sub[6 * p + j];
            for (int q = L.coff[p]; q < L.coff[p + 1]; ++q) s += L.sub[6 * L.clist[q] + j];
            L.sub[6 * p + j] = s;
          }
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
        }
      }
      __syncthreads();
    } else {
      for (int h = 0; h < T.H; ++h) {
        const int a = L.hoff[h], e = L.hoff[h + 1];
        for (int i = tid; i < 6 * (e - a); i += NT) {
          const int p = L.hord[a + i / 6], j = i % 6;
          double s = L.sub[6 * p + j];
          for (int q = L.coff[p]; q < L.coff[p + 1]; ++q) s += L.sub[6 * L.clist[q] + j];
          L.sub[6 * p + j] = s;
        }
        __syncthreads();
      }
    }
  }
  STAMP(2);
  for (int b = 1 + tid; b < nb; b += NT) {
    const int k = L.kind[b];
    if (k && !kin::joint_gradient(k, L.axis + 3 * b, L.Rb + 9 * b, L.tb + 3 * b, L.x + L.qoff[b], L.sub + 6 * b,
                                  L.g + L.qoff[b]))
      atomicOr(&bad, 1);
  }
  __syncthreads();
  for (int i = tid; i < nx; i += NT) {
    double gi = L.g[i] / st.n_points;
    if (L.div) gi = gi / L.div[i];
    L.g[i] = gi;
  }
  __syncthreads();
  STAMP(3);
  // |g|^2 in index order, as the host sums it: wave 0 squares in parallel, lane
  // 0 adds the squares in order, read straight from the lanes (readlane: no
  // LDS round trip per term)
  double nrm2 = 0.0;
  if (nx <= 64) {
    if (tid < 64) {
      const double gi = tid < nx ? L.g[tid] : 0.0;
      const double sq = gi * gi;
      for (int i = 0; i < nx; ++i) nrm2 += readlane_f64(sq, i);
    }
  } else if (tid == 0) {
    for (int i = 0; i < nx; ++i) nrm2 += L.g[i] * L.g[i];
  }
  const int it = it_before + 1;
  if (tid == 0) {
    const double cost = L.acc[0] + st.weight * 0.0;  // (rigid: the regularizer's sum is 0.0)
    s_f = cost / st.n_points;
    verdict = bad ? 3 : (sqrt(nrm2) < st.tol ? 1 : (it >= st.limit ? 2 : 0));
  }
  __syncthreads();
  const int v = verdict;
  const double f = s_f;
  if (v == 3 || v == 1) {  // failed / converged: x stays
    publish<TP, NT>(T, st, L, false, v == 3, f, it, 1, lm, pm);
    return;
  }
  for (int i = tid; i < nx; i += NT) L.x[i] = L.x[i] + kin::clipped_step(st.rate, L.g[i], st.max_step);
  if (v == 2) {  // the last iteration: no pass follows
    __syncthreads();
    publish<TP, NT>(T, st, L, false, 0, f, it, 1, lm, pm);
    return;
  }
  __syncthreads();
  STAMP(4);
#if FSDF_SOLVER_TIMES
  fk<NT>(T, L, &bad, it0);  // (ends with a barrier)
#else
  fk<NT>(T, L, &bad);  // (ends with a barrier)
#endif
  STAMP(6);
  publish<TP, NT>(T, st, L, true, bad, f, it, 0, lm, pm);
  STAMP(9);
}

template <typename TP>
__global__ __launch_bounds__(kStepThreads) void solver_step_kernel(SolverTree T, SolverState st,
                                                                   const double* __restrict__ accum, LocalModel lm,
                                                                   PosedModel pm, int it_before) {
  extern __shared__ double lds[];
  step_body<TP, kStepThreads>(T, st, accum, lds, lm, pm, it_before);
}

size_t solver_lds_bytes(const SolverTree& T) {
  return (size_t)T.chunks16 * 16 + work_doubles(T.nb, T.nx, T.S) * sizeof(double);
}

}  // namespace

// the blob (27 nb + 12 S doubles + ni ints) within kBlobPer chunks per thread,
// the dynamic loads within kDynPer, the whole carve within 64 KB of LDS
bool solver_fits(int nb, int nx, int S, int ni) {
  const size_t blob = ((27 * (size_t)nb + 12 * (size_t)S) * 8 + (size_t)ni * 4 + 15) / 16;
  const size_t dyn = 1 + 6 * (size_t)S + 12 * (size_t)nb + 2 * (size_t)nx;
  return nb >= 1 && blob <= (size_t)kBlobPer * kSolverBlock && dyn <= (size_t)kDynPer * kSolverBlock &&
         blob * 16 + work_doubles(nb, nx, S) * 8 <= 65536;
}

// one workgroup per kStepThreads work items of the pose, each running the whole
// step (the same arithmetic on the same inputs: the same values) and then
// posing its items — the pose in the step's launch, at the latency of one step
static dim3 solver_grid(const LocalModel& lm) {
  const int g = (pose_items(lm) + kStepThreads - 1) / kStepThreads;
  return dim3((unsigned)(g > 0 ? g : 1));
}

hipError_t launch_solver_init(const SolverTree& T, const SolverState& st, const LocalModel& lm,
                              const PosedModel& pm, int precision, hipStream_t s) {
  if (precision == 64)
    hipLaunchKernelGGL(solver_init_kernel<double>, solver_grid(lm), dim3(kStepThreads), solver_lds_bytes(T), s, T, st,
                       lm, pm);
  else
    hipLaunchKernelGGL(solver_init_kernel<float>, solver_grid(lm), dim3(kStepThreads), solver_lds_bytes(T), s, T, st,
                       lm, pm);
  return hipGetLastError();
}

void solver_times(unsigned long long* out) {
#if FSDF_SOLVER_TIMES
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_solver_times), 16 * sizeof(unsigned long long));
#else
  for (int i = 0; i < 16; ++i) out[i] = 0;
#endif
}

hipError_t launch_solver_step(const SolverTree& T, const SolverState& st, const double* d_accum,
                              const LocalModel& lm, const PosedModel& pm, int precision, int it_before,
                              hipStream_t s) {
  if (precision == 64)
    hipLaunchKernelGGL(solver_step_kernel<double>, solver_grid(lm), dim3(kStepThreads), solver_lds_bytes(T), s, T, st,
                       d_accum, lm, pm, it_before);
  else
    hipLaunchKernelGGL(solver_step_kernel<float>, solver_grid(lm), dim3(kStepThreads), solver_lds_bytes(T), s, T, st,
                       d_accum, lm, pm, it_before);
  return hipGetLastError();
}


}  // namespace fsdf
