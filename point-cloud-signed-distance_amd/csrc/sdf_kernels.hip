// sdf_kernels.hip — the residual pass of Flash.jl on CDNA4 (gfx950).
//
// Reference semantics (src/Flash.jl:265-268, src/gradientdescent.jl:28-39):
//   d*(p)  = minimum(s_k(p) for k in surfaces)       first k wins ties
//   s_k(p) = gjk!(cache, pose_k, Translation(p)).signed_distance   (:238-243)
//   c      = Σ_p d*(p)^2
// restated here as the EXACT signed distance to the convex polytope conv(V_k):
//   inside / on the surface:  max_f (n_f·p − d_f)
//   outside:                  Euclidean distance to the closest boundary point
// (EnhancedGJK returns the same value outside; its penetration value inside is a
//  termination-simplex estimate and is replaced by the exact one — DESIGN.md §2).
//
// Kernel design:
//   * one lane per point; each wave owns 64 consecutive (Hilbert-ordered)
//     resident points;
//   * exact-safe culling: hulls are dropped for the whole wave from its
//     bounding sphere, then per lane by |p−c_k|−r_k against min(upper bound,
//     best so far) plus a rounding margin; a wave evaluates hull k iff any
//     lane needs it, each lane's best-first seed first;
//   * a hull evaluation stages the hull once into the wave's LDS stage; the
//     plane max is an fp32 screen (packed FMA, two faces per instruction) with
//     an exact fp64 fix-up, and the closest feature a certified descent walk;
//   * per-hull wrench sums are segmented by k* inside the wave (ballot loop +
//     DPP sums), owned in LDS rows by lane k mod 64, combined per block in
//     fixed wave order, then reduced over blocks in fixed order: the whole
//     reduction is deterministic for a given (n, grid).
//
// All arithmetic is written with explicit fma() and compiled with
// -ffp-contract=off so that oracle/flash_oracle.c reproduces every per-hull
// value bit for bit (the argmin k* must match exactly).

#include "fsdf_internal.h"
#include "pose_impl.h"

#include <hip/hip_ext.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

namespace fsdf {

template <typename T> __device__ __forceinline__ T mfma_(T a, T b, T c);
template <> __device__ __forceinline__ double mfma_(double a, double b, double c) {
  return __builtin_fma(a, b, c);
}
template <> __device__ __forceinline__ float mfma_(float a, float b, float c) {
  return __builtin_fmaf(a, b, c);
}
template <typename T> __device__ __forceinline__ T tsqrt(T a);
template <> __device__ __forceinline__ double tsqrt(double a) { return __builtin_sqrt(a); }
template <> __device__ __forceinline__ float tsqrt(float a) { return __builtin_sqrtf(a); }
template <typename T> __device__ __forceinline__ T tinf();
template <> __device__ __forceinline__ double tinf() { return __builtin_huge_val(); }
template <> __device__ __forceinline__ float tinf() { return __builtin_huge_valf(); }

// (pose_item, the pose's work items: pose_impl.h)
template <typename T>
__device__ __forceinline__ void pose_body(const LocalModel& lm, const double* __restrict__ poses,
                                          T* __restrict__ planes_w, float* __restrict__ spheres_w,
                                          T* __restrict__ verts_w, T* __restrict__ hscale_w,
                                          float* __restrict__ screen_w, I4* __restrict__ image_w) {
  pose_item<T>(lm, poses, planes_w, spheres_w, verts_w, hscale_w, screen_w, image_w,
               (int)(blockIdx.x * blockDim.x + threadIdx.x));
}

// Poses from global memory (uploaded by a copy), or — for up to kPoseArgMax
// surfaces — straight from the kernel arguments: the launch carries the 12·S
// doubles, each workgroup copies them into LDS, and the per-pass host-to-device
// copy (a blit kernel of its own) disappears from the step.
// skip (optional): a device flag; set, the launch does nothing (the device
// solver loop's passes after convergence, solver.hip)
template <typename T>
__global__ __launch_bounds__(kBlock) void pose_kernel(LocalModel lm, const double* __restrict__ poses,
                                                      T* __restrict__ planes_w, float* __restrict__ spheres_w,
                                                      T* __restrict__ verts_w, T* __restrict__ hscale_w,
                                                      float* __restrict__ screen_w, I4* __restrict__ image_w,
                                                      const int* __restrict__ skip) {
  if (skip && *skip) return;
  pose_body<T>(lm, poses, planes_w, spheres_w, verts_w, hscale_w, screen_w, image_w);
}
template <typename T>
__global__ __launch_bounds__(kBlock) void pose_kernel_args(LocalModel lm, PoseArgs pa, T* __restrict__ planes_w,
                                                           float* __restrict__ spheres_w, T* __restrict__ verts_w,
                                                           T* __restrict__ hscale_w, float* __restrict__ screen_w,
                                                           I4* __restrict__ image_w) {
  __shared__ double sp[12 * kPoseArgMax];
  for (int i = threadIdx.x; i < 12 * lm.S; i += kBlock) sp[i] = pa.v[i];
  __syncthreads();
  pose_body<T>(lm, sp, planes_w, spheres_w, verts_w, hscale_w, screen_w, image_w);
}

// ---------------------------------------------------------------------------
// Closest point on triangle (a, b, c) to p — Voronoi-region walk.
// ---------------------------------------------------------------------------
template <typename T> struct Row4 { typedef T __attribute__((ext_vector_type(4))) type; };
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// reg: the Voronoi region of the result — 0, 1, 2 vertex a, b, c; 3, 4, 5 the
// edge a→b, b→c, c→a (face edges 0, 1, 2); 6 the interior.
// Branch-free: every region test is evaluated, the first that holds (the
// classic early-return order) selects the region, and the region's one
// division (edge parameter, or the interior's 1/(va+vb+vc)) runs once — a
// wave whose lanes sit in different regions no longer executes every
// region's division in turn. Each region's result is the same expression as
// in the early-return form (oracle/flash_oracle.c), so the bits are too.
template <typename T>
__device__ __forceinline__ void closest_on_triangle(T px, T py, T pz, const typename Row4<T>::type& A,
                                                    const typename Row4<T>::type& B,
                                                    const typename Row4<T>::type& C, T& qx, T& qy, T& qz,
                                                    int& reg) {
  const T ax = A[0], ay = A[1], az = A[2];
  const T bx = B[0], by = B[1], bz = B[2];
  const T cx = C[0], cy = C[1], cz = C[2];
  const T abx = bx - ax, aby = by - ay, abz = bz - az;
  const T acx = cx - ax, acy = cy - ay, acz = cz - az;
  const T apx = px - ax, apy = py - ay, apz = pz - az;
  const T d1 = mfma_(abx, apx, mfma_(aby, apy, abz * apz));
  const T d2 = mfma_(acx, apx, mfma_(acy, apy, acz * apz));
  const T bpx = px - bx, bpy = py - by, bpz = pz - bz;
  const T d3 = mfma_(abx, bpx, mfma_(aby, bpy, abz * bpz));
  const T d4 = mfma_(acx, bpx, mfma_(acy, bpy, acz * bpz));
  const T vc = mfma_(d1, d4, -(d3 * d2));
  const T cpx = px - cx, cpy = py - cy, cpz = pz - cz;
  const T d5 = mfma_(abx, cpx, mfma_(aby, cpy, abz * cpz));
  const T d6 = mfma_(acx, cpx, mfma_(acy, cpy, acz * cpz));
  const T vb = mfma_(d5, d2, -(d1 * d6));
  const T va = mfma_(d3, d6, -(d5 * d4));
  const T e43 = d4 - d3, e56 = d5 - d6;
  const bool c0 = d1 <= (T)0 && d2 <= (T)0;
  const bool c1 = d3 >= (T)0 && d4 <= d3;
  const bool c3 = vc <= (T)0 && d1 >= (T)0 && d3 <= (T)0;
  const bool c2 = d6 >= (T)0 && d5 <= d6;
  const bool c5 = vb <= (T)0 && d2 >= (T)0 && d6 <= (T)0;
  const bool c4 = va <= (T)0 && e43 >= (T)0 && e56 >= (T)0;
  reg = c0 ? 0 : (c1 ? 1 : (c3 ? 3 : (c2 ? 2 : (c5 ? 5 : (c4 ? 4 : 6)))));
  // the region's quotient: edge a→b t = d1/(d1−d3), c→a t = d2/(d2−d6),
  // b→c t = e43/(e43+e56), interior inv = 1/(va+vb+vc); vertices none
  T num = (T)1, den = (va + vb) + vc;
  if (reg == 3) { num = d1; den = d1 - d3; }
  if (reg == 5) { num = d2; den = d2 - d6; }
  if (reg == 4) { num = e43; den = e43 + e56; }
  if (reg <= 2) { num = (T)0; den = (T)1; }
  const T t = num / den;
  // q = fma(s1, D1, base) (+ the interior's second term)
  const bool edge_bc = reg == 4, edge_ca = reg == 5, inner = reg == 6;
  const T bsx = edge_bc ? bx : ax, bsy = edge_bc ? by : ay, bsz = edge_bc ? bz : az;
  const T dx1 = edge_bc ? cx - bx : (edge_ca ? acx : abx);
  const T dy1 = edge_bc ? cy - by : (edge_ca ? acy : aby);
  const T dz1 = edge_bc ? cz - bz : (edge_ca ? acz : abz);
  const T s1 = inner ? vb * t : t;
  const T q1x = mfma_(s1, dx1, bsx), q1y = mfma_(s1, dy1, bsy), q1z = mfma_(s1, dz1, bsz);
  const T w_ = vc * t;
  qx = inner ? mfma_(w_, acx, q1x) : q1x;
  qy = inner ? mfma_(w_, acy, q1y) : q1y;
  qz = inner ? mfma_(w_, acz, q1z) : q1z;
  if (reg <= 2) {
    qx = reg == 0 ? ax : (reg == 1 ? bx : cx);
    qy = reg == 0 ? ay : (reg == 1 ? by : cy);
    qz = reg == 0 ? az : (reg == 1 ? bz : cz);
  }
}

// Inward edge-plane value of edge u -> w of a face with unit normal n:
//   m = n x (w - u),  s = m·p − m·u   (s >= 0 on the triangle's side).
// Same operation order as oracle/flash_oracle.c (its pose step precomputes m, m·u).
template <typename T>
__device__ __forceinline__ T edge_value(const typename Row4<T>::type& n, const typename Row4<T>::type& u,
                                        const typename Row4<T>::type& w, T px, T py, T pz) {
  const T e0 = w[0] - u[0], e1 = w[1] - u[1], e2 = w[2] - u[2];
  const T m0 = mfma_(n[1], e2, -(n[2] * e1));
  const T m1 = mfma_(n[2], e0, -(n[0] * e2));
  const T m2 = mfma_(n[0], e1, -(n[1] * e0));
  const T o = mfma_(m0, u[0], mfma_(m1, u[1], m2 * u[2]));
  return mfma_(m0, px, mfma_(m1, py, mfma_(m2, pz, -o)));
}

// Posed model as the pass kernel sees it (device pointers, world frame).
template <typename T>
struct PassModel {
  int K;  // hulls
  int S;  // surfaces (hulls + RBF skins), the k* index space
  int R;  // RBF skins
  int stage_bytes;  // LDS stage per wave (bytes, multiple of 16)
  int planes64;     // f64 contexts: the fp64 planes are staged too (LocalModel::planes64)
  const int32_t* __restrict__ hull_surface;  // [K] surface index of hull h
  const int32_t* __restrict__ surface_kind;  // [S] FSDF_SURFACE_*
  const int32_t* __restrict__ rbf_surface;   // [R] surface index of RBF skin r
  const int32_t* __restrict__ rbf_row_off;   // [R+1] rows (n centres + 1 poly row)
  const int32_t* __restrict__ rbf_acc_off;   // [R+1] offsets in the RBF accumulator block
  const T* __restrict__ rbf_rows;            // [rows][4] (c, w) ... (a, b)
  const int32_t* __restrict__ face_off;
  const int32_t* __restrict__ vert_off;
  const I4* __restrict__ face_rows;          // [F] packed local vertex / neighbour indices
  const T* __restrict__ planes;
  const T* __restrict__ verts;
  const T* __restrict__ hscale;
  const float* __restrict__ spheres;
  const float* __restrict__ screen;          // fp32 screening pairs (f64 contexts)
  const I4* __restrict__ image;              // per-hull stage images (planes64; PosedModel::image_w)
};

// Per-workgroup LDS hull table, filled once in the kernel prologue (row K is
// a sentinel holding face_off[K] / vert_off[K]): the per-lane culling loops and
// every hull evaluation read it at LDS latency instead of a global round trip.
typedef float F4 __attribute__((ext_vector_type(4)));
struct HullRow {
  F4 sphere;      // world centroid + radius (f32, exact-safe culling)
  F4 box[4];      // world oriented box: (centre, 0), 3 x (body axis, half extent)
  int f0, v0;     // first face / vertex of the hull
  double hscale;  // certificate scale max_v |v|_1
};
static_assert(sizeof(HullRow) == 96, "HullRow is 96 bytes");

// Lower bound of hull k's signed distance at x from its oriented box (the hull
// lies inside the box): with u_i = |a_i·(x − c)| − e_i, outside the box
// d_k(x) >= |max(u, 0)| (distance to the box); inside, the hull's inner ball
// around x fits in the box, so d_k(x) >= max_i u_i. 1-Lipschitz in x. f32
// rounding (~1e-6 of |x|_1 + |c|_1 + the bound, |c|_1 <= |c_k|_1 + 3 r_k) is
// inside the culling margins. Returns max_i u_i and s = |max(u, 0)|^2: the
// bound is sqrt(s) when max_i u_i > 0, else max_i u_i.
__device__ __forceinline__ float box_bound(const HullRow& h, float x, float y, float z, float& s) {
  const F4 c = h.box[0];
  const float qx = x - c[0], qy = y - c[1], qz = z - c[2];
  float mx = -__builtin_huge_valf();
  s = 0.0f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const F4 a = h.box[1 + i];
    const float u = fabsf(__builtin_fmaf(a[0], qx, __builtin_fmaf(a[1], qy, a[2] * qz))) - a[3];
    mx = fmaxf(mx, u);
    const float pu = fmaxf(u, 0.0f);
    s = __builtin_fmaf(pu, pu, s);
  }
  return mx;
}
// box lower bound <= t
__device__ __forceinline__ bool box_within(const HullRow& h, float x, float y, float z, float t) {
  float s;
  const float mx = box_bound(h, x, y, z, s);
  // (bitwise & throughout: short-circuit && on lane values becomes exec-mask
  // branches; every operand here is cheap and already loaded)
  return ((mx <= 0.0f) & (mx <= t)) | ((mx > 0.0f) & (t >= 0.0f) & (s <= t * t));
}
__device__ __forceinline__ float box_lower(const HullRow& h, float x, float y, float z) {
  float s;
  const float mx = box_bound(h, x, y, z, s);
  return mx <= 0.0f ? mx : __builtin_sqrtf(s);
}

// Lane need test of hull k at threshold tb = min(ub, best) + margin: hull k is
// needed unless |p-c_k| - r_k > tb (tested without a sqrt: |p-c_k|^2 <=
// (tb + r_k)^2) or its box bound exceeds tb.
__device__ __forceinline__ bool needs_at(const HullRow& h, float x, float y, float z, float tb) {
  const F4 sp = h.sphere;
  const float dx = x - sp[0], dy = y - sp[1], dz = z - sp[2];
  const float dist2 = __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz));
  const float t = tb + sp[3];
  return (t >= 0.0f) & (dist2 <= t * t) & box_within(h, x, y, z, tb);
}

// Bounding sphere of the wave's points (f32, wave-uniform): every valid lane's
// point p satisfies |p - c| <= r up to f32 rounding (covered by the margins).
struct WaveSphere {
  float x, y, z, r;
};

// fill the table (whole workgroup; ends with a barrier) and return the
// culling-margin scale smax = max_k |c_k|_1 + 2 r_k (wave-uniform)
template <typename T>
__device__ __forceinline__ float load_hull_table(const PassModel<T>& m, HullRow* __restrict__ ht) {
  for (int k = threadIdx.x; k <= m.K; k += (int)blockDim.x) {
    HullRow r;
    const F4* b = (const F4*)(m.spheres + kBoundFloats * k);  // row K (sentinel) is not read
    r.sphere = k < m.K ? b[0] : F4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) r.box[i] = k < m.K ? b[1 + i] : F4{0.f, 0.f, 0.f, 0.f};
    r.f0 = m.face_off[k];
    r.v0 = m.vert_off[k];
    r.hscale = k < m.K ? (double)m.hscale[k] : 0.0;
    ht[k] = r;
  }
  __syncthreads();
  float smax = 0.f;
  for (int k = threadIdx.x & 63; k < m.K; k += 64) {
    const F4 sp = ht[k].sphere;
    smax = fmaxf(smax, fabsf(sp[0]) + fabsf(sp[1]) + fabsf(sp[2]) + 2.0f * sp[3]);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) smax = fmaxf(smax, __shfl_xor(smax, off, 64));
  return smax;
}

constexpr int kMaxRbfAcc = kMaxRbfAccum;
#ifndef FSDF_HPART
#define FSDF_HPART 4
#endif
constexpr int kHpart = FSDF_HPART;  // waves per chunk in the hull-partitioned pass (2 or 4)
static_assert(kHpart == 2 || kHpart == 4, "FSDF_HPART is 2 or 4");
// workgroups of the hull-partitioned and the one-chunk-per-wave pass
// (pass_kernel NB; 512-thread workgroups measured slower for both)
constexpr int kHpartBlock = kPassBlock;
// hpart_default_limits: models with at least kHpartFullHulls hulls use the
// M64-measured tiers, smaller ones kHpartSmall4 / kHpartSmall2 (measured on
// IRB140, C2)
constexpr int kHpartFullHulls = 32;
constexpr int64_t kHpartSmall4 = 98304;
constexpr int64_t kHpartSmall2 = 327680;
// planned pass up to (fsdf_set_plan max_points -1): above it the unplanned
// grid measured faster — M64 between 2^19 and 2^20 points, IRB140 between
// 393,216 and 2^19 (the planned reduction's extra launch outweighs a pass that
// is already short; profiles/r04/hpart_sweep_c2.jsonl)
constexpr int64_t kPlanMaxFull = 524288;
constexpr int64_t kPlanMaxSmall = 393216;
// ... and from above kPlanMinPoints: below it the unplanned 4-way tier measured
// faster for both models (2^16 points: M64 0.0644 vs 0.0662 ms, IRB140 0.0433
// vs 0.0448 — the planned reduction's second launch is not paid back)
constexpr int64_t kPlanMinPoints = 98304;
constexpr int kAliasBlock = kPassBlock;
// scene_eval's best-first seed takes max(sphere, box) lower bounds below this
// many hulls and the sphere bound alone at or above it (round 5 A/B, DESIGN §7:
// sphere-only at M64 = 64 hulls 0.0489 -> 0.0460 ms pass at 2^17, 0.0908 ->
// 0.0899 at 2^20; at C2 = 7 hulls 0.0680 -> 0.0687, so the box stays there)
constexpr int kSeedBoxMaxHulls = 32;

// The one diagnostic build (-DFSDF_WAVE_TIMES=1, tools/wave_times.py): a
// per-wave timeline with per-phase 100 MHz clocks and event counts; every hook
// below compiles to nothing in the product library.
#ifndef FSDF_WAVE_TIMES
#define FSDF_WAVE_TIMES 0
#endif
#if FSDF_WAVE_TIMES
// per wave-iteration, packed 16-bit fields:
//   ev[0]: hull evaluations | screen rejections << 16 | slow evaluations << 32 | walk steps << 48
//   ev[1]: seed evaluations | needing lanes << 16 | wave candidates << 32 | full fp64 scans << 48
//   ph[0]: 10-ns units in hull staging | screen | fast path | closest-feature search
//   ph[1]: culling | RBF | segmented reduction + stores | descent walk (within the search)
//   ev[2]: lane-evaluations through the closest-feature search | those whose
//          hull won the lane | lanes spared the search by the h_max bound |
//          10-ns units in the candidate need tests of phase C
constexpr int kWtWaves = kPassBlock / 64;
__shared__ unsigned long long fsdf_wave_ev[kWtWaves][3];
__shared__ bool fsdf_wt_slow[64 * kWtWaves];  // per lane: the last hull_sdf ran its search
__shared__ unsigned long long fsdf_wave_ph[kWtWaves][2];
//   ph2[0]: 10-ns units in walk certificates | walk closest points | vertex-
//           region lane-certificates | fan iterations (max over lanes, per step)
//   ph2[1]: 10-ns units in the screen loop | screen fix-up | edge-region
//           lane-certificates | interior-region lane-certificates
__shared__ unsigned long long fsdf_wave_ph2[kWtWaves][2];
#endif
__device__ __forceinline__ uint64_t wt_now() {
#if FSDF_WAVE_TIMES
  return __builtin_amdgcn_s_memrealtime();
#else
  return 0;
#endif
}
// adds the time since t0 to phase field f (0..7); returns now
__device__ __forceinline__ uint64_t wt_add(int f, uint64_t t0) {
#if FSDF_WAVE_TIMES
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) fsdf_wave_ph[threadIdx.x >> 6][f >> 2] += (t1 - t0) << (16 * (f & 3));
  return t1;
#else
  return t0;
#endif
}
// sub-phase clocks / counts (ph2 fields 0..7)
__device__ __forceinline__ uint64_t wt_add2(int f, uint64_t t0) {
#if FSDF_WAVE_TIMES
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) fsdf_wave_ph2[threadIdx.x >> 6][f >> 2] += (t1 - t0) << (16 * (f & 3));
  return t1;
#else
  return t0;
#endif
}
__device__ __forceinline__ void wt_count2(int f, uint64_t v) {
#if FSDF_WAVE_TIMES
  if ((threadIdx.x & 63) == 0) fsdf_wave_ph2[threadIdx.x >> 6][f >> 2] += v << (16 * (f & 3));
#endif
}
// adds v to event field f (0..7) of this wave-iteration
__device__ __forceinline__ void wt_count(int f, uint64_t v) {
#if FSDF_WAVE_TIMES
  if ((threadIdx.x & 63) == 0) fsdf_wave_ev[threadIdx.x >> 6][f >> 2] += v << (16 * (f & 3));
#endif
}
// the event counters (fsdf_kernel_stats) are off in the timeline build: their
// contended atomics would dominate the timed windows
__device__ __forceinline__ bool count_events(const unsigned long long* stats) {
  return !FSDF_WAVE_TIMES && stats != nullptr;
}
#ifndef FSDF_PASS_WAVES_PER_SIMD
#define FSDF_PASS_WAVES_PER_SIMD 4
#endif
constexpr int kPassWavesPerSimd = FSDF_PASS_WAVES_PER_SIMD;  // occupancy target (VGPR budget 512/w)

// Row-chunked per-wave LDS staging (RBF centre rows). Must be called with
// every lane of the wave active (wave-uniform control flow).
template <typename T>
__device__ __forceinline__ void stage_rows(T* __restrict__ lds, const T* __restrict__ src, int rows) {
  typedef typename Row4<T>::type R;
  const int lane = threadIdx.x & 63;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // prior reads of this stage precede the overwrite
  for (int r = lane; r < rows; r += 64) *(R*)(lds + 4 * r) = *(const R*)(src + 4 * r);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One bulk copy of everything hull k's evaluation reads — plane rows, vertex
// rows, packed face rows — into this wave's LDS stage: every 16-byte chunk of
// the hull is loaded before any is stored, so the wave pays ONE global-memory
// latency per hull evaluation; all later reads (broadcast plane reads, per-lane
// triangle / neighbour / certificate reads) are LDS. Whole wave active.
#ifndef FSDF_PLANE_BATCH
#define FSDF_PLANE_BATCH 8
#endif
constexpr int kPlaneBatch = FSDF_PLANE_BATCH;  // plane rows per LDS batch (power of 2, >= 2)
constexpr int kWalkSteps = 24;  // descent-walk cap before the exhaustive stage C

// Consecutive regions of 16-byte chunks: n0 from s0, n1 from s1, n2 from s2,
// n3 from s3.
__device__ __forceinline__ void stage_hull(void* __restrict__ lw, const I4* __restrict__ s0, int n0,
                                           const I4* __restrict__ s1, int n1, const I4* __restrict__ s2, int n2,
                                           const I4* __restrict__ s3 = nullptr, int n3 = 0) {
  const int P = n0, Q = P + n1, N3 = Q + n2, N = N3 + n3;
  const int lane = threadIdx.x & 63;
  I4* dst = (I4*)lw;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  for (int c0 = 0; c0 < N; c0 += 8 * 64) {
    I4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = min(c0 + 64 * j + lane, N - 1);
      const I4* src = c < P ? s0 + c : (c < Q ? s1 + (c - P) : (c < N3 ? s2 + (c - Q) : s3 + (c - N3)));
      v[j] = *src;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // lanes past the end hold chunk N-1 (clamped load) and store it there
      // again: same bits, and no exec-mask branch per store
      dst[min(c0 + 64 * j + lane, N - 1)] = v[j];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One contiguous region (a hull's stage image, PosedModel::image_w): the same
// one-latency bulk copy with no region selects.
__device__ __forceinline__ void stage_image(void* __restrict__ lw, const I4* __restrict__ src, int N) {
  const int lane = threadIdx.x & 63;
  I4* dst = (I4*)lw;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  for (int c0 = 0; c0 < N; c0 += 8 * 64) {
    I4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = src[min(c0 + 64 * j + lane, N - 1)];
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[min(c0 + 64 * j + lane, N - 1)] = v[j];
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
__device__ __forceinline__ T plane_h(const typename Row4<T>::type& pl, T px, T py, T pz) {
  return mfma_(pl[0], px, mfma_(pl[1], py, mfma_(pl[2], pz, -pl[3])));
}

template <typename T> __device__ __forceinline__ T cert_eps();
template <> __device__ __forceinline__ double cert_eps() { return 1e-13; }
template <> __device__ __forceinline__ float cert_eps() { return 4e-6f; }

// packed face row: (i0 | i1<<16, i2 | n0<<16, n1 | n2<<16, 0) with i_j the
// hull-local vertex indices and n_e the hull-local face across edge e (i_e -> i_e+1)
// Decoded with one variable 64-bit shift, no selects: with a lane-divergent j
// the compiler turns a select chain into a switch, i.e. an exec-mask branch
// tree (~25 scalar instructions and 6 branches per decode in the fan walk).
__device__ __forceinline__ int fr_vert(const I4& r, int j) {
  const uint64_t w = ((uint64_t)(uint32_t)r[1] << 32) | (uint32_t)r[0];
  return (int)((w >> (16 * j)) & 0xffff);
}
__device__ __forceinline__ int fr_nbr(const I4& r, int e) {
  const uint64_t w = ((uint64_t)(uint32_t)r[2] << 32) | (uint32_t)r[1];
  return (int)((w >> (16 * e + 16)) & 0xffff);
}

// Local optimality certificate of q = the closest point of triangle f (in
// Voronoi region reg) to p: q is the closest point of the convex hull iff
// w = p − q lies in the hull's normal cone at q (exact characterisation):
//   edge u→v of f, shared with face g:  m_f·w <= 0 and m_g·w <= 0 (m the
//     in-plane inward edge normals; m·w is the edge value of p since q is on
//     the edge line);
//   vertex v:  w·(u − v) <= 0 for every neighbour u of v — the fan of faces
//     around v is walked through the packed neighbour rows (<= 32 steps).
// When the test fails it names the faces holding strictly closer points (a
// descent step): across the edge, g; at a vertex whose edge v→u is violated,
// the face g of that edge in the fan and the face across it (n1, n2; -1 =
// none; the current face f is never repeated). An interior point is
// certified iff p is above f's plane; a fan longer than 32 gives no
// certificate and no step. Tolerances accept rounding-level violations (a
// false certificate moves the answer by O(tol^2)). oracle/flash_oracle.c:
// cert_step mirrors every operation.
template <typename T, typename LP>
__device__ __forceinline__ bool cert_step(T px, T py, T pz, int f, int reg, const LP& lp,
                                          const typename Row4<T>::type* __restrict__ lv,
                                          const I4* __restrict__ lf, T scale, int& n1, int& n2,
                                          int* __restrict__ fan_it = nullptr) {
  typedef typename Row4<T>::type R;
  n1 = -1;
  n2 = -1;
  // interior of triangle f: q is p's projection on f's plane, optimal iff p is
  // on the outer side (the plane supports the hull)
  if (reg == 6) return plane_h<T>(lp[f], px, py, pz) > (T)0;
  const I4 fr = lf[f];
  if (reg >= 3) {
    const int e = reg - 3;
    const R U = lv[fr_vert(fr, e)], W = lv[fr_vert(fr, e + 1 - 3 * (e == 2))];
    const int g = fr_nbr(fr, e);
    const T sf = edge_value<T>(lp[f], U, W, px, py, pz);
    const T sg = edge_value<T>(lp[g], W, U, px, py, pz);
    // |m| = |W − U|: the tolerance is a lateral offset of eps (|p|_1 + scale)
    const T tol = cert_eps<T>() * (((fabs(px) + fabs(py)) + fabs(pz)) + scale) *
                  ((fabs(W[0] - U[0]) + fabs(W[1] - U[1])) + fabs(W[2] - U[2]));
    if (sf <= tol && sg <= tol) return true;
    if (sg > tol && g != f) n1 = g;
    return false;
  }
  const int v = fr_vert(fr, reg);
  const R V = lv[v];
  const T wx = px - V[0], wy = py - V[1], wz = pz - V[2];
  const T tol = cert_eps<T>() * ((fabs(wx) + fabs(wy)) + fabs(wz)) * scale;
  int g = f, j = reg;
  I4 r = fr;
  for (int it = 0; it < 32; ++it) {
    if (fan_it) *fan_it = it + 1;
    const int g2 = fr_nbr(r, j);  // across edge v -> u
    const R Un = lv[fr_vert(r, j + 1 - 3 * (j == 2))];
    const T dot = mfma_(wx, Un[0] - V[0], mfma_(wy, Un[1] - V[1], wz * (Un[2] - V[2])));
    if (dot > tol) {
      n1 = g != f ? g : g2;
      n2 = g != f && g2 != f ? g2 : -1;
      return false;
    }
    if (g2 == f) return true;
    r = lf[g2];
    j = 2 - (fr_vert(r, 1) == v) - 2 * (fr_vert(r, 0) == v);  // (the row's vertices are distinct)
    g = g2;
  }
  return false;
}

// ---------------------------------------------------------------------------
// fp32-screened plane max (f64 contexts): the exact first-index argmax of the
// fp64 plane values h_f = n_f·p − d_f, from an fp32 pass over all faces plus
// an fp64 pass over ONE batch of 8.
//   Screen: h'_f = n'·q − d'' in packed fp32 (v_pk_fma_f32: two faces per
//   instruction, plane pairs read through the scalar unit), q = fl32(p − c),
//   c the hull's sphere centre, with |h'_f − h_f| <= E = 16u (|q|_1 + r)
//   (u = 2^-24; |n_i| <= 1 and |d − n·c| <= r). Per batch of 8 faces the
//   maximum b; b1 = best batch maximum, b2 = best over the other batches.
//   If b2 < b1 − 2E, every face g outside the best batch has
//   h_g <= b2 + E < b1 − E <= max h over the batch: the exact maximum lies in
//   the best batch only, and its first-index argmax over the batch's 8 faces
//   (fp64, the same plane_h arithmetic) IS the first-index argmax over all
//   faces — bit for bit the full fp64 scan (the oracle's). Lanes without that
//   margin (near-ties across batches) return false and take the full scan.
// Returns true iff the result is final for every lane that needs it.
// ---------------------------------------------------------------------------
template <typename T>
constexpr bool kStagePairs = sizeof(T) == 8 && FSDF_SCREEN32;
#ifndef FSDF_SCREEN_ILP
#define FSDF_SCREEN_ILP 4
#endif
constexpr int kScreenIlp = FSDF_SCREEN_ILP;  // independent 8-face batches per loop iteration  // see hull_sdf / fsdf_internal.h
typedef float F2v __attribute__((ext_vector_type(2)));

template <typename T, typename LP>
__device__ __forceinline__ bool screen_plane_max(T px, T py, T pz, int k, int f0, int nf, const PassModel<T>& m,
                                                 const HullRow* __restrict__ ht, const void* __restrict__ lw,
                                                 const LP& lp, bool active,
                                                 T bound, T& hA, int& iA, bool& rejected) {
  const F4 sp = ht[k].sphere;
  const float qx = (float)(px - (T)sp[0]), qy = (float)(py - (T)sp[1]), qz = (float)(pz - (T)sp[2]);
  // 2E, plus an absolute term for the fp64 rounding of h_f itself (~1e-15 |p|)
  const float E2 = 32.0f * 5.9604645e-8f * (((fabsf(qx) + fabsf(qy)) + fabsf(qz)) + sp[3]) * 1.0001f +
                   1e-12f * (1.0f + fabsf((float)px) + fabsf((float)py) + fabsf((float)pz) + sp[3]);
  const F2v qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
  const F4* ls = (const F4*)lw;  // staged pairs: two 16-byte chunks each
  const int np = (nf + 1) >> 1;
  float b1 = -__builtin_huge_valf(), b2 = -__builtin_huge_valf();
  int ib = 0;
  // maximum of the 8 faces in pairs i..i+3 (tail: indices clamped to the last pair)
  auto batch_max = [&](int i, bool tail) -> float {
    F4 c[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = tail ? min(i + q, np - 1) : i + q;
      c[2 * q] = ls[2 * j];
      c[2 * q + 1] = ls[2 * j + 1];
    }
    float hm[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const F4 u = c[2 * q], w = c[2 * q + 1];
      const F2v nx = {u[0], u[1]}, ny = {u[2], u[3]}, nz = {w[0], w[1]}, nd = {w[2], w[3]};
      const F2v h = __builtin_elementwise_fma(nx, qx2, __builtin_elementwise_fma(ny, qy2, __builtin_elementwise_fma(nz, qz2, nd)));
      hm[q] = fmaxf(h[0], h[1]);
    }
    return fmaxf(fmaxf(hm[0], hm[1]), fmaxf(hm[2], hm[3]));
  };
  auto update = [&](float mb, int i) {
    b2 = fmaxf(b2, fminf(b1, mb));
    if (mb > b1) { b1 = mb; ib = i; }
  };
  // Early rejection: h_max >= b1 − E, so once b1 − E exceeds a lane's best
  // distance the hull can neither win nor tie for it (d >= h_max). When that
  // holds for every lane that needs the hull, the scan stops (d = +inf).
  const float bf = (float)bound;
  const float thr = bf + E2 + 2.5e-7f * fabsf(bf);
  const uint64_t tw_screen = wt_now();
  rejected = false;
  int i0 = 0;
  // the first 16 faces get a rejection test of their own: a hull that cannot
  // win is usually exposed by its first planes (3 % faster than waiting for
  // the first 32-face round)
  if (np >= 8) {
    const float a = batch_max(0, false), b = batch_max(4, false);
    update(a, 0);
    update(b, 4);
    i0 = 8;
    if (!__any(active && !(b1 > thr))) { rejected = true; return true; }
  }
  // kScreenIlp independent batches per iteration; rejection tested once per round
  for (; i0 + 4 * kScreenIlp <= np; i0 += 4 * kScreenIlp) {
    float mx[kScreenIlp];
#pragma unroll
    for (int u = 0; u < kScreenIlp; ++u) mx[u] = batch_max(i0 + 4 * u, false);
#pragma unroll
    for (int u = 0; u < kScreenIlp; ++u) update(mx[u], i0 + 4 * u);
    if (!__any(active && !(b1 > thr))) { rejected = true; return true; }
  }
  for (; i0 < np; i0 += 4) update(batch_max(i0, i0 + 4 > np), i0);
  if (!__any(active && !(b1 > thr))) { rejected = true; return true; }
  // exact fp64 first-index argmax over the best batch's faces
  const uint64_t tw_fix = wt_add2(4, tw_screen);
  const int fb = 2 * ib;
  hA = -tinf<T>();
  iA = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int f = min(fb + q, nf - 1);
    const T h = plane_h<T>(lp[f], px, py, pz);
    if (h > hA) { hA = h; iA = f; }
  }
  const bool safe = b2 < b1 - E2;
  wt_add2(5, tw_fix);
  return !__any(active && !safe);
}

// ---------------------------------------------------------------------------
// Exact signed distance of p to posed hull k, with its unit gradient.
//   inside / on the surface: max_f h_f, gradient n_{f*} (first max face; f64
//     contexts find it with the fp32 screen above);
//   outside: if the projection on f* lies in triangle f*, d = h_{f*};
//     otherwise the closest point on triangle f* and a descent walk certified
//     by the hull's normal cone at the closest feature (cert_step); a stalled
//     walk falls back to the exhaustive scan of the visible faces.
// `active`: this lane's result is used (gates the wave-uniform slow branches).
// `bound`: the lane's best distance so far (only a result below it matters).
// `lw`: this wave's LDS stage (m.stage_bytes). Whole wave active.
// ---------------------------------------------------------------------------
template <typename T, bool P64 = false>
__device__ __forceinline__ void hull_sdf(T px, T py, T pz, int k, const PassModel<T>& m,
                                         const HullRow* __restrict__ ht, bool active, T bound,
                                         T& d, T& gx, T& gy, T& gz, T* __restrict__ lw,
                                         unsigned long long* __restrict__ stats) {
  typedef typename Row4<T>::type R;
  const int f0 = __builtin_amdgcn_readfirstlane(ht[k].f0);
  const int nf = __builtin_amdgcn_readfirstlane(ht[k + 1].f0) - f0;
  const int v0 = __builtin_amdgcn_readfirstlane(ht[k].v0);
  const int nv = __builtin_amdgcn_readfirstlane(ht[k + 1].v0) - v0;
  uint64_t tw = wt_now();
#if FSDF_WAVE_TIMES
  fsdf_wt_slow[threadIdx.x] = false;
#endif
  // Stage layout: f64 contexts stage the fp32 screening pairs (16 B per face)
  // and read the fp64 planes — needed per lane only for the batch fix-up, the
  // max face and the certificates — from global memory (L1/L2); f32 contexts
  // stage the planes themselves. Then vertex rows and packed face rows.
  constexpr int cpr = (int)sizeof(T) / 4;  // 16-byte chunks per row of 4 T
  const int np2 = kStagePairs<T> ? 2 * ((nf + 1) >> 1) : nf * cpr;  // chunks of region 0
  const I4* src0 = kStagePairs<T> ? (const I4*)(m.screen + 4 * (f0 + k)) : (const I4*)(m.planes + 4 * f0);
  // f64 contexts also stage the fp64 planes (after the pairs) in the
  // one-chunk-per-wave pass (P64: pass_kernel ALIAS, LocalModel::planes64)
  constexpr bool kP64 = kStagePairs<T> && P64;
  const int npl = kP64 ? nf * cpr : 0;
  // (P64: the hull's stage image, whose pair region is nf + 1 chunks)
  const int npr = kP64 ? nf + 1 : np2;
  if constexpr (kP64) {
    stage_image(lw, m.image + (4 * f0 + k + 2 * v0), npr + npl + nv * cpr + nf);
  } else {
    stage_hull(lw, src0, np2, (const I4*)(m.planes + 4 * f0), npl, (const I4*)(m.verts + 4 * v0), nv * cpr,
               m.face_rows + f0, nf);
  }
  tw = wt_add(0, tw);
  const R* lp = kP64 ? (const R*)((const I4*)lw + npr) : (kStagePairs<T> ? (const R*)(m.planes + 4 * f0) : (const R*)lw);
  const R* lv = (const R*)((const I4*)lw + npr + npl);
  const I4* lf = (const I4*)(lv + nv);
  const T scale = (T)ht[k].hscale;
  auto uplane = [&](int f) -> R { return lp[f]; };
  // two independent running maxima (even / odd faces) shorten the serial
  // compare chain; merged with the first-index rule, identical to one chain
  // Batches of kPlaneBatch rows, all of a batch's LDS reads issued before the
  // first is consumed. The loop keeps only the exact maximum (a v_max tree per
  // batch) and the first batch that strictly raised it; the first face of that
  // batch equal to the maximum is then found by re-evaluating the batch (same
  // operations, same bits) — the first-index argmax over all faces. Missing
  // rows of the last batch repeat the last face (same value, never first).
  T hA = -tinf<T>();
  int iA = 0;
  bool screened = false;
  if constexpr (sizeof(T) == 8) {
    bool rejected = false;
    if (FSDF_SCREEN32) screened = screen_plane_max(px, py, pz, k, f0, nf, m, ht, lw, lp, active, bound, hA, iA, rejected);
    if (count_events(stats) && lane_id() == 0) {
      if (rejected) atomicAdd(stats + 20, 1ull);
      else if (!screened) atomicAdd(stats + 19, 1ull);
    }
    if (rejected) wt_count(1, 1);
    else if (!screened) wt_count(7, 1);
    if (rejected) {  // cannot win nor tie for any lane that needs it
      d = tinf<T>();
      gx = gy = gz = (T)0;
      wt_add(1, tw);
      return;
    }
  }
  if (!screened) {
  hA = -tinf<T>();
  int ib = 0;
  auto batch = [&](int i, bool tail) {
    R c[kPlaneBatch];
#pragma unroll
    for (int q = 0; q < kPlaneBatch; ++q) c[q] = uplane(tail ? min(i + q, nf - 1) : i + q);
    T h[kPlaneBatch];
#pragma unroll
    for (int q = 0; q < kPlaneBatch; ++q) h[q] = plane_h<T>(c[q], px, py, pz);
#pragma unroll
    for (int w = 1; w < kPlaneBatch; w *= 2)
#pragma unroll
      for (int q = 0; q + w < kPlaneBatch; q += 2 * w) h[q] = __builtin_fmax(h[q], h[q + w]);
    if (h[0] > hA) { hA = h[0]; ib = i; }
  };
  int i0 = 0;
  for (; i0 + kPlaneBatch <= nf; i0 += kPlaneBatch) batch(i0, false);  // one base address, immediate offsets
  if (i0 < nf) batch(i0, true);
  // faces before batch ib are all < hA, so the window may start earlier
  const int fb = nf >= kPlaneBatch ? min(ib, nf - kPlaneBatch) : ib;
  iA = min(fb + kPlaneBatch - 1, nf - 1);
#pragma unroll
  for (int q = kPlaneBatch - 1; q >= 0; --q) {
    const int f = nf >= kPlaneBatch ? fb + q : min(fb + q, nf - 1);
    if (plane_h<T>(lp[f], px, py, pz) == hA) iA = f;
  }
  }
  tw = wt_add(1, tw);
  if (count_events(stats) && lane_id() == 0) {
    atomicAdd(stats + 9, (unsigned long long)nf);
  }
  const T hmax = hA;
  const int fs = iA;  // hull-local
  const R ns = lp[fs];
  d = hmax;
  gx = ns[0]; gy = ns[1]; gz = ns[2];
  bool slow = false;
  T s0 = (T)0, s1 = (T)0, s2 = (T)0;
  if (hmax > (T)0) {
    // Fast path: the projection of p on the max-violated face lies inside that
    // triangle => it is the closest point and the distance equals hmax.
    const I4 fr = lf[fs];
    const R a = lv[fr_vert(fr, 0)], b = lv[fr_vert(fr, 1)], c = lv[fr_vert(fr, 2)];
    s0 = edge_value<T>(ns, a, b, px, py, pz);
    s1 = edge_value<T>(ns, b, c, px, py, pz);
    s2 = edge_value<T>(ns, c, a, px, py, pz);
    slow = !(s0 >= (T)0 && s1 >= (T)0 && s2 >= (T)0);
  }
  // hmax is a lower bound of the distance: when it exceeds the lane's best so
  // far by more than the rounding of either value, hull k cannot win (nor tie)
  // and its exact distance is not needed — d stays hmax (> bound).
  const T lb_margin = (T)16 * cert_eps<T>() * (scale + ((fabs(px) + fabs(py)) + fabs(pz)));
#if FSDF_WAVE_TIMES
  wt_count(10, __builtin_popcountll(__ballot(slow && active && (hmax - lb_margin > bound))));
#endif
  slow = slow && active && !(hmax - lb_margin > bound);
  const uint64_t slow_mask = __ballot(slow);
#if FSDF_WAVE_TIMES
  wt_count(8, __builtin_popcountll(slow_mask));
  fsdf_wt_slow[threadIdx.x] = slow;
#endif
  tw = wt_add(2, tw);
  if (!slow_mask) return;
  wt_count(2, 1);
  if (count_events(stats) && (threadIdx.x & 63) == 0) {
    atomicAdd(stats + 2, 1ull);
    atomicAdd(stats + 4, (unsigned long long)__builtin_popcountll(slow_mask));
  }
  // stage A: closest point on triangle f*, certified by the normal cone at
  // its Voronoi feature
  const I4 frs = lf[fs];
  T qx, qy, qz;
  int rA;
  closest_on_triangle<T>(px, py, pz, lv[fr_vert(frs, 0)], lv[fr_vert(frs, 1)], lv[fr_vert(frs, 2)], qx, qy, qz, rA);
  T ex = px - qx, ey = py - qy, ez = pz - qz;
  T best2 = mfma_(ex, ex, mfma_(ey, ey, ez * ez));
  // stage B: descent walk — certify the current point; on failure move to the
  // face(s) the certificate names (each accepted step strictly lowers the
  // distance, so the walk cannot cycle); lanes that stall or exceed the step
  // cap keep `todo` for the exhaustive stage C.
  bool todo = slow;
  int cf = fs, cr = rA;
  bool walking = todo;
  const uint64_t tw_walk = wt_now();
  for (int step = 0; step < kWalkSteps && __any(walking); ++step) {
    if (count_events(stats) && lane_id() == 0) atomicAdd(stats + 21, 1ull);
    wt_count(3, 1);
#if FSDF_WAVE_TIMES
    const uint64_t tw_c = wt_now();
    int fan_it = 0;
    wt_count2(2, __builtin_popcountll(__ballot(walking && cr <= 2)));
    wt_count2(6, __builtin_popcountll(__ballot(walking && cr >= 3 && cr <= 5)));
    wt_count2(7, __builtin_popcountll(__ballot(walking && cr == 6)));
    int* fan_p = &fan_it;
#else
    int* fan_p = nullptr;
#endif
    int n1 = -1, n2 = -1;
    const bool certified = walking && cert_step<T>(px, py, pz, cf, cr, lp, lv, lf, scale, n1, n2, fan_p);
#if FSDF_WAVE_TIMES
    {
      int fm = fan_it;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) fm = max(fm, __shfl_xor(fm, off, 64));
      wt_count2(3, fm);
    }
    const uint64_t tw_s = wt_add2(0, tw_c);
#endif
    if (walking) {
      if (certified) {
        todo = false;
        walking = false;
      } else {
        bool moved = false;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int g = t == 0 ? n1 : n2;
          if (g >= 0) {
            const I4 gr = lf[g];
            T cx, cy, cz;
            int rg;
            closest_on_triangle<T>(px, py, pz, lv[fr_vert(gr, 0)], lv[fr_vert(gr, 1)], lv[fr_vert(gr, 2)], cx, cy, cz,
                                   rg);
            const T dx = px - cx, dy = py - cy, dz = pz - cz;
            const T d2 = mfma_(dx, dx, mfma_(dy, dy, dz * dz));
            if (d2 < best2) { best2 = d2; qx = cx; qy = cy; qz = cz; cf = g; cr = rg; moved = true; }
          }
        }
        walking = moved;
      }
    }
#if FSDF_WAVE_TIMES
    wt_add2(1, tw_s);
#endif
  }
  wt_add(7, tw_walk);  // (the descent walk: certificates and steps)
  if (__any(todo)) {
    if (count_events(stats) && (threadIdx.x & 63) == 0) atomicAdd(stats + 6, 1ull);
    const uint64_t scan_mask = __ballot(todo);
    if (scan_mask) {
      // stage C: exhaustive scan of the visible faces (the closest boundary
      // point of a convex polytope lies on one of them); a face whose plane
      // distance already exceeds the best distance cannot improve it.
      if (count_events(stats) && (threadIdx.x & 63) == 0) atomicAdd(stats + 7, (unsigned long long)__builtin_popcountll(scan_mask));
      // starts from the stage-B point (strict < keeps it on ties): with b2
      // already near the optimum, the plane-distance test h^2 < b2 leaves only
      // the few faces around the closest feature for closest_on_triangle
      T b2 = best2;
      T bx = qx, by = qy, bz = qz;
      // Per chunk of 64 faces: a wave-uniform pass marks, per lane, the faces
      // that pass the test against the stage-B distance (broadcast plane rows,
      // no branches); then each lane walks its own marks in index order,
      // re-testing against its current b2 — the oracle's sequential scan,
      // without running closest_on_triangle for faces no lane needs.
      for (int c0 = 0; c0 < nf; c0 += 64) {
        const int cn = min(64, nf - c0);
        uint64_t mark = 0;
        for (int j = 0; j < cn; ++j) {
          const T h = plane_h<T>(uplane(c0 + j), px, py, pz);
          if (h > (T)0 && h * h < b2) mark |= 1ull << j;
        }
        if (!todo) mark = 0;
        while (mark) {
          const int ff = c0 + __builtin_ctzll(mark);
          mark &= mark - 1;
          const T h = plane_h<T>(lp[ff], px, py, pz);
          if (h * h < b2) {
            const I4 gr = lf[ff];
            T cx, cy, cz;
            int rg;
            closest_on_triangle<T>(px, py, pz, lv[fr_vert(gr, 0)], lv[fr_vert(gr, 1)], lv[fr_vert(gr, 2)], cx, cy,
                                   cz, rg);
            const T dx = px - cx, dy = py - cy, dz = pz - cz;
            const T d2 = mfma_(dx, dx, mfma_(dy, dy, dz * dz));
            if (d2 < b2) { b2 = d2; bx = cx; by = cy; bz = cz; }
          }
        }
      }
      if (todo) { best2 = b2; qx = bx; qy = by; qz = bz; }
    }
  }
  wt_add(3, tw);
  if (slow) {
    if (best2 > (T)0) {
      d = tsqrt(best2);
      const T inv = (T)1 / d;
      gx = (px - qx) * inv; gy = (py - qy) * inv; gz = (pz - qz) * inv;
    } else {
      // p on the boundary (a vertex/edge): d = 0, subgradient = face normal
      d = (T)0;
    }
  }
}

// ---------------------------------------------------------------------------
// RBF interpolating skin (src/Flash.jl:207-213; SpatialFields XCubed + affine):
//   f(x) = Σ w_i |x-c_i|^3 + a + b·x,   s = f/|∇f|,
//   ∇s = ∇f/|∇f| − f (H ∇f)/|∇f|^3      (H = Hessian of f).
// Centre rows are LDS-staged per wave (call with the whole wave active).
// ---------------------------------------------------------------------------
template <typename T>
struct RbfField {
  T f, gx, gy, gz, hxx, hyy, hzz, hxy, hxz, hyz;
};

template <typename T>
__device__ __forceinline__ void rbf_field(T px, T py, T pz, const T* __restrict__ rows, int nc,
                                          T* __restrict__ lw, int cap, RbfField<T>& F) {
  typedef typename Row4<T>::type R4;
  const R4 poly = *(const R4*)(rows + 4 * nc);
  F.f = mfma_(poly[1], px, mfma_(poly[2], py, mfma_(poly[3], pz, poly[0])));
  F.gx = poly[1]; F.gy = poly[2]; F.gz = poly[3];
  F.hxx = F.hyy = F.hzz = F.hxy = F.hxz = F.hyz = (T)0;
  for (int c0 = 0; c0 < nc; c0 += cap) {
    const int cn = min(cap, nc - c0);
    stage_rows(lw, rows + 4 * c0, cn);
    for (int i = 0; i < cn; ++i) {
      const R4 c = *(const R4*)(lw + 4 * i);
      const T dx = px - c[0], dy = py - c[1], dz = pz - c[2];
      const T r2 = mfma_(dx, dx, mfma_(dy, dy, dz * dz));
      const T r = tsqrt(r2);
      const T wr = c[3] * r;
      F.f = mfma_(wr, r2, F.f);
      const T t3 = (T)3 * wr;
      F.gx = mfma_(t3, dx, F.gx); F.gy = mfma_(t3, dy, F.gy); F.gz = mfma_(t3, dz, F.gz);
      const T hq = r2 > (T)0 ? ((T)3 * c[3]) / r : (T)0;
      F.hxx = mfma_(hq * dx, dx, F.hxx + t3);
      F.hyy = mfma_(hq * dy, dy, F.hyy + t3);
      F.hzz = mfma_(hq * dz, dz, F.hzz + t3);
      F.hxy = mfma_(hq * dx, dy, F.hxy);
      F.hxz = mfma_(hq * dx, dz, F.hxz);
      F.hyz = mfma_(hq * dy, dz, F.hyz);
    }
  }
}

// s and ∇s from the field; also returns c = f/|∇f|^3 and 1/|∇f| for the adjoint.
template <typename T>
__device__ __forceinline__ void rbf_skin_from_field(const RbfField<T>& F, T& s, T& gx, T& gy, T& gz, T& c,
                                                    T& invG) {
  const T G2 = mfma_(F.gx, F.gx, mfma_(F.gy, F.gy, F.gz * F.gz));
  const T G = tsqrt(G2);
  s = F.f / G;
  invG = (T)1 / G;
  c = F.f / (G2 * G);
  const T hgx = mfma_(F.hxx, F.gx, mfma_(F.hxy, F.gy, F.hxz * F.gz));
  const T hgy = mfma_(F.hxy, F.gx, mfma_(F.hyy, F.gy, F.hyz * F.gz));
  const T hgz = mfma_(F.hxz, F.gx, mfma_(F.hyz, F.gy, F.hzz * F.gz));
  gx = mfma_(-c, hgx, F.gx * invG);
  gy = mfma_(-c, hgy, F.gy * invG);
  gz = mfma_(-c, hgz, F.gz * invG);
}

// Wave-wide f64 sum in the VALU (DPP, no LDS round trips): inclusive scan
// within each 16-lane row (row_shr 1, 2, 4, 8), then row_bcast 15 / 31 carry
// the row totals; lane 63 holds the sum, returned to every lane. Fixed order
// (deterministic). Whole wave active.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_shifted(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xf, true);
  return __hiloint2double(hi, lo);
}
// Wave-wide f32 min / max in the VALU (DPP scan, identity fill), result to
// every lane. Whole wave active.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_shifted_f(float v, float identity) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(identity), __float_as_int(v), CTRL, ROW_MASK,
                                                    0xf, false));
}
template <bool MAX>
__device__ __forceinline__ float wave_minmax(float v) {
  const float id = MAX ? -__builtin_huge_valf() : __builtin_huge_valf();
  auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : fminf(a, b); };
  v = op(v, dpp_shifted_f<0x111, 0xf>(v, id));
  v = op(v, dpp_shifted_f<0x112, 0xf>(v, id));
  v = op(v, dpp_shifted_f<0x114, 0xf>(v, id));
  v = op(v, dpp_shifted_f<0x118, 0xf>(v, id));
  v = op(v, dpp_shifted_f<0x142, 0xa>(v, id));
  v = op(v, dpp_shifted_f<0x143, 0xc>(v, id));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Bounding sphere (bbox centre, half diagonal) of the wave's valid lanes'
// points (invalid lanes stand in for the first valid one). Whole wave active.
__device__ __forceinline__ WaveSphere wave_sphere(float pxf, float pyf, float pzf, bool valid) {
  const uint64_t vm = __ballot(valid);
  const int src = vm ? __builtin_ctzll(vm) : 0;
  float qx = pxf, qy = pyf, qz = pzf;
  if (!valid) { qx = __shfl(pxf, src, 64); qy = __shfl(pyf, src, 64); qz = __shfl(pzf, src, 64); }
  const float lx = wave_minmax<false>(qx), ly = wave_minmax<false>(qy), lz = wave_minmax<false>(qz);
  const float hx = wave_minmax<true>(qx), hy = wave_minmax<true>(qy), hz = wave_minmax<true>(qz);
  const float ex = hx - lx, ey = hy - ly, ez = hz - lz;
  WaveSphere ws;
  ws.x = 0.5f * (lx + hx); ws.y = 0.5f * (ly + hy); ws.z = 0.5f * (lz + hz);
  ws.r = 0.5f * __builtin_sqrtf(__builtin_fmaf(ex, ex, __builtin_fmaf(ey, ey, ez * ez)));
  return ws;
}

// Per-chunk bounding spheres of a resident cloud (one wave per 64 points),
// read by the pass kernel instead of recomputing them every pass. `nchunks`
// may exceed ceil(n/64) (padding to whole pass workgroups): a chunk past the
// cloud's end gets the zero-radius sphere of the last point, so a
// hull-partitioned workgroup's empty second chunk reads a defined row.
template <typename T>
__global__ __launch_bounds__(kBlock) void chunk_sphere_kernel(const T* __restrict__ pts, int64_t n, int64_t nchunks,
                                                              F4* __restrict__ out) {
  const int64_t base = ((int64_t)blockIdx.x * kBlock + threadIdx.x) & ~(int64_t)63;
  if (base >= 64 * nchunks) return;  // wave-uniform
  const int64_t i = base + (threadIdx.x & 63);
  const bool valid = i < n;
  const int64_t ii = valid ? i : n - 1;
  const WaveSphere ws = wave_sphere((float)pts[3 * ii], (float)pts[3 * ii + 1], (float)pts[3 * ii + 2], valid);
  if ((threadIdx.x & 63) == 0) out[base >> 6] = F4{ws.x, ws.y, ws.z, ws.r};
}

__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_shifted<0x111, 0xf>(v);  // row_shr:1
  v += dpp_shifted<0x112, 0xf>(v);  // row_shr:2
  v += dpp_shifted<0x114, 0xf>(v);  // row_shr:4
  v += dpp_shifted<0x118, 0xf>(v);  // row_shr:8
  v += dpp_shifted<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_shifted<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63),
                          __builtin_amdgcn_readlane(__double2loint(v), 63));
}

// Adjoint contributions of the lanes whose nearest surface is RBF skin r
// (sel): per centre λ_w_i = Σ 2s ∂s/∂w_i and E_i = Σ 2s ∂s/∂c_i (coefficients
// fixed), then λ_a, λ_b — wave-summed, added by lane 0 into acc (LDS):
//   acc[0..n) = λ_w, acc[n] = λ_a, acc[n+1..n+4) = λ_b, acc[n+4+3i..] = E_i.
template <typename T>
__device__ __forceinline__ void rbf_adjoint(T px, T py, T pz, const T* __restrict__ rows, int nc,
                                            T* __restrict__ lw, int cap, bool sel, double* __restrict__ acc) {
  typedef typename Row4<T>::type R4;
  RbfField<T> F;
  rbf_field(px, py, pz, rows, nc, lw, cap, F);
  T s, sgx, sgy, sgz, c, invG;
  rbf_skin_from_field(F, s, sgx, sgy, sgz, c, invG);
  const T two_s = (T)2 * s;
  const T dsdf = invG;
  const T ux = -c * F.gx, uy = -c * F.gy, uz = -c * F.gz;  // ∂s/∂∇f
  const int lane = threadIdx.x & 63;
  for (int c0 = 0; c0 < nc; c0 += cap) {
    const int cn = min(cap, nc - c0);
    stage_rows(lw, rows + 4 * c0, cn);
    for (int i = 0; i < cn; ++i) {
      const R4 cw = *(const R4*)(lw + 4 * i);
      const T dx = px - cw[0], dy = py - cw[1], dz = pz - cw[2];
      const T r2 = mfma_(dx, dx, mfma_(dy, dy, dz * dz));
      const T r = tsqrt(r2);
      const T e = mfma_(dx, ux, mfma_(dy, uy, dz * uz));
      const T lam = two_s * mfma_(dsdf * r2, r, (T)3 * r * e);
      const T k1 = mfma_((T)3 * r, dsdf, r2 > (T)0 ? ((T)3 * e) / r : (T)0);
      const T k2 = (T)3 * r;
      const T sc = -two_s * cw[3];
      double v[4] = {(double)lam, (double)(sc * mfma_(k1, dx, k2 * ux)), (double)(sc * mfma_(k1, dy, k2 * uy)),
                     (double)(sc * mfma_(k1, dz, k2 * uz))};
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = wave_sum(sel ? v[j] : 0.0);
      if (lane == 0) {
        acc[c0 + i] += v[0];
        double* E = acc + nc + 4 + 3 * (c0 + i);
        E[0] += v[1]; E[1] += v[2]; E[2] += v[3];
      }
    }
  }
  double w[4] = {(double)(two_s * dsdf), (double)(two_s * mfma_(dsdf, px, ux)),
                 (double)(two_s * mfma_(dsdf, py, uy)), (double)(two_s * mfma_(dsdf, pz, uz))};
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = wave_sum(sel ? w[j] : 0.0);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[nc + j] += w[j];
  }
}

// ---------------------------------------------------------------------------
// Scene signed distance of this lane's point: minimum over all surfaces with
// the first-index tie rule (src/Flash.jl:265-268), its surface index and
// gradient. Wave-cooperative (ballots, LDS staging): call with the whole wave
// active; `valid` marks lanes whose result is used.
// ---------------------------------------------------------------------------
template <typename T, int SLOTS, bool CULL, bool RBF, bool P64 = false, int NSHARE = 1>
__device__ __forceinline__ void scene_eval(T px, T py, T pz, bool valid, const PassModel<T>& m,
                                           const HullRow* __restrict__ ht, float smax, T* __restrict__ lw,
                                           unsigned long long* __restrict__ stats, T& best, int& bk, T& gx, T& gy,
                                           T& gz, const F4* __restrict__ cws = nullptr, uint64_t partmask = ~0ull,
                                           double* shbest = nullptr, int prior = -1) {
  // partmask (hull-partitioned pass, pass_kernel HPART): this wave evaluates
  // only the hulls whose bit (k & 63) is set; culling and the upper bound
  // still use every hull
  const int K = m.K;
  const int lane = threadIdx.x & 63;
  // Phase A (fp32, exact-safe): with c_k inside hull k and r_k its bounding
  // radius, d_k(p) >= |p-c_k| - r_k and d_k(p) >= the oriented-box bound
  // (lower bounds), d_k(p) <= |p-c_k| (upper bound). ub = min_k |p-c_k|; the
  // best-first seed is the hull of least lower bound (a heuristic: any seed
  // is exact).
  float ub2 = __builtin_huge_valf(), lb_min = __builtin_huge_valf();
  int kseed = 0;
  float pxf = 0.f, pyf = 0.f, pzf = 0.f;
  // candidate hulls of the wave (bit k&63 of cand[k>>6]); all hulls without culling
  uint64_t cand[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int left = K - 64 * s;
    cand[s] = left >= 64 ? ~0ull : (left > 0 ? (1ull << left) - 1 : 0ull);
  }
  uint64_t tw = wt_now();
  // the wave's bounding sphere (bbox centre, half diagonal) over the valid
  // lanes: precomputed per resident chunk at set_points (pose-independent,
  // the same arithmetic) or computed here
  pxf = (float)px; pyf = (float)py; pzf = (float)pz;
  WaveSphere ws;
  if (cws) {
    const F4 v = *cws;
    ws = WaveSphere{v[0], v[1], v[2], v[3]};
  } else {
    ws = wave_sphere(pxf, pyf, pzf, valid);
  }
  if (CULL) {
    // Wave-level culling, one hull per lane: with the wave's points inside the
    // sphere (c_w, r_w) and D_k = |c_w - c_k|, every point of the wave has
    // d_k >= D_k - r_w - r_k and d_k <= D_k + r_w, so a hull whose lower bound
    // exceeds UB_w = min_k (D_k + r_w) by the fp32 margin is needed by no lane.
    const float cwx = ws.x, cwy = ws.y, cwz = ws.z, rw = ws.r;
    float Dk[SLOTS];
    float ubw = __builtin_huge_valf();
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const int k = 64 * s + lane;
      Dk[s] = __builtin_huge_valf();
      if (k < K) {
        const F4 sp = ht[k].sphere;
        const float dx = cwx - sp[0], dy = cwy - sp[1], dz = cwz - sp[2];
        Dk[s] = __builtin_sqrtf(__builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz)));
        ubw = fminf(ubw, Dk[s] + rw);
      }
    }
    ubw = wave_minmax<false>(ubw);
    const float mrgw = 1e-5f * (1.0f + fabsf(cwx) + fabsf(cwy) + fabsf(cwz) + smax + 4.0f * rw + 2.0f * ubw);
    // ... and so does one whose box bound at c_w (1-Lipschitz) minus r_w does
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const int k = 64 * s + lane;
      const HullRow& h = ht[k < K ? k : 0];
      const bool c = (k < K) & (Dk[s] - rw - h.sphere[3] <= ubw + mrgw) & box_within(h, cwx, cwy, cwz, ubw + mrgw + rw);
      cand[s] = __ballot(c);
    }
    if (count_events(stats) && lane == 0) {
      unsigned long long nc = 0;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) nc += __builtin_popcountll(cand[s]);
      atomicAdd(stats + 8, nc);
    }
    // per lane over the candidates: ub = min_k |p-c_k| and the best-first seed
    // (hull-partitioned pass: over this wave's part only — its ub is still an
    // upper bound of d*, and the chunk's waves share their bests anyway)
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      uint64_t cm = cand[s] & partmask;
      while (cm) {
        const int k = 64 * s + __builtin_ctzll(cm);
        cm &= cm - 1;
        const F4 sp = ht[k].sphere;
        const float dx = pxf - sp[0], dy = pyf - sp[1], dz = pzf - sp[2];
        const float dist2 = __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz));
        ub2 = fminf(ub2, dist2);
        // seed: the least lower bound — sphere, and on scenes of few hulls also
        // box (a heuristic only: every candidate is still searched, so either
        // seed gives the same bits; kSeedBoxMaxHulls)
        float lb = __builtin_sqrtf(dist2) - sp[3];
        if (K < kSeedBoxMaxHulls) lb = fmaxf(lb, box_lower(ht[k], pxf, pyf, pzf));
        if (lb < lb_min) { lb_min = lb; kseed = k; }
      }
    }
  }
  // the point's nearest surface in the previous pass over this cloud, when
  // known (PassOutputs::prior_in), is its seed instead: tracking passes move
  // the model little, so it is usually this pass's nearest too, and `best` is
  // tight after the first evaluation (any seed gives the same bits)
  const bool prior_ok = CULL && !RBF && SLOTS == 1 && prior >= 0 && prior < K && ((partmask >> (prior & 63)) & 1);
  if (prior_ok) kseed = prior;
  const float ub = __builtin_sqrtf(ub2);
  tw = wt_add(4, tw);
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) wt_count(6, __builtin_popcountll(cand[s]));
  // one rounding margin per lane, >= 1e-5 x every magnitude in the test below
  const float mrg = 1e-5f * (1.0f + fabsf(pxf) + fabsf(pyf) + fabsf(pzf) + smax + 2.0f * ub);

  best = tinf<T>();
  bk = 0x7fffffff;
  gx = (T)0; gy = (T)0; gz = (T)0;
  if (RBF) {
    // RBF skins first: always needed (no cheap bound), and they tighten `best`
    for (int r = 0; r < m.R; ++r) {
      const int ks = m.rbf_surface[r];
      const int r0 = m.rbf_row_off[r];
      const int nc = m.rbf_row_off[r + 1] - r0 - 1;
      RbfField<T> F;
      rbf_field(px, py, pz, m.rbf_rows + 4 * r0, nc, lw, m.stage_bytes / (4 * (int)sizeof(T)), F);
      T sv, hx, hy, hz, c_, iG;
      rbf_skin_from_field(F, sv, hx, hy, hz, c_, iG);
      if (valid && (sv < best || (sv == best && ks < bk))) { best = sv; bk = ks; gx = hx; gy = hy; gz = hz; }
    }
    wt_add(5, tw);
  }
  // hull k is needed by a lane unless its lower bound exceeds min(ub, best)
  // by more than the fp32 rounding margin
  // hull k is needed by a lane unless |p-c_k| - r_k > min(ub, best) + mrg,
  // tested without a sqrt: |p-c_k|^2 <= (min(ub, best) + mrg + r_k)^2
  // (HPART) the least best distance the chunk's waves have found so far, per
  // lane, one LDS slot kept by ds_min_f64: an upper bound of d* — as exact-safe
  // a pruning bound as this wave's own best (a stale read only bounds less).
  // (One slot read per test: 2.6 % faster at 2^17 than a slot per wave, a
  // cached copy refreshed per evaluation no faster; profiles/r03/experiments)
  // (NSHARE == 0: shared iff shbest is given — the planned pass decides per
  // workgroup at run time)
  auto bound_now = [&]() -> T {
    T b = best;
    if constexpr (NSHARE > 1) {
      const T o = (T)((const volatile double*)shbest)[lane];
      b = o < b ? o : b;
    } else if constexpr (NSHARE == 0) {
      if (shbest) {
        const T o = (T)((const volatile double*)shbest)[lane];
        b = o < b ? o : b;
      }
    }
    return b;
  };
  auto needs = [&](int k) -> bool {
    if (!CULL) return valid;
    const T b = bound_now();
    return valid & needs_at(ht[k], pxf, pyf, pzf, fminf(ub, (float)b) + mrg);
  };
  // evaluations may run out of index order: ties keep the smaller k
#if FSDF_WAVE_TIMES
  uint64_t wt_slowk = 0;  // hulls whose evaluation ran this lane's search
#endif
  auto evaluate = [&](int k, bool need) {
    wt_count(0, 1);
    wt_count(5, __builtin_popcountll(__ballot(need)));
    T dk, hx, hy, hz;
    hull_sdf<T, P64>(px, py, pz, k, m, ht, need, bound_now(), dk, hx, hy, hz, lw, stats);
#if FSDF_WAVE_TIMES
    if (fsdf_wt_slow[threadIdx.x]) wt_slowk |= 1ull << (k & 63);
#endif
    if (count_events(stats)) {
      const uint64_t nm = __ballot(need);
      if (lane == 0) {
        atomicAdd(stats + 1, 1ull);
        atomicAdd(stats + 3, (unsigned long long)__builtin_popcountll(nm));
      }
    }
    const int ks = RBF ? m.hull_surface[k] : k;
    if (need && (dk < best || (dk == best && ks < bk))) { best = dk; bk = ks; gx = hx; gy = hy; gz = hz; }
    if constexpr (NSHARE > 1)  // (one slot per lane: the minimum over the chunk's waves, ds_min_f64)
      __hip_atomic_fetch_min(shbest + lane, (double)best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if constexpr (NSHARE == 0)
      if (shbest) __hip_atomic_fetch_min(shbest + lane, (double)best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  uint64_t done[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) done[s] = 0;
#if FSDF_WAVE_TIMES
  auto wt_won = [&]() { wt_count(9, __builtin_popcountll(__ballot(valid && ((wt_slowk >> (bk & 63)) & 1)))); };
#endif
  // ONE evaluation site (hull_sdf is large: two inlined copies doubled the
  // kernel's code to ~40 KB): first each lane's seed hull (Phase B, one
  // evaluation per distinct seed in the wave, so that `best` is tight), then
  // the remaining candidates in index order (Phase C).
  uint64_t pend = (CULL && K > 0) ? __ballot(valid && (lb_min < __builtin_huge_valf() || prior_ok)) : 0ull;
  int slot = -1;      // Phase C slot; -1 while seeds are pending
  uint64_t cm = 0ull;  // Phase C candidates left in `slot`
  for (;;) {
    int k;
    bool need;
    if (pend) {
      k = __builtin_amdgcn_readfirstlane(__shfl(kseed, __builtin_ctzll(pend), 64));
      pend &= ~__ballot(valid && kseed == k);
#pragma unroll
      for (int s = 0; s < SLOTS; ++s)
        if ((k >> 6) == s) done[s] |= 1ull << (k & 63);
      need = needs(k);
      if (count_events(stats) && lane == 0) atomicAdd(stats + 5, 1ull);
      wt_count(4, 1);
      // a seed the earlier seeds' results have ruled out for every lane (its
      // bit is in `done`; bounds only tighten, so Phase C would skip it too):
      // no staging, no screen (2^17: 0.0464 -> 0.0454 ms pass)
      if (!__any(need)) continue;
    } else {
      while (!cm && slot < SLOTS - 1) {
        ++slot;
#pragma unroll
        for (int s = 0; s < SLOTS; ++s)
          if (s == slot) cm = cand[s] & ~done[s] & partmask;
      }
      if (!cm) break;
      k = 64 * slot + __builtin_ctzll(cm);
      cm &= cm - 1;
#if FSDF_WAVE_TIMES
      const uint64_t tw_need = wt_now();
      need = needs(k);
      const bool any_need = __any(need);
      wt_count(11, wt_now() - tw_need);
      if (!any_need) continue;
#else
      need = needs(k);
      if (!__any(need)) continue;
#endif
    }
    evaluate(k, need);
  }
#if FSDF_WAVE_TIMES
  wt_won();
#endif
  if (count_events(stats) && lane == 0) atomicAdd(stats + 0, 1ull);
}

// Per-chunk epilogue (pass and merge kernels): this wave's contributions
//   c += d^2;  F_k += 2 d g;  M_k += 2 d (p x g)   (RBF skins: adjoint sums)
// segmented by k* (ballot loop + DPP wave sums) into the LDS rows owned by
// lane k, then the per-point outputs. Whole wave active.
template <typename T, int SLOTS, bool RBF>
__device__ __forceinline__ uint64_t emit_chunk(T px, T py, T pz, bool valid, T best, int bk, T gx, T gy, T gz, int64_t i,
                                           int64_t base, int64_t n, const PassModel<T>& m, const PassOutputs& out,
                                           double* __restrict__ acc_row, double& cost_acc,
                                           double* __restrict__ rbf_wave, T* __restrict__ stage, int stage_cap) {
  const int lane = threadIdx.x & 63;
  // contributions: c += d^2; F_k += 2 d g; M_k += 2 d (p x g)
  double cF[3] = {0.0, 0.0, 0.0}, cM[3] = {0.0, 0.0, 0.0};
  if (valid) {
    const double bd = (double)best;
    const double dgx = gx, dgy = gy, dgz = gz;
    const double dpx = px, dpy = py, dpz = pz;
    cost_acc = __builtin_fma(bd, bd, cost_acc);
    const double w = 2.0 * bd;
    cF[0] = w * dgx; cF[1] = w * dgy; cF[2] = w * dgz;
    cM[0] = w * __builtin_fma(dpy, dgz, -(dpz * dgy));
    cM[1] = w * __builtin_fma(dpz, dgx, -(dpx * dgz));
    cM[2] = w * __builtin_fma(dpx, dgy, -(dpy * dgx));
  }
  const uint64_t tw = wt_now();
  uint64_t pending = __ballot(valid);
  uint64_t touched = 0;  // surfaces (k & 63) of this chunk's points
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const int kk = __builtin_amdgcn_readfirstlane(__shfl(bk, leader, 64));
    const bool sel = valid && (bk == kk);
    pending &= ~__ballot(sel);
    touched |= 1ull << (kk & 63);
    if (RBF && m.surface_kind[kk] != 0) {
      // RBF skin: adjoint sums instead of a rigid wrench
      int r = 0;
      while (m.rbf_surface[r] != kk) ++r;
      const int r0 = m.rbf_row_off[r];
      rbf_adjoint(px, py, pz, m.rbf_rows + 4 * r0, m.rbf_row_off[r + 1] - r0 - 1, stage, stage_cap, sel,
                  rbf_wave + m.rbf_acc_off[r]);
      continue;
    }
    double v[6];
#pragma unroll
    for (int j = 0; j < 3; ++j) { v[j] = sel ? cF[j] : 0.0; v[3 + j] = sel ? cM[j] : 0.0; }
#pragma unroll
    for (int j = 0; j < 6; ++j) v[j] = wave_sum(v[j]);
    if (lane == (kk & 63)) {
      double* r = acc_row + (kk >> 6) * 64 * 6;
#pragma unroll
      for (int j = 0; j < 6; ++j) r[j] += v[j];
    }
  }

  {
    // the next pass's seed hint (resident order), stored only where it changed
    // (re-read here rather than carried from the seed load: a register live
    // through scene_eval spills at the budget)
    if (out.prior_out && valid && out.prior_out[i] != (uint8_t)bk) out.prior_out[i] = (uint8_t)bk;
    if (out.perm) {  // caller order: scattered through the sort permutation
      if (valid) {
        const int64_t o = out.perm[i];
        if (out.kstar) out.kstar[o] = bk;
        if (out.d) out.d[o] = (double)best;
        if (out.grad) {
          out.grad[3 * o + 0] = (double)gx;
          out.grad[3 * o + 1] = (double)gy;
          out.grad[3 * o + 2] = (double)gz;
        }
      }
    } else {  // resident order: coalesced
      if (valid) {
        if (out.kstar) out.kstar[i] = bk;
        if (out.d) out.d[i] = (double)best;
      }
      if (out.grad) {
        // the wave's [64][3] gradient block is contiguous: transpose it
        // through this wave's (now free) stage and store whole 16-B chunks —
        // three strided 8-B stores per lane would each write a third of
        // every 64-B granule (3x the bytes at the memory side)
        double* sg = (double*)stage;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        sg[3 * lane + 0] = (double)gx;
        sg[3 * lane + 1] = (double)gy;
        sg[3 * lane + 2] = (double)gz;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int nvalid = (int)(n - base < 64 ? n - base : 64);
        typedef double D2 __attribute__((ext_vector_type(2)));
        D2* dst = (D2*)(out.grad + 3 * base);  // 16-B aligned: base is a multiple of 64
        const D2* src = (const D2*)sg;
        for (int c = lane; 2 * c < 3 * nvalid; c += 64) {
          if (2 * c + 1 < 3 * nvalid) dst[c] = src[c];
          else out.grad[3 * base + 2 * c] = sg[2 * c];  // odd tail (3 * nvalid odd)
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // stage reads before the next overwrite
      }
    }
  }
  wt_add(6, tw);
  return touched;
}

// Per-block partial sums in line tiles: entry t of logical block b at
// partials[t / 8][b][t % 8] — a block writes whole 64-B lines and
// reduce_tiles_kernel reads whole lines (entry-major columns
// wrote one 8-B entry per line, block-major rows made the reduce stride).
__device__ __forceinline__ int64_t pidx(int t, int b, int nblocks) {
  return ((int64_t)(t >> 3) * nblocks + b) * 8 + (t & 7);
}

// ---------------------------------------------------------------------------
// Residual pass.
// ---------------------------------------------------------------------------
extern __shared__ __attribute__((aligned(16))) char fsdf_lds[];

// ALIAS (one chunk per wave: n <= grid * 256; hull-only, <= 64 surfaces; f64
// models with LocalModel::planes64): the wave's wrench rows live in its own
// hull stage, which is free once the chunk's scene evaluation is done — 12 KiB
// less LDS per workgroup, spent on staging the fp64 planes with the hull
// (hull_sdf P64) at the same occupancy.
//
// HPART (hull-partitioned, with ALIAS; small clouds, hpart_pass): kHpart
// waves share one 64-point chunk and split its hull evaluations by hull index
// (part j of the chunk evaluates hulls k with k % kHpart == j; culling and the
// upper bound use every hull, each wave prunes with its own best). Any upper
// bound of d* is exact-safe, so each wave's result is the exact first-index
// minimum over its hulls, and the lexicographic (d, k) minimum over the
// chunk's waves is the full scene's — bit for bit. The heaviest chunks'
// serial evaluations are spread over kHpart waves where a one-wave-per-chunk
// grid would leave most wave slots idle.
template <typename T, int SLOTS, bool CULL, bool RBF, bool ALIAS = false, bool HPART = false, int NB = kPassBlock,
          int NPART = kHpart>
// (occupancy target in waves per SIMD, whatever the workgroup size NB; NPART:
// waves per chunk of the hull-partitioned pass, 4 or 2 — hpart_parts)
__global__ __launch_bounds__(NB) __attribute__((
    amdgpu_waves_per_eu((SLOTS == 1 ? kPassWavesPerSimd : (SLOTS == 2 ? 3 : 2)) - (RBF ? 1 : 0)))) void pass_kernel(
    const T* __restrict__ pts, int64_t n, PassModel<T> m, PassOutputs out) {
  if (out.skip && *out.skip) return;  // (uniform: a converged device solver loop)
  static_assert(!ALIAS || (SLOTS == 1 && !RBF), "aliased wrench rows: hull-only, <= 64 surfaces");
  static_assert(!HPART || ALIAS, "the hull-partitioned pass is an aliased pass");
  constexpr int kParts = HPART ? NPART : 1;
  constexpr int kChunkStride = NB / kParts;  // points per logical block
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // (wave-uniform: readfirstlane keeps the hull mask and the loops scalar)
  const int part = HPART ? __builtin_amdgcn_readfirstlane(wave % kParts) : 0;  // (HPART) this wave's hull residue
  const int cw = HPART ? __builtin_amdgcn_readfirstlane(wave / kParts) : wave;  // the block's chunk this wave works on
  // All LDS is one dynamic region (16-byte aligned carve, see pass_lds_bytes):
  //   red     [4 waves][kRedStride] f64  per-hull wrench sums + cost (not ALIAS)
  //   rbf_acc [4 waves][kMaxRbfAcc] f64  (RBF variants only)
  //   stage   [4 waves][m.stage_bytes]   hull / RBF row stage (ALIAS: after the
  //                                      evaluation, the wave's red rows, then
  //                                      the gradient transpose)
  // per-hull wrench sums: row (s*64 + lane) of this wave's slab is owned by
  // lane `lane` (hull s*64 + lane)
  constexpr int kRedStride = SLOTS * 64 * 6 + 2;
  double* red = (double*)fsdf_lds;
  HullRow* ht = (HullRow*)(fsdf_lds + (ALIAS ? 0 : ((NB / 64) * kRedStride + (RBF ? (NB / 64) * kMaxRbfAcc : 0)) * 8));
  T* stage = (T*)((char*)(ht + m.K + 1) + wave * m.stage_bytes);
  auto red_of = [&](int w) -> double* {
    return ALIAS ? (double*)((char*)(ht + m.K + 1) + w * m.stage_bytes) : red + w * kRedStride;
  };
  double* acc_row = red_of(wave) + lane * 6;
  auto zero_rows = [&]() {
#pragma unroll
    for (int s = 0; s < SLOTS; ++s)
#pragma unroll
      for (int j = 0; j < 6; ++j) acc_row[s * 64 * 6 + j] = 0.0;
  };
  if (!ALIAS) zero_rows();
  double cost_acc = 0.0;
  // RBF adjoint sums of this wave (lane 0 adds)
  double* rbf_acc = red + (NB / 64) * kRedStride;
  double* rbf_wave = rbf_acc + wave * kMaxRbfAcc;
  const int stage_cap = m.stage_bytes / (4 * (int)sizeof(T));
  if (RBF)
    for (int e = lane; e < m.rbf_acc_off[m.R]; e += 64) rbf_wave[e] = 0.0;
  // logical block of this launch slot (cost-ordered schedule, see PassOutputs)
  const int lb = out.order ? __builtin_amdgcn_readfirstlane(out.order[blockIdx.x]) : (int)blockIdx.x;
  // (ALIAS: a wave past the cloud's end never evaluates; its rows are zeroed now)
  if (ALIAS && (int64_t)lb * kChunkStride + cw * 64 >= n) {
    zero_rows();
    if (lane == 0) red_of(wave)[SLOTS * 64 * 6] = 0.0;
  }
  const uint64_t t_block = out.cost ? __builtin_amdgcn_s_memrealtime() : 0;
#if FSDF_WAVE_TIMES
  const uint64_t t_block0 = __builtin_amdgcn_s_memrealtime();
#endif
  const float smax = load_hull_table(m, ht);
  const int64_t stride = (int64_t)gridDim.x * kChunkStride;
  // (HPART: exactly one iteration for every wave, also for a chunk past the
  // cloud's end — its lanes are all invalid — because the combine below holds
  // workgroup barriers)
  const int64_t base0 = (int64_t)lb * kChunkStride + cw * 64;
  for (int64_t base = base0; HPART ? base == base0 : base < n; base += stride) {
    const int64_t i = base + lane;
    const bool valid = i < n;
    const int64_t ii = valid ? i : n - 1;
    const T px = pts[3 * ii + 0], py = pts[3 * ii + 1], pz = pts[3 * ii + 2];
#if FSDF_WAVE_TIMES
    const uint64_t w_t0 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0)
      fsdf_wave_ev[wave][0] = fsdf_wave_ev[wave][1] = fsdf_wave_ev[wave][2] = fsdf_wave_ph[wave][0] =
          fsdf_wave_ph[wave][1] = fsdf_wave_ph2[wave][0] = fsdf_wave_ph2[wave][1] = 0;
#endif

    T best, gx, gy, gz;
    int bk;
    const F4* cws = out.chunk_ws ? (const F4*)out.chunk_ws + (base >> 6) : nullptr;
    double* shb = nullptr;
    if constexpr (HPART) {  // the chunk's shared per-lane bests, after the stages
      shb = (double*)((char*)(ht + m.K + 1) + (NB / 64) * m.stage_bytes) + 64 * cw;
      if (part == 0) ((volatile double*)shb)[lane] = __builtin_huge_val();
      __syncthreads();
    }
    // (not in the hull-partitioned tiers: bound by their heaviest chunk's
    // latency, the prior's load in front of it cost 2^16 0.0501 -> 0.0532 ms)
    const int prior = (!HPART && out.prior_in && valid) ? (int)out.prior_in[i] : -1;
    scene_eval<T, SLOTS, CULL, RBF, ALIAS, kParts>(px, py, pz, valid, m, ht, smax, stage, out.stats, best, bk, gx, gy,
                                                   gz, cws,
                                                   HPART ? ((kParts == 8 ? 0x0101010101010101ull
                                                                         : (kParts == 4 ? 0x1111111111111111ull
                                                                                        : 0x5555555555555555ull))
                                                            << part)
                                                         : ~0ull,
                                                   shb, prior);
    if constexpr (HPART) {
      // the chunk's waves' results meet in their stages; part 0 keeps the
      // lexicographic (d, k) minimum per point
      T* rs = stage;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      rs[4 * lane + 0] = best; rs[4 * lane + 1] = gx; rs[4 * lane + 2] = gy; rs[4 * lane + 3] = gz;
      ((int*)(rs + 256))[lane] = bk;
      __syncthreads();
      if (part == 0) {
#pragma unroll
        for (int w = 1; w < kParts; ++w) {
          const T* ro = (const T*)((char*)(ht + m.K + 1) + (wave + w) * m.stage_bytes);
          const T d2 = ro[4 * lane];
          const int k2 = ((const int*)(ro + 256))[lane];
          if (d2 < best || (d2 == best && k2 < bk)) {
            best = d2; bk = k2; gx = ro[4 * lane + 1]; gy = ro[4 * lane + 2]; gz = ro[4 * lane + 3];
          }
        }
      }
      __syncthreads();
    }
    if (!valid) bk = 0;

    if (ALIAS) {  // the stage is free: this wave's rows go there (once: one chunk per wave)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      zero_rows();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    T* tstage = ALIAS ? (T*)((char*)stage + kRedStride * 8) : stage;  // gradient transpose after the rows
    // (ALIAS: the wave's one chunk; its cost is summed and parked in the
    // wave's row now — a per-lane accumulator live through the whole kernel
    // was spilled to scratch at the register budget)
    double cost_chunk = 0.0;
    if (!HPART || part == 0)  // (HPART: part 0 emits the chunk; the other waves' rows stay zero)
      emit_chunk<T, SLOTS, RBF>(px, py, pz, valid, best, bk, gx, gy, gz, i, base, n, m, out, acc_row,
                                ALIAS ? cost_chunk : cost_acc, rbf_wave, tstage, stage_cap);
    if (ALIAS) {
      cost_chunk = wave_sum(cost_chunk);
      if (lane == 0) red_of(wave)[SLOTS * 64 * 6] = cost_chunk;
    }
#if FSDF_WAVE_TIMES
    // diagnostic: 100 MHz wall clock around each wave-iteration of the first
    // grid pass (stats + 32 + 2 * wave), written by lane 0
    if (out.stats && lane == 0 && (!HPART || part == 0) && base < (int64_t)64 * 4 * kMaxBlocks) {
      const int64_t wv = base / 64;
      out.stats[32 + 2 * wv] = w_t0;
      out.stats[33 + 2 * wv] = __builtin_amdgcn_s_memrealtime();
      out.stats[32 + 8 * kMaxBlocks + 2 * wv] = fsdf_wave_ev[wave][0];
      out.stats[33 + 8 * kMaxBlocks + 2 * wv] = fsdf_wave_ev[wave][1];
      out.stats[32 + 18 * kMaxBlocks + 2 * wv] = fsdf_wave_ph[wave][0];
      out.stats[33 + 18 * kMaxBlocks + 2 * wv] = fsdf_wave_ph[wave][1];
      out.stats[32 + 26 * kMaxBlocks + wv] = fsdf_wave_ev[wave][2];
      if (wv < kMaxBlocks) {
        out.stats[32 + 30 * kMaxBlocks + 2 * wv] = fsdf_wave_ph2[wave][0];
        out.stats[33 + 30 * kMaxBlocks + 2 * wv] = fsdf_wave_ph2[wave][1];
      }
    }
#endif
  }

  // ---- block combine (fixed order) ----
  if (!ALIAS) {
    cost_acc = wave_sum(cost_acc);
    if (lane == 0) red_of(wave)[SLOTS * 64 * 6] = cost_acc;
  }
  __syncthreads();
  const int len6 = 1 + 6 * m.S;
  const int len = len6 + (RBF ? m.rbf_acc_off[m.R] : 0);
  for (int t = threadIdx.x; t < len; t += NB) {
    double s;
    if (t < len6) {
      const int src = (t == 0) ? SLOTS * 64 * 6 : t - 1;
      s = red_of(0)[src];
#pragma unroll
      for (int w = 1; w < NB / 64; ++w) s += red_of(w)[src];
    } else {
      const int src = RBF ? t - len6 : 0;
      s = rbf_acc[src];
#pragma unroll
      for (int w = 1; w < NB / 64; ++w) s += rbf_acc[w * kMaxRbfAcc + src];
    }
    out.partials[pidx(t, lb, gridDim.x)] = s;
  }
  if (out.cost && threadIdx.x == 0) out.cost[lb] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_block);
#if FSDF_WAVE_TIMES
  if (out.stats && threadIdx.x == 0 && lb < kMaxBlocks) {  // diagnostic: block start / end (100 MHz)
    out.stats[32 + 16 * kMaxBlocks + 2 * lb] = t_block0;
    out.stats[33 + 16 * kMaxBlocks + 2 * lb] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// ---------------------------------------------------------------------------
// Planned pass: resident clouds of hull-only scenes with <= 64 surfaces whose
// fp64 planes are staged (the aliased layout, pass_kernel ALIAS / HPART).
//
// Launch slot b runs plan[b], one of three workgroup shapes — 4 chunks of 64
// points one wave each; 2 chunks over 2 waves each; 1 chunk over all 4 waves
// (hull-partitioned: wave j evaluates the hulls k = j mod parts, bests shared
// through one ds_min_f64 slot per lane, merged by the first-index (d, k) rule,
// exactly as pass_kernel HPART) — chosen per chunk from the chunks' measured
// durations (plan_kernel: the heaviest chunks split over 4 or 2 waves, the
// rest grouped by similar cost, heaviest workgroups first). The pass is bound
// by its heaviest chunks' serial hull evaluations (~100 us at 2^20 points
// against ~70 us of average wave work); a per-chunk split only
// where it pays leaves the rest of the grid one wave per chunk. Without a
// plan (a new cloud's first pass) slot b runs `dparts` waves per chunk in
// index order — the size tiers of hpart_parts.
//
// Every chunk writes its OWN partial row — the chunk's Σ d², and its wrench
// sums (F, M) per nearest surface as up to 4 (k, F, M) entries, or a dense
// [S][6] row when more than 4 surfaces meet in the chunk — so the
// accumulator (reduce_chunks_kernel, one launch) sums the chunk rows in a
// fixed order whatever the plan: bit-identical across plans, schedules and
// passes. No block combine, no
// barrier after the prologue for one-wave chunks.
// ---------------------------------------------------------------------------
constexpr int kPlanChunkMask = (1 << kPlanPartsShift) - 1;

// One chunk's epilogue in the planned pass: the wave's wrench
// rows (lane k owns surface k) in its free stage, the per-point outputs, and
// the chunk's partial row — Σ d², then sparse (k, F, M) entries in ascending k
// or, when more than 4 surfaces meet in the chunk, a dense [S][6] row.
template <typename T>
__device__ __forceinline__ void emit_chunk_row(T px, T py, T pz, bool valid, T best, int bk, T gx, T gy, T gz, int cid,
                                               int64_t n, const PassModel<T>& m, const PassOutputs& out,
                                               const ChunkOutputs& co, T* __restrict__ stage) {
  const int lane = threadIdx.x & 63;
  const int64_t base = (int64_t)cid * 64;
  const int64_t i = base + lane;
  double* acc_row = (double*)stage + lane * 6;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
  for (int j = 0; j < 6; ++j) acc_row[j] = 0.0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  T* tstage = (T*)((char*)stage + (64 * 6 + 2) * 8);  // gradient transpose after the rows
  double cost_chunk = 0.0;
  const uint64_t touched = emit_chunk<T, 1, false>(px, py, pz, valid, best, bk, gx, gy, gz, i, base, n, m, out,
                                                   acc_row, cost_chunk, nullptr, tstage,
                                                   m.stage_bytes / (4 * (int)sizeof(T)));
  cost_chunk = wave_sum(cost_chunk);
  const int cnt = __builtin_popcountll(touched);
  if (cnt <= 4) {
    if ((touched >> lane) & 1) {
      const int sl = __builtin_popcountll(touched & ((1ull << lane) - 1));
      double* e = co.ent + ((int64_t)cid * 4 + sl) * 6;
#pragma unroll
      for (int j = 0; j < 6; ++j) e[j] = acc_row[j];
    }
    if (lane == 0) {
      I4 h = I4{-1, -1, -1, -1};
      uint64_t t = touched;
      for (int sl = 0; sl < 4 && t; ++sl) {
        h[sl] = __builtin_ctzll(t);
        t &= t - 1;
      }
      ((I4*)co.hdr)[cid] = h;
      co.csum[cid] = cost_chunk;
    }
  } else {
    if (lane < m.S) {
      double* r = co.dense + ((int64_t)cid * m.S + lane) * 6;  // [nc][S][6]
#pragma unroll
      for (int j = 0; j < 6; ++j) r[j] = acc_row[j];
    }
    if (lane == 0) {
      ((I4*)co.hdr)[cid] = I4{-2, -1, -1, -1};
      co.csum[cid] = cost_chunk;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // row reads before the stage is overwritten
}

template <typename T, bool CULL>
__global__ __launch_bounds__(kPassBlock) __attribute__((amdgpu_waves_per_eu(kPassWavesPerSimd))) void planned_pass_kernel(
    const T* __restrict__ pts, int64_t n, PassModel<T> m, PassOutputs out, ChunkOutputs co) {
  static_assert(kPassBlock == 256, "the planned pass runs 4-wave workgroups");
  if (out.skip && *out.skip) return;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  HullRow* ht = (HullRow*)fsdf_lds;
  char* stages = (char*)(ht + m.K + 1);
  T* stage = (T*)(stages + wave * m.stage_bytes);
  double* shb_all = (double*)(stages + 4 * m.stage_bytes);  // [4][64] shared per-lane bests
  uint64_t* t0_lds = (uint64_t*)(shb_all + 4 * 64);         // [4] chunk start times
  // this wave's (waves per chunk, chunk): re-read after the scene evaluation
  // rather than kept live through it (scalar registers are spilled to vector
  // lanes at this kernel's register budget)
  auto slot_of = [&](int& parts_, int& cid_) {
    if (co.plan) {
      const I4 e = ((const I4*)co.plan)[blockIdx.x];
      parts_ = (e[0] >> kPlanPartsShift) & 7;
      const int sl = wave / parts_;
      cid_ = sl == 0 ? (e[0] & kPlanChunkMask) : (sl == 1 ? e[1] : (sl == 2 ? e[2] : e[3]));
    } else {
      parts_ = co.dparts;
      cid_ = (int)blockIdx.x * (4 / parts_) + wave / parts_;
    }
    parts_ = __builtin_amdgcn_readfirstlane(parts_);
    cid_ = __builtin_amdgcn_readfirstlane(cid_);
  };
  int parts, cid;
  slot_of(parts, cid);
  const float smax = load_hull_table(m, ht);  // (the workgroup's one barrier for one-wave chunks)
  bool has = cid >= 0 && (int64_t)cid * 64 < n;
  if (!has && parts == 1) return;  // wave-uniform; no barrier follows for one-wave chunks
  if (lane == 0) t0_lds[wave] = __builtin_amdgcn_s_memrealtime();
  const int part = __builtin_amdgcn_readfirstlane(wave % parts);
  int64_t base = (int64_t)cid * 64;
  const bool valid = has && base + lane < n;
  const int64_t ii = valid ? base + lane : (has ? n - 1 : 0);
  const T px = pts[3 * ii + 0], py = pts[3 * ii + 1], pz = pts[3 * ii + 2];
  double* shb = parts > 1 ? shb_all + 64 * (wave / parts) : nullptr;
  if (parts > 1) {
    if (part == 0) ((volatile double*)shb)[lane] = __builtin_huge_val();
    __syncthreads();
  }
  T best = tinf<T>(), gx = (T)0, gy = (T)0, gz = (T)0;
  int bk = 0x7fffffff;
  if (has) {
    const uint64_t pm = parts == 4 ? (0x1111111111111111ull << part)
                                   : (parts == 2 ? (0x5555555555555555ull << part) : ~0ull);
    const F4* cws = out.chunk_ws ? (const F4*)out.chunk_ws + cid : nullptr;
    const int prior = (out.prior_in && valid) ? (int)out.prior_in[base + lane] : -1;
    scene_eval<T, 1, CULL, false, true, 0>(px, py, pz, valid, m, ht, smax, stage, out.stats, best, bk, gx, gy, gz,
                                           cws, pm, shb, prior);
  }
  if (parts > 1) {
    // the chunk's waves' results meet in their stages; part 0 keeps the
    // lexicographic (d, k) minimum per point (pass_kernel HPART's merge)
    T* rs = stage;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    rs[4 * lane + 0] = best; rs[4 * lane + 1] = gx; rs[4 * lane + 2] = gy; rs[4 * lane + 3] = gz;
    ((int*)(rs + 256))[lane] = bk;
    __syncthreads();
    if (part == 0) {
      for (int w = 1; w < parts; ++w) {
        const T* ro = (const T*)(stages + (wave + w) * m.stage_bytes);
        const T d2 = ro[4 * lane];
        const int k2 = ((const int*)(ro + 256))[lane];
        if (d2 < best || (d2 == best && k2 < bk)) {
          best = d2; bk = k2; gx = ro[4 * lane + 1]; gy = ro[4 * lane + 2]; gz = ro[4 * lane + 3];
        }
      }
    }
    __syncthreads();
  }
  if (!has || part != 0) return;  // (no barrier follows)
  slot_of(parts, cid);
  base = (int64_t)cid * 64;
  if (!valid) bk = 0;
  emit_chunk_row<T>(px, py, pz, valid, best, bk, gx, gy, gz, cid, n, m, out, co, stage);
  if (co.dur && lane == 0) {
    // serial-equivalent duration: a split chunk's wall time scaled by the
    // speed-up its split buys (ChunkOutputs::r4n / r4d, r2n / r2d)
    const uint64_t dt = __builtin_amdgcn_s_memrealtime() - t0_lds[wave];
    const uint64_t est = parts == 4 ? (dt * (uint64_t)co.r4n) / (uint64_t)co.r4d
                                    : (parts == 2 ? (dt * (uint64_t)co.r2n) / (uint64_t)co.r2d : dt);
    co.dur[cid] = (uint32_t)(est < 0xffffffffull ? est : 0xffffffffull);
  }
}

// The planned pass's reduction, stage 1: workgroup g sums the chunk rows of
// chunks 16g .. 16g+15 into row g of the line-tiled partials, which
// reduce_tiles_kernel (the unplanned pass's stage 2) then sums. The group's
// rows are expanded in LDS into a dense [16][len] table — zeros, each sparse
// entry scattered to its surface's columns, dense rows copied — and thread t
// sums column t over the 16 chunks in order. The sparse entries and Σ d² are
// one coalesced, unconditional read each (whatever the header says), issued
// before the headers are known: one memory latency per group. Deterministic,
// and it reads only the chunk rows: independent of the plan.
// (Gathering entry columns straight from the chunk rows — a thread per entry,
// a lane per chunk — touches 64 lines per wave load: 17 us at 2^17 points,
// 70 us at 2^20, tag-lookup bound on the few CUs the 49 tiles occupy.)
constexpr int kGroupChunks = 16;
constexpr int kGroupBlock = 512;
static_assert(kGroupChunks * 24 <= kGroupBlock, "one sparse entry per thread");
__global__ __launch_bounds__(kGroupBlock) void chunk_groups_kernel(const I4* __restrict__ hdr,
                                                                   const double* __restrict__ ent,
                                                                   const double* __restrict__ csum,
                                                                   const double* __restrict__ dense, int nc, int S,
                                                                   double* __restrict__ partials, int ngroups,
                                                                   const int* __restrict__ skip) {
  if (skip && *skip) return;
  const int len = 1 + 6 * S;
  const int g = blockIdx.x, tid = threadIdx.x;
  const int c0 = g * kGroupChunks;
  double* tab = (double*)fsdf_lds;                // [kGroupChunks][len]
  I4* sh = (I4*)(tab + kGroupChunks * len);       // [kGroupChunks] headers
  const int ec = tid / 24;                         // this thread's sparse entry: chunk c0 + ec, slot (tid % 24) / 6
  const bool inr = tid < kGroupChunks * 24 && c0 + ec < nc;
  const double v = ent[inr ? (int64_t)c0 * 24 + tid : 0];
  const int hc = c0 + (tid & (kGroupChunks - 1));
  const bool hv = hc < nc;
  const I4 h = hdr[hv ? hc : 0];
  const double cs = csum[hv ? hc : 0];
  for (int i = tid; i < kGroupChunks * len; i += kGroupBlock) tab[i] = 0.0;
  if (tid < kGroupChunks) sh[tid] = hv ? h : I4{-1, -1, -1, -1};
  __syncthreads();
  if (tid < kGroupChunks && hv) tab[tid * len] = cs;
  if (inr) {
    const I4 hh = sh[ec];
    const int sl = (tid % 24) / 6, j = tid % 6;
    const int k = sl == 0 ? hh[0] : (sl == 1 ? hh[1] : (sl == 2 ? hh[2] : hh[3]));
    if (hh[0] != -2 && k >= 0 && k < S) tab[ec * len + 1 + 6 * k + j] = v;
  }
  // dense rows (a chunk that met more than 4 surfaces): entry 1 + i = dense[i]
  for (int c = 0; c < kGroupChunks; ++c) {
    if (sh[c][0] == -2)
      for (int i = tid; i < 6 * S; i += kGroupBlock) tab[c * len + 1 + i] = dense[(int64_t)(c0 + c) * 6 * S + i];
  }
  __syncthreads();
  for (int t = tid; t < len; t += kGroupBlock) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < kGroupChunks; ++c) s += tab[c * len + t];
    partials[pidx(t, g, ngroups)] = s;
  }
}

// The plan for the next passes (one workgroup, kPlanBlock threads): a counting
// sort of the chunks' serial-equivalent durations into kPlanBuckets buckets,
// heaviest first; the first n4 chunks of that order get a workgroup each (4
// waves), the next n2 one per 2 waves (pairs of similar cost), the rest one
// wave each in groups of 4 consecutive (similar cost: little idle inside a
// workgroup). Workgroups are listed in that order — heaviest first, longest-
// processing-time-first list scheduling. `order` is [nc] scratch.
constexpr int kPlanBlock = 1024;
constexpr int kPlanBuckets = 256;
__global__ __launch_bounds__(kPlanBlock) void plan_kernel(const uint32_t* __restrict__ dur, int nc, int n4, int n2,
                                                          int32_t* __restrict__ order, I4* __restrict__ plan) {
  __shared__ unsigned hist[kPlanBuckets];
  __shared__ unsigned wmax[kPlanBlock / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned mx = 0;
  for (int c = t; c < nc; c += kPlanBlock) mx = max(mx, dur[c]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, off, 64));
  if (lane == 0) wmax[w] = mx;
  for (int b = t; b < kPlanBuckets; b += kPlanBlock) hist[b] = 0;
  __syncthreads();
  mx = 0;
  for (int j = 0; j < kPlanBlock / 64; ++j) mx = max(mx, wmax[j]);
  const float sc = (float)(kPlanBuckets - 1) / (float)(mx ? mx : 1u);
  auto bucket = [&](int c) { return kPlanBuckets - 1 - min(kPlanBuckets - 1, (int)((float)dur[c] * sc)); };
  for (int c = t; c < nc; c += kPlanBlock) atomicAdd(&hist[bucket(c)], 1u);
  __syncthreads();
  if (t == 0) {  // exclusive scan (256 buckets, once per plan)
    unsigned acc = 0;
    for (int b = 0; b < kPlanBuckets; ++b) {
      const unsigned h = hist[b];
      hist[b] = acc;
      acc += h;
    }
  }
  __syncthreads();
  for (int c = t; c < nc; c += kPlanBlock) order[atomicAdd(&hist[bucket(c)], 1u)] = c;
  __threadfence();
  __syncthreads();
  const int n1 = nc - n4 - n2;
  const int g2 = n2 / 2 + (n2 & 1), g1 = (n1 + 3) / 4;
  for (int b = t; b < n4 + g2 + g1; b += kPlanBlock) {
    I4 e = I4{-1, -1, -1, -1};
    if (b < n4) {
      e[0] = order[b] | (4 << kPlanPartsShift);
    } else if (b < n4 + g2) {
      const int p0 = n4 + 2 * (b - n4);
      e[0] = order[p0] | (2 << kPlanPartsShift);
      if (p0 + 1 < n4 + n2) e[1] = order[p0 + 1];
    } else {
      const int p0 = n4 + n2 + 4 * (b - n4 - g2);
      e[0] = order[p0] | (1 << kPlanPartsShift);
      for (int j = 1; j < 4; ++j)
        if (p0 + j < nc) e[j] = order[p0 + j];
    }
    plan[b] = e;
  }
}

// ---------------------------------------------------------------------------
// Depth-sensor raycast (src/depthsensors.jl:56-97, doRaycast): secant march
// along each ray on the scene SDF from the sensor origin:
//   step = -last/est_grad, clamped to |step| <= 0.4; est_grad starts at -1;
//   stop when |SDF| <= 1e-5 or after 60 steps; depth = NaN when the final
//   |SDF| > 1e-2. One lane per ray; each step is one wave-cooperative
//   scene_eval (lanes that have converged ride along as invalid).
// ---------------------------------------------------------------------------
struct RayOrigin {
  double x, y, z;
};

template <typename T, int SLOTS, bool CULL, bool RBF>
__global__ __launch_bounds__(kBlock, (SLOTS == 1 ? kPassWavesPerSimd : (SLOTS == 2 ? 3 : 2)) - (RBF ? 1 : 0)) void
raycast_kernel(RayOrigin o, const double* __restrict__ rays, int64_t n, PassModel<T> m, double* __restrict__ depth) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  HullRow* ht = (HullRow*)fsdf_lds;  // dynamic LDS: hull table, then 4 wave stages
  T* stage = (T*)((char*)(ht + m.K + 1) + wave * m.stage_bytes);
  const float smax = load_hull_table(m, ht);
  const T EPS = (T)1e-5, SAFE_RATE = (T)0.4;
  const int SAFE_ITER_LIMIT = 60;
  const T ox = (T)o.x, oy = (T)o.y, oz = (T)o.z;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t base = (int64_t)blockIdx.x * kBlock + wave * 64; base < n; base += stride) {
    const int64_t i = base + lane;
    const bool valid = i < n;
    const int64_t ii = valid ? i : n - 1;
    const T rx = (T)rays[3 * ii + 0], ry = (T)rays[3 * ii + 1], rz = (T)rays[3 * ii + 2];
    T dist = (T)0, est = (T)-1, last, gx, gy, gz;
    int bk, k = 0;
    scene_eval<T, SLOTS, CULL, RBF>(ox + dist * rx, oy + dist * ry, oz + dist * rz, valid, m, ht, smax, stage, nullptr,
                                    last, bk, gx, gy, gz);
    bool active = valid && fabs(last) > EPS;
    while (__any(active)) {
      T step = (T)0;
      if (active) {
        step = -last / est;
        const T a = fabs(step);
        step = copysign(a < SAFE_RATE ? a : SAFE_RATE, step);
        dist += step;
      }
      T v;
      scene_eval<T, SLOTS, CULL, RBF>(ox + dist * rx, oy + dist * ry, oz + dist * rz, active, m, ht, smax, stage,
                                      nullptr, v, bk, gx, gy, gz);
      if (active) {
        est = (v - last) / step;
        last = v;
        ++k;
        active = fabs(last) > EPS && k < SAFE_ITER_LIMIT;
      }
    }
    if (valid) depth[i] = fabs(last) > (T)1000 * EPS ? __builtin_nan("") : (double)dist;
  }
}

// Schedule for the next pass (one workgroup): the workgroups of a pass hold
// their slot until their slowest wave ends and durations vary ~10x (waves
// whose points span several hulls), so launching the logical blocks in index
// order leaves a tail of late heavy blocks. Counting sort of this pass's
// durations into 64 buckets, heaviest first (list scheduling, longest first).
__device__ void build_order(const uint32_t* __restrict__ cost, int nb, int32_t* __restrict__ order) {
  constexpr int kPer = 16;  // costs per thread and tile (tile = 4,096 blocks)
  __shared__ uint8_t bkt[kMaxBlocks];
  __shared__ unsigned hist[64][kBlock / 64];  // [bucket][wave]: 4x less atomic contention
  __shared__ unsigned wmax[kBlock / 64];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  unsigned mx = 0;
  for (int b0 = 0; b0 < nb; b0 += kPer * kBlock) {
    unsigned c[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = b0 + u * kBlock + t;
      c[u] = i < nb ? cost[i] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) mx = max(mx, c[u]);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, off, 64));
  if (lane == 0) wmax[w] = mx;
  hist[lane][w] = 0;
  __syncthreads();
  mx = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
  const float sc = 63.0f / (float)(mx ? mx : 1u);
  for (int b0 = 0; b0 < nb; b0 += kPer * kBlock) {
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = b0 + u * kBlock + t;
      if (i < nb) {
        const int b = 63 - min(63, (int)((float)cost[i] * sc));  // 0 = heaviest
        bkt[i] = (uint8_t)b;
        atomicAdd(&hist[b][w], 1u);
      }
    }
  }
  __syncthreads();
  // exclusive scan over (bucket, wave) in bucket-major order: wave 0, lane = bucket
  if (w == 0) {
    const unsigned h0 = hist[lane][0], h1 = hist[lane][1], h2 = hist[lane][2], h3 = hist[lane][3];
    const unsigned tot = h0 + h1 + h2 + h3;
    unsigned inc = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned o = (unsigned)__shfl_up((int)inc, off, 64);
      if (lane >= off) inc += o;
    }
    const unsigned ex = inc - tot;
    hist[lane][0] = ex;
    hist[lane][1] = ex + h0;
    hist[lane][2] = ex + h0 + h1;
    hist[lane][3] = ex + h0 + h1 + h2;
  }
  __syncthreads();
  for (int b0 = 0; b0 < nb; b0 += kPer * kBlock) {
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = b0 + u * kBlock + t;
      if (i < nb) order[atomicAdd(&hist[bkt[i]][w], 1u)] = i;
    }
  }
}

// Line-tiled partials: workgroup x (16 waves) sums
// entries 8x .. 8x+7 over all blocks. The tile is read as a flat array of
// 16-B pairs, fully coalesced: thread i reads pairs i + 1024 j (pair e holds
// entries 2 (e & 3), +1 of block e >> 2), 16 loads in flight, so it always
// sums the same two entries over blocks (i >> 2) + 256 j, in order; then per
// entry pair a masked DPP wave sum and a fixed-order 16-wave combine
// (deterministic). The schedule rebuild is a launch of its own (order_kernel).
constexpr int kTileBlock = 1024;
__global__ __launch_bounds__(kTileBlock) void reduce_tiles_kernel(const double* __restrict__ partials, int nblocks,
                                                                  int len, double* __restrict__ accum,
                                                                  const int* __restrict__ skip) {
  if (skip && *skip) return;
  const int x = blockIdx.x;
  typedef double D2 __attribute__((ext_vector_type(2)));
  const D2* tile = (const D2*)(partials + (int64_t)x * nblocks * 8);
  const int np = 4 * nblocks;  // pairs in the tile
  double s0 = 0.0, s1 = 0.0;
  int e = threadIdx.x;
  // U loads in flight per thread, the last batch predicated (a serial tail
  // loop cost one L2 round trip per pair: 5.5 us at 2^17 points, where a
  // thread has 8 pairs). Same addition order; the missing pairs add +0.0,
  // which leaves a sum that started at +0.0 bit for bit unchanged.
  constexpr int U = 16;
  for (; e < np; e += U * kTileBlock) {
    D2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = e + u * kTileBlock;
      v[u] = i < np ? tile[i] : D2{0.0, 0.0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) { s0 += v[u][0]; s1 += v[u][1]; }
  }
  constexpr int W = kTileBlock / 64;
  __shared__ double sh[8][W];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane & 3;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const double w0 = wave_sum(q == r ? s0 : 0.0), w1 = wave_sum(q == r ? s1 : 0.0);
    if (lane == 0) { sh[2 * r][wave] = w0; sh[2 * r + 1][wave] = w1; }
  }
  __syncthreads();
  const int t = 8 * x + (int)threadIdx.x;
  if (threadIdx.x < 8 && t < len) {
    double a[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
      a[g] = (sh[threadIdx.x][4 * g] + sh[threadIdx.x][4 * g + 1]) + (sh[threadIdx.x][4 * g + 2] + sh[threadIdx.x][4 * g + 3]);
    accum[t] = (a[0] + a[1]) + (a[2] + a[3]);
  }
}

__global__ __launch_bounds__(kBlock) void order_kernel(const uint32_t* __restrict__ cost, int nblocks,
                                                       int32_t* __restrict__ order) {
  build_order(cost, nblocks, order);
}


__global__ void to_f32_kernel(const double* __restrict__ src, float* __restrict__ dst, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) dst[i] = (float)src[i];
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
// the aliased pass's LDS plus the hull-partitioned pass's shared per-lane bests
// (one 64-double slot row per chunk of the workgroup)
static size_t hpart_lds_bytes(const LocalModel& lm, int parts) {
  return (size_t)(kHpartBlock / 64) * lm.stage_bytes + (size_t)(lm.K + 1) * sizeof(HullRow) +
         (size_t)kHpartBlock / parts * sizeof(double);
}

// Waves per chunk of the hull-partitioned pass (pass_kernel HPART) for a cloud
// of n points, 0 = the one-wave-per-chunk pass: kHpart (4) up to the model's
// hpart4 limit, 2 up to its hpart2 limit (LocalModel; fsdf_set_partition
// overrides them per context, 0 disables a tier).
void hpart_default_limits(const LocalModel& lm, int64_t* four, int64_t* two) {
  // Measured crossovers (same-box size sweeps of every tier):
  // M64 (64 hulls) 4-way up to 196,608 points, 2-way up to 393,216
  // (profiles/r04/plan_sweeps_r04def.jsonl); IRB140 (7 hulls) 4-way up to
  // 98,304, 2-way up to 327,680 (profiles/r04/hpart_sweep_c2.jsonl: 4-way
  // best at 2^16, 2-way at 2^17..2^18, one wave from 393,216)
  if (lm.K >= kHpartFullHulls) {
    *four = 196608;
    *two = 393216;
  } else {
    *four = kHpartSmall4;
    *two = kHpartSmall2;
  }
}

int64_t planned_default_max_points(const LocalModel& lm) {
  return lm.K >= kHpartFullHulls ? kPlanMaxFull : kPlanMaxSmall;
}
int64_t planned_default_min_points() { return kPlanMinPoints; }

int hpart_parts(const LocalModel& lm, int64_t n) {
  if (!(FSDF_RED_IN_STAGE && lm.planes64 && lm.S <= 64 && lm.R == 0 && n > 0)) return 0;
  int64_t limit4, limit2;
  hpart_default_limits(lm, &limit4, &limit2);
  if (lm.hpart4_points >= 0) limit4 = lm.hpart4_points;
  if (lm.hpart2_points >= 0) limit2 = lm.hpart2_points;
  const int parts = n <= limit4 ? kHpart : (n <= limit2 ? 2 : 0);
  if (!parts) return 0;
  const int64_t per = kHpartBlock / parts;  // points per workgroup
  if ((n + per - 1) / per > kMaxBlocks) return 0;
  if (hpart_lds_bytes(lm, parts) > (size_t)kLdsPerCu * kHpartBlock / 1024) return 0;  // (4 waves per SIMD)
  return parts;
}
bool hpart_pass(const LocalModel& lm, int64_t n) { return hpart_parts(lm, n) > 0; }

static bool alias_pass(const LocalModel& lm, int64_t n) {
  return FSDF_RED_IN_STAGE && lm.planes64 && lm.S <= 64 && lm.R == 0 && n > 0 && (n + kAliasBlock - 1) / kAliasBlock <= kMaxBlocks;
}
static size_t alias_lds_bytes(const LocalModel& lm) {
  return (size_t)(kAliasBlock / 64) * lm.stage_bytes + (size_t)(lm.K + 1) * sizeof(HullRow);
}

int pass_blocks(int64_t n, const LocalModel& lm) {
  if (const int parts = hpart_parts(lm, n)) return (int)((n + kHpartBlock / parts - 1) / (kHpartBlock / parts));
  if (alias_pass(lm, n)) return (int)((n + kAliasBlock - 1) / kAliasBlock);
  int64_t b = (n + kPassBlock - 1) / kPassBlock;
  if (b < 1) b = 1;
  if (b > kMaxBlocks) b = kMaxBlocks;
  return (int)b;
}

hipError_t launch_pose(int precision, const LocalModel& lm, const double* d_poses, const PosedModel& pm,
                       hipStream_t s, const double* h_poses, const int* skip) {
  const int total = ((lm.F + lm.V + 63) & ~63) + 64 * lm.K;
  if (total == 0) return hipSuccess;  // RBF-only scene: nothing to pose
  const int grid = (total + kBlock - 1) / kBlock;
  if (h_poses) {
    PoseArgs pa;
    memcpy(pa.v, h_poses, (size_t)12 * lm.S * sizeof(double));
    if (precision == 64)
      hipLaunchKernelGGL(pose_kernel_args<double>, dim3(grid), dim3(kBlock), 0, s, lm, pa, (double*)pm.planes_w,
                         pm.spheres_w, (double*)pm.verts_w, (double*)pm.hscale_w, pm.screen_w, (I4*)pm.image_w);
    else
      hipLaunchKernelGGL(pose_kernel_args<float>, dim3(grid), dim3(kBlock), 0, s, lm, pa, (float*)pm.planes_w,
                         pm.spheres_w, (float*)pm.verts_w, (float*)pm.hscale_w, (float*)nullptr, (I4*)nullptr);
    return hipGetLastError();
  }
  if (precision == 64) {
    hipLaunchKernelGGL(pose_kernel<double>, dim3(grid), dim3(kBlock), 0, s, lm, d_poses,
                       (double*)pm.planes_w, pm.spheres_w, (double*)pm.verts_w, (double*)pm.hscale_w,
                       pm.screen_w, (I4*)pm.image_w, skip);
  } else {
    hipLaunchKernelGGL(pose_kernel<float>, dim3(grid), dim3(kBlock), 0, s, lm, d_poses, (float*)pm.planes_w,
                       pm.spheres_w, (float*)pm.verts_w, (float*)pm.hscale_w, (float*)nullptr, (I4*)nullptr, skip);
  }
  return hipGetLastError();
}

template <typename T>
static PassModel<T> pass_model(const LocalModel& lm, const PosedModel& pm) {
  PassModel<T> m;
  m.K = lm.K;
  m.S = lm.S;
  m.R = lm.R;
  m.stage_bytes = lm.stage_bytes;
  m.planes64 = lm.planes64;
  m.hull_surface = lm.hull_surface;
  m.surface_kind = lm.surface_kind;
  m.rbf_surface = lm.rbf_surface;
  m.rbf_row_off = lm.rbf_row_off;
  m.rbf_acc_off = lm.rbf_acc_off;
  m.rbf_rows = (const T*)pm.rbf_rows;
  m.face_off = lm.face_off;
  m.vert_off = lm.vert_off;
  m.face_rows = (const I4*)lm.face_rows;
  m.planes = (const T*)pm.planes_w;
  m.verts = (const T*)pm.verts_w;
  m.hscale = (const T*)pm.hscale_w;
  m.spheres = pm.spheres_w;
  m.screen = pm.screen_w;
  m.image = (const I4*)pm.image_w;
  return m;
}

static int slots_for(int S) { return S <= 64 ? 1 : (S <= 128 ? 2 : 4); }

size_t pass_lds_bytes(const LocalModel& lm, bool raycast, bool alias) {
  const size_t waves = (size_t)(raycast ? kBlock : kPassBlock) / 64;
  const size_t stage = waves * (size_t)lm.stage_bytes + (size_t)(lm.K + 1) * sizeof(HullRow);
  if (raycast || alias) return stage;
  const size_t red = waves * (size_t)(slots_for(lm.S) * 64 * 6 + 2) * sizeof(double);
  const size_t rbf = lm.R > 0 ? waves * kMaxRbfAcc * sizeof(double) : 0;
  return red + rbf + stage;
}

// start/stop events of the next pass launch (launch_pass; this thread only):
// hipExtLaunchKernel stamps them in the dispatch itself, where a separate
// hipEventRecord is a stream packet of its own that held the next kernel
// back by ~5-10 us (profiles/r03, step_trace)
static thread_local hipEvent_t g_pass_ev0 = nullptr, g_pass_ev1 = nullptr;

template <typename K, typename... Args>
static void launch_lds(K kernel, int grid, int block, size_t lds, hipStream_t s, Args... args) {
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (g_pass_ev0 || g_pass_ev1) {
    hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(block), (uint32_t)lds, s, g_pass_ev0, g_pass_ev1, 0u, args...);
    g_pass_ev0 = g_pass_ev1 = nullptr;
  } else {
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), lds, s, args...);
  }
}

static thread_local char g_pass_name[96] = "";
const char* last_pass_kernel() { return g_pass_name; }

template <typename T> constexpr const char* type_name();
template <> constexpr const char* type_name<double>() { return "double"; }
template <> constexpr const char* type_name<float>() { return "float"; }

// launch one pass_kernel variant and record its name (last_pass_kernel)
template <typename T, int SLOTS, bool CULL, bool RBF, bool ALIAS = false, bool HPART = false, int NB = kPassBlock,
          int NPART = kHpart>
static void launch_pass_variant(int grid, size_t lds, hipStream_t s, const T* pts, int64_t n, const PassModel<T>& m,
                                const PassOutputs& out) {
  auto b = [](bool v) { return v ? "true" : "false"; };
  snprintf(g_pass_name, sizeof g_pass_name, "pass_kernel<%s, %d, %s, %s, %s, %s, %d, %d>", type_name<T>(), SLOTS,
           b(CULL), b(RBF), b(ALIAS), b(HPART), NB, NPART);
  launch_lds(pass_kernel<T, SLOTS, CULL, RBF, ALIAS, HPART, NB, NPART>, grid, NB, lds, s, pts, n, m, out);
}

template <typename T, bool CULL, bool RBF>
static void launch_pass_t(const LocalModel& lm, const PosedModel& pm, const void* d_pts, int64_t n, int nblocks,
                          const PassOutputs& out, hipStream_t s) {
  const PassModel<T> m = pass_model<T>(lm, pm);
  const T* pts = (const T*)d_pts;
  const size_t lds = pass_lds_bytes(lm, false);
  if constexpr (!RBF && FSDF_RED_IN_STAGE) {
    // one chunk per wave: the wrench rows alias the stage (pass_kernel ALIAS)
    if (const int parts = hpart_parts(lm, n)) {
      if (parts == kHpart)
        launch_pass_variant<T, 1, CULL, false, true, true, kHpartBlock, kHpart>(nblocks, hpart_lds_bytes(lm, parts), s,
                                                                                pts, n, m, out);
      else
        launch_pass_variant<T, 1, CULL, false, true, true, kHpartBlock, 2>(nblocks, hpart_lds_bytes(lm, parts), s, pts,
                                                                           n, m, out);
      return;
    }
    if (alias_pass(lm, n) && (int64_t)nblocks * kAliasBlock >= n) {
      launch_pass_variant<T, 1, CULL, false, true, false, kAliasBlock>(nblocks, alias_lds_bytes(lm), s, pts, n, m, out);
      return;
    }
  }
  if (lm.S <= 64) launch_pass_variant<T, 1, CULL, RBF>(nblocks, lds, s, pts, n, m, out);
  else if (lm.S <= 128) launch_pass_variant<T, 2, CULL, RBF>(nblocks, lds, s, pts, n, m, out);
  else launch_pass_variant<T, 4, CULL, RBF>(nblocks, lds, s, pts, n, m, out);
}

// FSDF_BENCH_ONLY=1: A/B timing builds instantiate only the bench variant
// (f64, culled, hulls only, <= 64 surfaces); every other pass is refused.
#ifndef FSDF_BENCH_ONLY
#define FSDF_BENCH_ONLY 0
#endif

template <typename T>
static void launch_pass_p(bool cull, const LocalModel& lm, const PosedModel& pm, const void* d_pts, int64_t n,
                          int nblocks, const PassOutputs& out, hipStream_t s) {
#if FSDF_BENCH_ONLY
  const PassModel<T> m = pass_model<T>(lm, pm);
  const int parts = hpart_parts(lm, n);
  const T* pts = (const T*)d_pts;
  if (parts == kHpart)
    launch_pass_variant<T, 1, true, false, true, true, kHpartBlock, kHpart>(nblocks, hpart_lds_bytes(lm, parts), s,
                                                                            pts, n, m, out);
  else if (parts == 2)
    launch_pass_variant<T, 1, true, false, true, true, kHpartBlock, 2>(nblocks, hpart_lds_bytes(lm, parts), s, pts, n,
                                                                       m, out);
  else if (alias_pass(lm, n) && (int64_t)nblocks * kAliasBlock >= n)
    launch_pass_variant<T, 1, true, false, true, false, kAliasBlock>(nblocks, alias_lds_bytes(lm), s, pts, n, m, out);
  else
    launch_pass_variant<T, 1, true, false>(nblocks, pass_lds_bytes(lm, false), s, pts, n, m, out);
#else
  if (lm.R > 0) {
    if (cull) launch_pass_t<T, true, true>(lm, pm, d_pts, n, nblocks, out, s);
    else launch_pass_t<T, false, true>(lm, pm, d_pts, n, nblocks, out, s);
  } else {
    if (cull) launch_pass_t<T, true, false>(lm, pm, d_pts, n, nblocks, out, s);
    else launch_pass_t<T, false, false>(lm, pm, d_pts, n, nblocks, out, s);
  }
#endif
}

hipError_t launch_pass(int precision, bool cull, const LocalModel& lm, const PosedModel& pm, const void* d_pts,
                       int64_t n, int nblocks, const PassOutputs& out, hipStream_t s, hipEvent_t ev_start,
                       hipEvent_t ev_stop) {
  // the events belong to this call only: cleared on every exit (a refused or
  // failed launch must not leave them for the next launch_lds on this thread)
  struct ClearEvents {
    ~ClearEvents() { g_pass_ev0 = g_pass_ev1 = nullptr; }
  } clear_events;
  g_pass_name[0] = 0;
  g_pass_ev0 = ev_start;
  g_pass_ev1 = ev_stop;
#if FSDF_BENCH_ONLY
  if (precision != 64 || !cull || lm.R > 0 || lm.S > 64) return hipErrorNotSupported;
  launch_pass_p<double>(cull, lm, pm, d_pts, n, nblocks, out, s);
#else
  if (precision == 64) launch_pass_p<double>(cull, lm, pm, d_pts, n, nblocks, out, s);
  else launch_pass_p<float>(cull, lm, pm, d_pts, n, nblocks, out, s);
#endif
  return hipGetLastError();
}

template <typename T, bool CULL, bool RBF>
static void launch_raycast_t(const LocalModel& lm, const PosedModel& pm, const double* origin, const double* rays,
                             int64_t n, double* depth, hipStream_t s) {
  const PassModel<T> m = pass_model<T>(lm, pm);
  const RayOrigin o{origin[0], origin[1], origin[2]};
  const int nb = (int)std::min<int64_t>((n + kBlock - 1) / kBlock, kMaxBlocks);
  const size_t lds = pass_lds_bytes(lm, true);
  if (lm.S <= 64) launch_lds(raycast_kernel<T, 1, CULL, RBF>, nb, kBlock, lds, s, o, rays, n, m, depth);
  else if (lm.S <= 128) launch_lds(raycast_kernel<T, 2, CULL, RBF>, nb, kBlock, lds, s, o, rays, n, m, depth);
  else launch_lds(raycast_kernel<T, 4, CULL, RBF>, nb, kBlock, lds, s, o, rays, n, m, depth);
}

template <typename T>
static void launch_raycast_p(bool cull, const LocalModel& lm, const PosedModel& pm, const double* origin,
                             const double* rays, int64_t n, double* depth, hipStream_t s) {
  if (lm.R > 0) {
    if (cull) launch_raycast_t<T, true, true>(lm, pm, origin, rays, n, depth, s);
    else launch_raycast_t<T, false, true>(lm, pm, origin, rays, n, depth, s);
  } else {
    if (cull) launch_raycast_t<T, true, false>(lm, pm, origin, rays, n, depth, s);
    else launch_raycast_t<T, false, false>(lm, pm, origin, rays, n, depth, s);
  }
}

hipError_t launch_raycast(int precision, bool cull, const LocalModel& lm, const PosedModel& pm, const double* origin,
                          const double* d_rays, int64_t n, double* d_depth, hipStream_t s) {
  if (n <= 0) return hipSuccess;
#if FSDF_BENCH_ONLY
  return hipErrorNotSupported;
#else
  if (precision == 64) launch_raycast_p<double>(cull, lm, pm, origin, d_rays, n, d_depth, s);
  else launch_raycast_p<float>(cull, lm, pm, origin, d_rays, n, d_depth, s);
#endif
  return hipGetLastError();
}

hipError_t launch_reduce(const double* partials, int nblocks, int len, double* d_accum, hipStream_t s,
                         const uint32_t* cost, int32_t* order, hipEvent_t ev_stop, const int* skip) {
  if (ev_stop)
    hipExtLaunchKernelGGL(reduce_tiles_kernel, dim3((len + 7) / 8), dim3(kTileBlock), 0u, s, nullptr, ev_stop, 0u,
                          partials, nblocks, len, d_accum, skip);
  else
    hipLaunchKernelGGL(reduce_tiles_kernel, dim3((len + 7) / 8), dim3(kTileBlock), 0, s, partials, nblocks, len,
                       d_accum, skip);
  if (cost) hipLaunchKernelGGL(order_kernel, dim3(1), dim3(kBlock), 0, s, cost, nblocks, order);
  return hipGetLastError();
}

// the planned pass's LDS: the hull-partitioned layout + 4 chunk start times
static size_t planned_lds_bytes(const LocalModel& lm) { return hpart_lds_bytes(lm, 1) + 4 * sizeof(uint64_t); }

bool planned_pass(const LocalModel& lm, int64_t n) {
  return FSDF_RED_IN_STAGE && lm.planes64 && lm.S <= 64 && lm.R == 0 && n > 0 && (n + 63) / 64 <= kMaxPlanChunks &&
         planned_lds_bytes(lm) <= (size_t)kLdsPerCu / 4;
}

template <typename T>
static void launch_planned_t(bool cull, const LocalModel& lm, const PosedModel& pm, const void* d_pts, int64_t n,
                             int grid, const PassOutputs& out, const ChunkOutputs& co, hipStream_t s) {
  const PassModel<T> m = pass_model<T>(lm, pm);
  auto b = [](bool v) { return v ? "true" : "false"; };
  snprintf(g_pass_name, sizeof g_pass_name, "planned_pass_kernel<%s, %s>", type_name<T>(), b(cull));
  if (cull)
    launch_lds(planned_pass_kernel<T, true>, grid, kPassBlock, planned_lds_bytes(lm), s, (const T*)d_pts, n, m, out,
               co);
  else
    launch_lds(planned_pass_kernel<T, false>, grid, kPassBlock, planned_lds_bytes(lm), s, (const T*)d_pts, n, m, out,
               co);
}

hipError_t launch_planned_pass(int precision, bool cull, const LocalModel& lm, const PosedModel& pm, const void* d_pts,
                               int64_t n, int grid, const PassOutputs& out, const ChunkOutputs& co, hipStream_t s,
                               hipEvent_t ev_start, hipEvent_t ev_stop) {
  struct ClearEvents {
    ~ClearEvents() { g_pass_ev0 = g_pass_ev1 = nullptr; }
  } clear_events;
  g_pass_name[0] = 0;
  if (precision != 64) return hipErrorNotSupported;  // (planes64: f64 contexts only)
  g_pass_ev0 = ev_start;
  g_pass_ev1 = ev_stop;
  launch_planned_t<double>(cull, lm, pm, d_pts, n, grid, out, co, s);
  return hipGetLastError();
}

hipError_t launch_reduce_chunks(const ChunkOutputs& co, int64_t nc, int S, double* partials, double* d_accum,
                                hipStream_t s, hipEvent_t ev_stop, const int* skip) {
  const int len = 1 + 6 * S;
  const int ngroups = (int)reduce_chunk_groups(nc);
  const size_t lds = (size_t)kGroupChunks * len * sizeof(double) + kGroupChunks * sizeof(I4);
  hipLaunchKernelGGL(chunk_groups_kernel, dim3(ngroups), dim3(kGroupBlock), lds, s, (const I4*)co.hdr, co.ent, co.csum,
                     co.dense, (int)nc, S, partials, ngroups, skip);
  return launch_reduce(partials, ngroups, len, d_accum, s, nullptr, nullptr, ev_stop, skip);
}

int64_t reduce_chunk_groups(int64_t nc) { return (nc + kGroupChunks - 1) / kGroupChunks; }

hipError_t launch_plan(const uint32_t* dur, int64_t nc, int n4, int n2, int32_t* order, int32_t* plan, hipStream_t s) {
  hipLaunchKernelGGL(plan_kernel, dim3(1), dim3(kPlanBlock), 0, s, dur, (int)nc, n4, n2, order, (I4*)plan);
  return hipGetLastError();
}

hipError_t launch_chunk_spheres(int precision, const void* d_pts, int64_t n, int64_t nchunks, float* d_out,
                                hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned grid = (unsigned)((64 * nchunks + kBlock - 1) / kBlock);
  if (precision == 64)
    hipLaunchKernelGGL(chunk_sphere_kernel<double>, dim3(grid), dim3(kBlock), 0, s, (const double*)d_pts, n, nchunks,
                       (F4*)d_out);
  else
    hipLaunchKernelGGL(chunk_sphere_kernel<float>, dim3(grid), dim3(kBlock), 0, s, (const float*)d_pts, n, nchunks,
                       (F4*)d_out);
  return hipGetLastError();
}

hipError_t launch_to_f32(const double* src, float* dst, int64_t count, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  const int64_t grid = (count + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(to_f32_kernel, dim3((unsigned)grid), dim3(kBlock), 0, s, src, dst, count);
  return hipGetLastError();
}

}  // namespace fsdf
