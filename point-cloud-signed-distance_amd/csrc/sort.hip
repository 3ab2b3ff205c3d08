// sort.hip — spatial ordering of the resident cloud (fsdf_opts.sort_points).
//
// The pass kernel evaluates a hull for a whole wave when any of its 64 lanes
// needs it, so its cost follows the spatial coherence of consecutive points.
// Depth sensors deliver raster order (src/depthdata.jl:19-30,
// src/depthsensors.jl:99-113), which is already coherent; an arbitrary order
// is made coherent here once per frame: 30-bit Hilbert keys (10 bits per axis)
// over the cloud's bounding box, a device radix sort (rocPRIM) of (key, int32
// index) pairs, and a gather. The permutation is kept so per-point outputs
// still land in the caller's order. Hilbert rather than Morton order: a Morton
// curve jumps at every octree boundary, so some 64-point chunks straddle two
// distant regions and need the hulls of both; on the bench cloud the pass is
// 8.5 % faster (0.144 -> 0.132 ms; -DFSDF_HILBERT=0 restores Morton keys).
//
// Per frame: bbox partials (<= 256 blocks) -> one-block finalize -> keys ->
// radix sort -> gather. All scratch lives in the context (SortScratch, grown
// only), so a frame makes no allocation and no implicit device sync.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "fsdf_internal.h"

namespace fsdf {

namespace {

constexpr int kBoxBlocks = 256;

__global__ __launch_bounds__(kBlock) void bbox_partial_kernel(const double* __restrict__ pts, int64_t n,
                                                              double* __restrict__ part) {
  double lo[3] = {__builtin_huge_val(), __builtin_huge_val(), __builtin_huge_val()};
  double hi[3] = {-__builtin_huge_val(), -__builtin_huge_val(), -__builtin_huge_val()};
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double v = pts[3 * i + j];
      lo[j] = fmin(lo[j], v);
      hi[j] = fmax(hi[j], v);
    }
  }
  __shared__ double sh[6][kBlock];
#pragma unroll
  for (int j = 0; j < 3; ++j) { sh[j][threadIdx.x] = lo[j]; sh[3 + j][threadIdx.x] = hi[j]; }
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        sh[j][threadIdx.x] = fmin(sh[j][threadIdx.x], sh[j][threadIdx.x + w]);
        sh[3 + j][threadIdx.x] = fmax(sh[3 + j][threadIdx.x], sh[3 + j][threadIdx.x + w]);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x < 6) part[6 * blockIdx.x + threadIdx.x] = sh[threadIdx.x][0];
}

// one block: the <= 256 partials -> box[6] = (lo xyz, hi xyz)
__global__ __launch_bounds__(kBlock) void bbox_final_kernel(const double* __restrict__ part, int nparts,
                                                            double* __restrict__ box) {
  __shared__ double sh[6][kBlock];
  const int t = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 6; ++j) sh[j][t] = t < nparts ? part[6 * t + j] : (j < 3 ? __builtin_huge_val() : -__builtin_huge_val());
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (t < w) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        sh[j][t] = fmin(sh[j][t], sh[j][t + w]);
        sh[3 + j][t] = fmax(sh[3 + j][t], sh[3 + j][t + w]);
      }
    }
    __syncthreads();
  }
  if (t < 6) box[t] = sh[t][0];
}

__device__ __forceinline__ uint32_t spread10(uint32_t v) {
  v &= 0x3ff;
  v = (v | (v << 16)) & 0x030000ff;
  v = (v | (v << 8)) & 0x0300f00f;
  v = (v | (v << 4)) & 0x030c30c3;
  v = (v | (v << 2)) & 0x09249249;
  return v;
}

#ifndef FSDF_HILBERT
#define FSDF_HILBERT 1
#endif
// 3-D Hilbert index of 10-bit cell coordinates (Skilling's transpose form:
// undo the excess work, Gray-encode, interleave with x most significant).
// Unlike Morton order the curve never jumps: consecutive cells are adjacent.
__device__ __forceinline__ uint32_t hilbert10(const uint32_t* c) {
  uint32_t X[3] = {c[0], c[1], c[2]};
  for (uint32_t Q = 1u << 9; Q > 1; Q >>= 1) {
    const uint32_t P = Q - 1;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (X[i] & Q) {
        X[0] ^= P;
      } else {
        const uint32_t t = (X[0] ^ X[i]) & P;
        X[0] ^= t;
        X[i] ^= t;
      }
    }
  }
  X[1] ^= X[0];
  X[2] ^= X[1];
  uint32_t t = 0;
  for (uint32_t Q = 1u << 9; Q > 1; Q >>= 1)
    if (X[2] & Q) t ^= Q - 1;
#pragma unroll
  for (int i = 0; i < 3; ++i) X[i] ^= t;
  return spread10(X[2]) | (spread10(X[1]) << 1) | (spread10(X[0]) << 2);
}

__global__ __launch_bounds__(kBlock) void curve_key_kernel(const double* __restrict__ pts, int64_t n,
                                                        const double* __restrict__ box, uint32_t* __restrict__ keys,
                                                        int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t q[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double lo = box[j], ext = box[3 + j] - lo;
    const double u = ext > 0 ? (pts[3 * i + j] - lo) / ext : 0.0;
    int c = (int)(u * 1024.0);
    q[j] = (uint32_t)(c < 0 ? 0 : (c > 1023 ? 1023 : c));
  }
#if FSDF_HILBERT
  keys[i] = hilbert10(q);
#else
  keys[i] = spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2);
#endif
  if (idx) idx[i] = (int32_t)i;
}

// composite (30-bit curve key, int31 whole-cloud index) keys and positions for
// the keyed resident order (sort_points_keyed)
__global__ __launch_bounds__(kBlock) void composite_key_kernel(const uint32_t* __restrict__ keys,
                                                            const int64_t* __restrict__ index, int64_t n,
                                                            uint64_t* __restrict__ out, int32_t* __restrict__ pos) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  out[i] = ((uint64_t)(keys[i] & 0x3fffffffu) << 31) | (uint64_t)(index[i] & 0x7fffffff);
  pos[i] = (int32_t)i;
}

// resident i <- source pos[i]: the point (context precision) and its whole-cloud index
template <typename T>
__global__ __launch_bounds__(kBlock) void gather_keyed_kernel(const double* __restrict__ src,
                                                           const int64_t* __restrict__ index, int64_t n,
                                                           const int32_t* __restrict__ pos, T* __restrict__ dst,
                                                           int32_t* __restrict__ perm) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t o = pos[i];
#pragma unroll
  for (int j = 0; j < 3; ++j) dst[3 * i + j] = (T)src[3 * o + j];
  perm[i] = (int32_t)index[o];
}

template <typename T>
__global__ __launch_bounds__(kBlock) void gather_kernel(const double* __restrict__ src, int64_t n,
                                                        const int32_t* __restrict__ order, T* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t o = order[i];
#pragma unroll
  for (int j = 0; j < 3; ++j) dst[3 * i + j] = (T)src[3 * o + j];
}

// regroup_points: a stable counting sort of the resident cloud on each point's
// last nearest surface (prior < 64), in three launches over windows of
// kRegroupWindow points: (1) each window's count per surface, (2) one
// exclusive scan of those counts in surface-major order — the start of every
// (surface, window) run in the regrouped cloud, (3) each window ranks its
// points again and moves them there. Ranks: sub-chunks of 64 points, one per
// wave-iteration in order, a lane's rank among the earlier lanes of its
// surface from ballots over the surface's 6 bits; per surface an exclusive
// scan over the window's sub-chunks in LDS. Stable: the previous (Hilbert)
// order holds within each surface's group.
constexpr int kRegroupWindow = 4096;
constexpr int kRegroupSubs = kRegroupWindow / 64;
constexpr int kRegroupBlock = 256;
constexpr int kRegroupSubsPerWave = kRegroupSubs / (kRegroupBlock / 64);
constexpr int kRegroupScanBlock = 1024;

// this lane's surface (-1: past the cloud) and rank among the earlier lanes
// of its sub-chunk with the same surface; the mask of those lanes
__device__ __forceinline__ int regroup_rank(int pv, bool valid, int& k, uint64_t& eq) {
  const int lane = threadIdx.x & 63;
  k = valid ? (pv & 63) : -1;
  eq = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    const uint64_t m = __ballot(valid && ((k >> b) & 1));
    eq &= (valid && ((k >> b) & 1)) ? m : ~m;
  }
  if (!valid) eq = 0;
  return __builtin_popcountll(eq & ((1ull << lane) - 1));
}

__global__ __launch_bounds__(kRegroupBlock) void regroup_count_kernel(const uint8_t* __restrict__ prior, int64_t n,
                                                                   uint32_t* __restrict__ counts, int nwin) {
  __shared__ uint32_t cnt[64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * kRegroupWindow;
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
  __syncthreads();
  int pv[kRegroupSubsPerWave];  // every load issued before the first ballot
#pragma unroll
  for (int j = 0; j < kRegroupSubsPerWave; ++j) {
    const int64_t i = w0 + 64 * (wave * kRegroupSubsPerWave + j) + lane;
    pv[j] = i < n ? prior[i] : 0;
  }
#pragma unroll
  for (int j = 0; j < kRegroupSubsPerWave; ++j) {
    int k;
    uint64_t eq;
    const int r = regroup_rank(pv[j], w0 + 64 * (wave * kRegroupSubsPerWave + j) + lane < n, k, eq);
    if (k >= 0 && r == 0) atomicAdd(&cnt[k], (uint32_t)__builtin_popcountll(eq));
  }
  __syncthreads();
  if (threadIdx.x < 64) counts[(int64_t)threadIdx.x * nwin + blockIdx.x] = cnt[threadIdx.x];
}

// exclusive prefix sum of counts[0, m) in place (one workgroup): super-tiles
// of 16 tiles x 1,024 entries, all 16 coalesced loads issued at once (one CU
// walking 64-B-strided lines was line-rate bound: 16 us for 16 K entries),
// then per tile in order a wave scan (shuffles) and a scan of the 16 wave
// totals in LDS
constexpr int kRegroupScanPer = 16;
__global__ __launch_bounds__(kRegroupScanBlock) void regroup_scan_kernel(uint32_t* __restrict__ counts, int64_t m) {
  __shared__ uint32_t wsum[2][kRegroupScanBlock / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t carry = 0;
  for (int64_t base = 0; base < m; base += (int64_t)kRegroupScanPer * kRegroupScanBlock) {
    uint32_t v[kRegroupScanPer];
#pragma unroll
    for (int j = 0; j < kRegroupScanPer; ++j) {
      const int64_t i = base + (int64_t)j * kRegroupScanBlock + t;
      v[j] = i < m ? counts[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kRegroupScanPer; ++j) {
      uint32_t x = v[j];  // inclusive wave scan
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(x, off, 64);
        if (lane >= off) x += o;
      }
      uint32_t* ws = wsum[j & 1];  // (alternating: one barrier per tile)
      if (lane == 63) ws[wave] = x;
      __syncthreads();
      uint32_t y = lane < kRegroupScanBlock / 64 ? ws[lane] : 0u;  // every wave scans the 16 totals itself
#pragma unroll
      for (int off = 1; off < kRegroupScanBlock / 64; off <<= 1) {
        const uint32_t o = __shfl_up(y, off, 64);
        if (lane >= off) y += o;
      }
      const uint32_t before = wave ? __shfl(y, wave - 1, 64) : 0u;
      const uint32_t total = __shfl(y, kRegroupScanBlock / 64 - 1, 64);
      const int64_t i = base + (int64_t)j * kRegroupScanBlock + t;
      if (i < m) counts[i] = carry + before + x - v[j];
      carry += total;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kRegroupBlock) void regroup_scatter_kernel(const T* __restrict__ pts,
                                                                     const int32_t* __restrict__ perm,
                                                                     const uint8_t* __restrict__ prior, int64_t n,
                                                                     const uint32_t* __restrict__ start, int nwin,
                                                                     T* __restrict__ dst_pts, int32_t* __restrict__ dst_perm,
                                                                     uint8_t* __restrict__ dst_prior) {
  __shared__ uint32_t cnt[kRegroupSubs][64];  // per sub-chunk, per surface: count, then offset in the window's run
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * kRegroupWindow;
  int key[kRegroupSubsPerWave], rank[kRegroupSubsPerWave];
#pragma unroll
  for (int j = 0; j < kRegroupSubsPerWave; ++j) {  // every load issued before the first ballot
    const int64_t i = w0 + 64 * (wave * kRegroupSubsPerWave + j) + lane;
    key[j] = i < n ? prior[i] : 0;
  }
#pragma unroll
  for (int j = 0; j < kRegroupSubsPerWave; ++j) {
    const int sub = wave * kRegroupSubsPerWave + j;
    uint64_t eq;
    rank[j] = regroup_rank(key[j], w0 + 64 * sub + lane < n, key[j], eq);
    cnt[sub][lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (key[j] >= 0 && rank[j] == 0) cnt[sub][key[j]] = (uint32_t)__builtin_popcountll(eq);
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // per surface: exclusive scan over the sub-chunks, from the run's start
    const int k = threadIdx.x;
    uint32_t run = start[(int64_t)k * nwin + blockIdx.x];
    for (int sub = 0; sub < kRegroupSubs; ++sub) {
      const uint32_t c = cnt[sub][k];
      cnt[sub][k] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRegroupSubsPerWave; ++j) {
    if (key[j] < 0) continue;
    const int sub = wave * kRegroupSubsPerWave + j;
    const int64_t i = w0 + 64 * sub + lane;
    const int64_t d = (int64_t)cnt[sub][key[j]] + rank[j];
#pragma unroll
    for (int c = 0; c < 3; ++c) dst_pts[3 * d + c] = pts[3 * i + c];
    dst_perm[d] = perm[i];
    dst_prior[d] = (uint8_t)key[j];
  }
}

__global__ __launch_bounds__(kBlock) void widen_kernel(const int32_t* __restrict__ src, int64_t n,
                                                       int64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

template <typename P>
hipError_t grow(P** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return hipSuccess;
  if (*p) {
    hipError_t e = hipFree((void*)*p);
    if (e != hipSuccess) return e;
  }
  *p = nullptr;
  *cap = 0;
  hipError_t e = hipMalloc((void**)p, need ? need : 1);
  if (e == hipSuccess) *cap = need;
  return e;
}

// Seed carry-over between frames (the new cloud's first pass seeded by the
// nearest surface the previous cloud's last pass found nearby): a coarse
// voxel grid over a box fixed per context; each previous point writes its k*
// into its voxel (any writer wins: a seed only orders the search, every seed
// gives the same bits), each new point reads its voxel's (0xFF: none).
__device__ __forceinline__ int vox_cell(double x, double y, double z, const VoxBox& b) {
  const double u = (x - b.lo[0]) * b.inv[0], v = (y - b.lo[1]) * b.inv[1], w = (z - b.lo[2]) * b.inv[2];
  if (!(u >= 0.0 && u < kVoxDim && v >= 0.0 && v < kVoxDim && w >= 0.0 && w < kVoxDim)) return -1;
  return ((int)w * kVoxDim + (int)v) * kVoxDim + (int)u;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void vox_scatter_kernel(const T* __restrict__ pts, int64_t n,
                                                             const uint8_t* __restrict__ prior, VoxBox b,
                                                             uint8_t* __restrict__ grid) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint8_t k = prior[i];
  if (k >= 64) return;
  const int c = vox_cell((double)pts[3 * i], (double)pts[3 * i + 1], (double)pts[3 * i + 2], b);
  if (c >= 0) grid[c] = k;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void vox_gather_kernel(const T* __restrict__ pts, int64_t n, VoxBox b,
                                                            const uint8_t* __restrict__ grid,
                                                            uint8_t* __restrict__ prior) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int c = vox_cell((double)pts[3 * i], (double)pts[3 * i + 1], (double)pts[3 * i + 2], b);
  prior[i] = c >= 0 ? grid[c] : (uint8_t)0xFF;
}

}  // namespace

hipError_t vox_scatter(int precision, const void* d_pts, int64_t n, const uint8_t* d_prior, const VoxBox& b,
                       uint8_t* d_grid, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  if (precision == 64)
    hipLaunchKernelGGL(vox_scatter_kernel<double>, dim3(grid), dim3(kBlock), 0, st, (const double*)d_pts, n, d_prior,
                       b, d_grid);
  else
    hipLaunchKernelGGL(vox_scatter_kernel<float>, dim3(grid), dim3(kBlock), 0, st, (const float*)d_pts, n, d_prior, b,
                       d_grid);
  return hipGetLastError();
}

hipError_t vox_gather(int precision, const void* d_pts, int64_t n, const VoxBox& b, const uint8_t* d_grid,
                      uint8_t* d_prior, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  if (precision == 64)
    hipLaunchKernelGGL(vox_gather_kernel<double>, dim3(grid), dim3(kBlock), 0, st, (const double*)d_pts, n, b, d_grid,
                       d_prior);
  else
    hipLaunchKernelGGL(vox_gather_kernel<float>, dim3(grid), dim3(kBlock), 0, st, (const float*)d_pts, n, b, d_grid,
                       d_prior);
  return hipGetLastError();
}

void free_sort_scratch(SortScratch& s) {
  if (s.part) (void)hipFree(s.part);
  if (s.k0) (void)hipFree(s.k0);
  if (s.k1) (void)hipFree(s.k1);
  if (s.i1) (void)hipFree(s.i1);
  if (s.tmp) (void)hipFree(s.tmp);
  if (s.pts) (void)hipFree(s.pts);
  if (s.q0) (void)hipFree(s.q0);
  if (s.q1) (void)hipFree(s.q1);
  s = SortScratch();
}

hipError_t sort_points_spatial(const double* d_src, int64_t n, int precision, void* d_dst, int32_t* d_perm,
                              SortScratch& s, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n > INT32_MAX) return hipErrorInvalidValue;
  const int nb = (int)std::min<int64_t>(kBoxBlocks, (n + kBlock - 1) / kBlock);
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  hipError_t e;
  if ((e = grow(&s.part, &s.part_cap, (size_t)(kBoxBlocks + 1) * 6 * sizeof(double))) != hipSuccess) return e;
  if ((e = grow(&s.k0, &s.k_cap0, (size_t)n * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = grow(&s.k1, &s.k_cap1, (size_t)n * sizeof(uint32_t))) != hipSuccess) return e;
  if ((e = grow(&s.i1, &s.i_cap1, (size_t)n * sizeof(int32_t))) != hipSuccess) return e;
  double* box = s.part + 6 * kBoxBlocks;
  hipLaunchKernelGGL(bbox_partial_kernel, dim3(nb), dim3(kBlock), 0, st, d_src, n, s.part);
  hipLaunchKernelGGL(bbox_final_kernel, dim3(1), dim3(kBlock), 0, st, s.part, nb, box);
  // keys and the identity index go to (k0, d_perm); sorted pairs end in the
  // double buffers' current halves
  hipLaunchKernelGGL(curve_key_kernel, dim3(grid), dim3(kBlock), 0, st, d_src, n, box, s.k0, d_perm);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  rocprim::double_buffer<uint32_t> keys(s.k0, s.k1);
  rocprim::double_buffer<int32_t> vals(d_perm, s.i1);
  size_t need = 0;
  if ((e = rocprim::radix_sort_pairs(nullptr, need, keys, vals, (size_t)n, 0, 30, st)) != hipSuccess) return e;
  if ((e = grow((char**)&s.tmp, &s.tmp_cap, need)) != hipSuccess) return e;
  if ((e = rocprim::radix_sort_pairs(s.tmp, need, keys, vals, (size_t)n, 0, 30, st)) != hipSuccess) return e;
  if (vals.current() != d_perm)
    if ((e = hipMemcpyAsync(d_perm, vals.current(), (size_t)n * sizeof(int32_t), hipMemcpyDeviceToDevice, st)) !=
        hipSuccess)
      return e;
  if (precision == 64)
    hipLaunchKernelGGL(gather_kernel<double>, dim3(grid), dim3(kBlock), 0, st, d_src, n, d_perm, (double*)d_dst);
  else
    hipLaunchKernelGGL(gather_kernel<float>, dim3(grid), dim3(kBlock), 0, st, d_src, n, d_perm, (float*)d_dst);
  return hipGetLastError();
}

hipError_t cloud_box(const double* d_src, int64_t n, SortScratch& s, hipStream_t st, double** d_box) {
  hipError_t e;
  if ((e = grow(&s.part, &s.part_cap, (size_t)(kBoxBlocks + 1) * 6 * sizeof(double))) != hipSuccess) return e;
  double* box = s.part + 6 * kBoxBlocks;
  *d_box = box;
  if (n <= 0) return hipSuccess;  // (the slot only: curve_keys_device fills it from the host)
  const int nb = (int)std::min<int64_t>(kBoxBlocks, (n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(bbox_partial_kernel, dim3(nb), dim3(kBlock), 0, st, d_src, n, s.part);
  hipLaunchKernelGGL(bbox_final_kernel, dim3(1), dim3(kBlock), 0, st, s.part, nb, box);
  return hipGetLastError();
}

hipError_t curve_keys(const double* d_src, int64_t n, const double* d_box, uint32_t* d_keys, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(curve_key_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, d_src, n,
                     d_box, d_keys, (int32_t*)nullptr);
  return hipGetLastError();
}

hipError_t sort_points_keyed(const double* d_src, const uint32_t* d_keys, const int64_t* d_index, int64_t n,
                             int precision, void* d_dst, int32_t* d_perm, SortScratch& s, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n > INT32_MAX) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  hipError_t e;
  if ((e = grow(&s.q0, &s.q_cap0, (size_t)n * sizeof(uint64_t))) != hipSuccess) return e;
  if ((e = grow(&s.q1, &s.q_cap1, (size_t)n * sizeof(uint64_t))) != hipSuccess) return e;
  if ((e = grow(&s.i1, &s.i_cap1, (size_t)n * sizeof(int32_t))) != hipSuccess) return e;
  if ((e = grow(&s.k0, &s.k_cap0, (size_t)n * sizeof(int32_t))) != hipSuccess) return e;
  int32_t* pos0 = (int32_t*)s.k0;
  hipLaunchKernelGGL(composite_key_kernel, dim3(grid), dim3(kBlock), 0, st, d_keys, d_index, n, s.q0, pos0);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  rocprim::double_buffer<uint64_t> keys(s.q0, s.q1);
  rocprim::double_buffer<int32_t> vals(pos0, s.i1);
  size_t need = 0;
  if ((e = rocprim::radix_sort_pairs(nullptr, need, keys, vals, (size_t)n, 0, 61, st)) != hipSuccess) return e;
  if ((e = grow((char**)&s.tmp, &s.tmp_cap, need)) != hipSuccess) return e;
  if ((e = rocprim::radix_sort_pairs(s.tmp, need, keys, vals, (size_t)n, 0, 61, st)) != hipSuccess) return e;
  if (precision == 64)
    hipLaunchKernelGGL(gather_keyed_kernel<double>, dim3(grid), dim3(kBlock), 0, st, d_src, d_index, n, vals.current(),
                       (double*)d_dst, d_perm);
  else
    hipLaunchKernelGGL(gather_keyed_kernel<float>, dim3(grid), dim3(kBlock), 0, st, d_src, d_index, n, vals.current(),
                       (float*)d_dst, d_perm);
  return hipGetLastError();
}

hipError_t regroup_points(void** d_pts, int64_t* pts_cap, int64_t n, int precision, int32_t* d_perm, uint8_t* prior,
                          SortScratch& s, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n > INT32_MAX) return hipErrorInvalidValue;
  const size_t tsz = precision == 64 ? sizeof(double) : sizeof(float);
  const int nwin = (int)((n + kRegroupWindow - 1) / kRegroupWindow);
  hipError_t e;
  if ((e = grow((char**)&s.pts, &s.pts_cap, (size_t)n * 3 * tsz)) != hipSuccess) return e;
  if ((e = grow(&s.k0, &s.k_cap0, (size_t)n * sizeof(uint32_t))) != hipSuccess) return e;  // the permutation
  if ((e = grow(&s.k1, &s.k_cap1, (size_t)n)) != hipSuccess) return e;                     // the priors
  if ((e = grow(&s.i1, &s.i_cap1, (size_t)64 * nwin * sizeof(int32_t))) != hipSuccess) return e;  // run starts
  int32_t* perm2 = (int32_t*)s.k0;
  uint8_t* prior2 = (uint8_t*)s.k1;
  uint32_t* start = (uint32_t*)s.i1;
  hipLaunchKernelGGL(regroup_count_kernel, dim3(nwin), dim3(kRegroupBlock), 0, st, prior, n, start, nwin);
  hipLaunchKernelGGL(regroup_scan_kernel, dim3(1), dim3(kRegroupScanBlock), 0, st, start, (int64_t)64 * nwin);
  if (precision == 64)
    hipLaunchKernelGGL(regroup_scatter_kernel<double>, dim3(nwin), dim3(kRegroupBlock), 0, st, (const double*)*d_pts,
                       d_perm, prior, n, start, nwin, (double*)s.pts, perm2, prior2);
  else
    hipLaunchKernelGGL(regroup_scatter_kernel<float>, dim3(nwin), dim3(kRegroupBlock), 0, st, (const float*)*d_pts,
                       d_perm, prior, n, start, nwin, (float*)s.pts, perm2, prior2);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // the regrouped cloud becomes the resident one (the old buffer the scratch)
  void* old = *d_pts;
  const int64_t old_cap = *pts_cap;
  *d_pts = s.pts;
  *pts_cap = (int64_t)(s.pts_cap / (3 * tsz));
  s.pts = old;
  s.pts_cap = (size_t)old_cap * 3 * tsz;
  if ((e = hipMemcpyAsync(d_perm, perm2, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToDevice, st)) != hipSuccess)
    return e;
  return hipMemcpyAsync(prior, prior2, (size_t)n, hipMemcpyDeviceToDevice, st);
}

hipError_t widen_permutation(const int32_t* d_perm, int64_t n, int64_t* d_out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(widen_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, d_perm, n, d_out);
  return hipGetLastError();
}

}  // namespace fsdf
