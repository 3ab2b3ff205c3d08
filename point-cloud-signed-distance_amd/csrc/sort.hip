// sort.hip — spatial ordering of the resident cloud (fsdf_opts.sort_points).
//
// The pass kernel evaluates a hull for a whole wave when any of its 64 lanes
// needs it, so its cost follows the spatial coherence of consecutive points.
// Depth sensors deliver raster order (src/depthdata.jl:19-30,
// src/depthsensors.jl:99-113), which is already coherent; an arbitrary order
// is made coherent here once per frame: 30-bit Hilbert keys (10 bits per axis)
// over the cloud's bounding box, a device radix sort (rocPRIM), and a gather.
// The permutation is kept so per-point outputs still land in the caller's
// order. Hilbert rather than Morton order: a Morton curve jumps at every
// octree boundary, so some 64-point chunks straddle two distant regions and
// need the hulls of both; on the bench cloud the pass is 8.5 % faster
// (0.144 -> 0.132 ms; -DFSDF_HILBERT=0 restores Morton keys).

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
                                                        const double* __restrict__ part, int nparts,
                                                        uint32_t* __restrict__ keys, int64_t* __restrict__ idx) {
  __shared__ double box[6];
  if (threadIdx.x < 6) {
    const bool is_lo = threadIdx.x < 3;
    double b = is_lo ? __builtin_huge_val() : -__builtin_huge_val();
    for (int p = 0; p < nparts; ++p) {
      const double v = part[6 * p + threadIdx.x];
      b = is_lo ? fmin(b, v) : fmax(b, v);
    }
    box[threadIdx.x] = b;
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t q[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double ext = box[3 + j] - box[j];
    const double u = ext > 0 ? (pts[3 * i + j] - box[j]) / ext : 0.0;
    int c = (int)(u * 1024.0);
    q[j] = (uint32_t)(c < 0 ? 0 : (c > 1023 ? 1023 : c));
  }
#if FSDF_HILBERT
  keys[i] = hilbert10(q);
#else
  keys[i] = spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2);
#endif
  idx[i] = i;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void gather_kernel(const double* __restrict__ src, int64_t n,
                                                        const int64_t* __restrict__ order, T* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t o = order[i];
#pragma unroll
  for (int j = 0; j < 3; ++j) dst[3 * i + j] = (T)src[3 * o + j];
}

}  // namespace

hipError_t sort_points_spatial(const double* d_src, int64_t n, int precision, void* d_dst, int64_t* d_perm,
                              hipStream_t s) {
  if (n <= 0) return hipSuccess;
  double* part = nullptr;
  uint32_t *k0 = nullptr, *k1 = nullptr;
  int64_t* i0 = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  hipError_t e = hipSuccess;
  const int nb = (int)std::min<int64_t>(kBoxBlocks, (n + kBlock - 1) / kBlock);
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
#define FSDF_TRY(x) \
  do {              \
    e = (x);        \
    if (e != hipSuccess) goto done; \
  } while (0)
  FSDF_TRY(hipMalloc(&part, (size_t)nb * 6 * sizeof(double)));
  FSDF_TRY(hipMalloc(&k0, (size_t)n * sizeof(uint32_t)));
  FSDF_TRY(hipMalloc(&k1, (size_t)n * sizeof(uint32_t)));
  FSDF_TRY(hipMalloc(&i0, (size_t)n * sizeof(int64_t)));
  hipLaunchKernelGGL(bbox_partial_kernel, dim3(nb), dim3(kBlock), 0, s, d_src, n, part);
  FSDF_TRY(hipGetLastError());
  hipLaunchKernelGGL(curve_key_kernel, dim3(grid), dim3(kBlock), 0, s, d_src, n, part, nb, k0, i0);
  FSDF_TRY(hipGetLastError());
  FSDF_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, k1, i0, d_perm, (size_t)n, 0, 30, s));
  FSDF_TRY(hipMalloc(&tmp, tmp_bytes));
  FSDF_TRY(rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, i0, d_perm, (size_t)n, 0, 30, s));
  if (precision == 64)
    hipLaunchKernelGGL(gather_kernel<double>, dim3(grid), dim3(kBlock), 0, s, d_src, n, d_perm, (double*)d_dst);
  else
    hipLaunchKernelGGL(gather_kernel<float>, dim3(grid), dim3(kBlock), 0, s, d_src, n, d_perm, (float*)d_dst);
  FSDF_TRY(hipGetLastError());
  FSDF_TRY(hipStreamSynchronize(s));
#undef FSDF_TRY
done:
  if (part) (void)hipFree(part);
  if (k0) (void)hipFree(k0);
  if (k1) (void)hipFree(k1);
  if (i0) (void)hipFree(i0);
  if (tmp) (void)hipFree(tmp);
  return e;
}

}  // namespace fsdf
