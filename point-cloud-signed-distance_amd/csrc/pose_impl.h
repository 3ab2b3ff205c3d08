// pose_impl.h — the pose of the local model for one pass: world-frame planes,
// screening pairs, stage images, vertices, bounding spheres / boxes and
// certificate scales of every hull from the surfaces' 3x4 poses. One function
// per work item, shared by the pose kernels (sdf_kernels.hip) and the device
// solver step (solver.hip), which poses the next pass's model itself.
#pragma once

#include <hip/hip_runtime.h>

#include "fsdf_internal.h"

namespace fsdf {

// ---------------------------------------------------------------------------
// Pose kernel: local model + poses -> world-frame planes and vertices.
// One thread per face, one per vertex, then one wave per hull (sphere + scale).
// ---------------------------------------------------------------------------
typedef int I4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void xf_point(const double* P, const double* v, double* o) {
  // o = R v + t, R row-major P[0..8], t = P[9..11]
  o[0] = __builtin_fma(P[0], v[0], __builtin_fma(P[1], v[1], __builtin_fma(P[2], v[2], P[9])));
  o[1] = __builtin_fma(P[3], v[0], __builtin_fma(P[4], v[1], __builtin_fma(P[5], v[2], P[10])));
  o[2] = __builtin_fma(P[6], v[0], __builtin_fma(P[7], v[1], __builtin_fma(P[8], v[2], P[11])));
}
__device__ __forceinline__ void rot_vec(const double* P, const double* v, double* o) {
  o[0] = __builtin_fma(P[0], v[0], __builtin_fma(P[1], v[1], P[2] * v[2]));
  o[1] = __builtin_fma(P[3], v[0], __builtin_fma(P[4], v[1], P[5] * v[2]));
  o[2] = __builtin_fma(P[6], v[0], __builtin_fma(P[7], v[1], P[8] * v[2]));
}
// One work item `tid` of the pose: items [0, F) a face, [F, F+V) a vertex,
// then (from the next multiple of 64) one wave per hull — the whole wave's
// items in that range (its lanes are 64 consecutive items).
template <typename T>
__device__ __forceinline__ void pose_item(const LocalModel& lm, const double* __restrict__ poses,
                                          T* __restrict__ planes_w, float* __restrict__ spheres_w,
                                          T* __restrict__ verts_w, T* __restrict__ hscale_w,
                                          float* __restrict__ screen_w, I4* __restrict__ image_w, int tid) {
  const int fv = lm.F + lm.V, fv_pad = (fv + 63) & ~63;
  if (tid >= fv && tid < fv_pad) return;  // padding: hull waves start wave-aligned
  if (tid >= fv_pad) tid -= fv_pad - fv;
  if (tid < lm.F) {
    const int f = tid;
    const I4 meta = ((const I4*)lm.item_meta)[f];
    const int k = meta[0] & 0xffff;
    double P[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) P[i] = poses[12 * k + i];
    const double* pl = lm.planes_l + 4 * f;
    double n[3] = {pl[0], pl[1], pl[2]};
    double nw[3];
    rot_vec(P, n, nw);
    // d_w = d + n_w · t
    const double dw = __builtin_fma(nw[0], P[9], __builtin_fma(nw[1], P[10], __builtin_fma(nw[2], P[11], pl[3])));
    T* pw = planes_w + 4 * f;
    pw[0] = (T)nw[0]; pw[1] = (T)nw[1]; pw[2] = (T)nw[2]; pw[3] = (T)dw;
    if (screen_w) {
      // fp32 screening copy, centred on the hull's f32 sphere centre c (the
      // same bits the sphere thread below stores): d' = d - n·c
      const int h = meta[1], fo = meta[2];
      const int j = f - fo, nf = meta[0] >> 16;
      double cw[3];
      xf_point(P, lm.sphere_l + 4 * h, cw);
      const double c0 = (double)(float)cw[0], c1 = (double)(float)cw[1], c2 = (double)(float)cw[2];
      const double dc = dw - __builtin_fma(nw[0], c0, __builtin_fma(nw[1], c1, nw[2] * c2));
      float* pair = screen_w + 4 * (fo + h + (j & ~1));
      // an exact duplicate of an earlier face's plane (face row word 3) is
      // screened out: h = -1e30, never a maximum nor a near-tie
      const bool dup = lm.face_rows[4 * f + 3] != 0;
      const float v[4] = {dup ? 0.0f : (float)nw[0], dup ? 0.0f : (float)nw[1], dup ? 0.0f : (float)nw[2],
                          dup ? -1e30f : (float)(-dc)};
#pragma unroll
      for (int c = 0; c < 4; ++c) pair[2 * c + (j & 1)] = v[c];
      if ((nf & 1) && j == nf - 1)  // odd count: the last pair repeats its face
#pragma unroll
        for (int c = 0; c < 4; ++c) pair[2 * c + 1] = v[c];
      if (sizeof(T) == 8 && image_w) {  // the hull's stage image: same pair words, then the fp64 plane
        I4* img = image_w + 4 * fo + h + 2 * meta[3];
        float* ip = (float*)(img + (j & ~1));
#pragma unroll
        for (int c = 0; c < 4; ++c) ip[2 * c + (j & 1)] = v[c];
        if ((nf & 1) && j == nf - 1)
#pragma unroll
          for (int c = 0; c < 4; ++c) ip[2 * c + 1] = v[c];
        double* q = (double*)(img + nf + 1 + 2 * j);
        q[0] = nw[0]; q[1] = nw[1]; q[2] = nw[2]; q[3] = dw;
      }
    }
  } else if (tid < lm.F + lm.V) {
    const int v = tid - lm.F;
    const I4 meta = ((const I4*)lm.item_meta)[tid];
    const double* P = poses + 12 * (meta[0] & 0xffff);
    double w[3];
    xf_point(P, lm.verts_l + 3 * v, w);
    T* o = verts_w + 4 * v;
    o[0] = (T)w[0]; o[1] = (T)w[1]; o[2] = (T)w[2]; o[3] = (T)0;
    if (sizeof(T) == 8 && image_w) {
      const int h = meta[1], nf = meta[0] >> 16;
      double* q = (double*)(image_w + 4 * meta[2] + h + 2 * meta[3] + 3 * nf + 1 + 2 * (v - meta[3]));
      q[0] = w[0]; q[1] = w[1]; q[2] = w[2]; q[3] = 0.0;
    }
  } else if (tid < lm.F + lm.V + 64 * lm.K) {
    // one wave per hull (the wave is entirely inside this range: F + V is
    // padded to a multiple of 64 by the launcher): sphere + certificate scale
    const int r = tid - lm.F - lm.V;
    const int k = r >> 6, lane = r & 63;
    const double* P = poses + 12 * lm.hull_surface[k];
    T sc = (T)0;
    for (int v = lm.vert_off[k] + lane; v < lm.vert_off[k + 1]; v += 64) {
      double w[3];
      xf_point(P, lm.verts_l + 3 * v, w);
      const T l1 = (T)fabs(w[0]) + (T)fabs(w[1]) + (T)fabs(w[2]);
      sc = l1 > sc ? l1 : sc;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const T o = __shfl_xor(sc, off, 64);
      sc = o > sc ? o : sc;
    }
    if (lane == 0) {
      double cw[3];
      xf_point(P, lm.sphere_l + 4 * k, cw);
      float* bw = spheres_w + kBoundFloats * k;
      bw[0] = (float)cw[0];
      bw[1] = (float)cw[1];
      bw[2] = (float)cw[2];
      // radius and half extents were rounded up to float on the host (exact-safe)
      bw[3] = (float)lm.sphere_l[4 * k + 3];
      // oriented box: body axis i is column i of R
      const double* B = lm.box_l + 8 * k;
      double cb[3];
      xf_point(P, B, cb);
      bw[4] = (float)cb[0];
      bw[5] = (float)cb[1];
      bw[6] = (float)cb[2];
      bw[7] = 0.0f;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        bw[8 + 4 * i + 0] = (float)P[i];
        bw[8 + 4 * i + 1] = (float)P[3 + i];
        bw[8 + 4 * i + 2] = (float)P[6 + i];
        bw[8 + 4 * i + 3] = (float)B[4 + i];
      }
      hscale_w[k] = sc;
    }
  }
}


// the pose's work items: faces and vertices (padded to whole waves), then one wave per hull
__host__ __device__ inline int pose_items(const LocalModel& lm) { return ((lm.F + lm.V + 63) & ~63) + 64 * lm.K; }

}  // namespace fsdf
