// kinematics.cpp — host forward kinematics of the mechanism tree (no device).
//
// transform_to_root of every body, the poses the residual pass consumes
// (src/Flash.jl:248, RigidBodyDynamics.transform_to_root). The Python host
// (flash/mechanism.py body_transform_arrays) batched this per tree level in
// numpy, ~0.2 ms for M64's 64 bodies — more than the GPU pass it feeds; here it
// is one loop over the bodies in topological order (parent[b] < b).
//
// Per body b >= 1 (same factors as the numpy path):
//   J   = joint motion: fixed I; revolute I + sin(a) K + (1 - cos(a)) K^2
//         (K = [axis]x, unit axis); quaternion-floating R(q/|q|), t = q[4:7]
//   L   = joint_to_parent · J · body_to_joint
//   T_b = T_parent(b) · L
//   Tb_b = T_parent(b) · joint_to_parent   (the joint frame before its motion)

#include <math.h>
#include <stdint.h>

#include "flashsdf.h"

namespace {

// C = A · B (3x3, row-major), each entry summed in k order
inline void mul33(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
// y = A · x + c
inline void mul3(const double* A, const double* x, const double* c, double* y) {
  for (int i = 0; i < 3; ++i) y[i] = (A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2]) + c[i];
}

}  // namespace

extern "C" int fsdf_tree_transforms(int32_t nb, const int32_t* parent, const int32_t* kind, const int32_t* qoff,
                                    const double* axis, const double* AR, const double* At, const double* BR,
                                    const double* Bt, const double* q, double* R, double* t, double* Rb,
                                    double* tb) {
  if (nb < 1 || !parent || !kind || !qoff || !axis || !AR || !At || !BR || !Bt || !q || !R || !t || !Rb || !tb)
    return FSDF_ERR_ARG;
  static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  for (int i = 0; i < 9; ++i) R[i] = Rb[i] = I[i];
  for (int i = 0; i < 3; ++i) t[i] = tb[i] = 0.0;
  for (int b = 1; b < nb; ++b) {
    const int p = parent[b];
    if (p < 0 || p >= b) return FSDF_ERR_ARG;  // topological order required
    double JR[9], Jt[3] = {0, 0, 0};
    if (kind[b] == 1) {  // revolute
      const double* a = axis + 3 * b;
      const double ang = q[qoff[b]], s = sin(ang), c1 = 1.0 - cos(ang);
      const double K[9] = {0, -a[2], a[1], a[2], 0, -a[0], -a[1], a[0], 0};
      double KK[9];
      mul33(K, K, KK);
      for (int i = 0; i < 9; ++i) JR[i] = (I[i] + s * K[i]) + c1 * KK[i];
    } else if (kind[b] == 2) {  // quaternion floating: (w, x, y, z, tx, ty, tz)
      const double* qq = q + qoff[b];
      const double nrm = sqrt(qq[0] * qq[0] + qq[1] * qq[1] + qq[2] * qq[2] + qq[3] * qq[3]);
      if (!(nrm > 0)) return FSDF_ERR_ARG;
      const double w = qq[0] / nrm, x = qq[1] / nrm, y = qq[2] / nrm, z = qq[3] / nrm;
      const double M[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                           2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                           2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)};
      for (int i = 0; i < 9; ++i) JR[i] = M[i];
      for (int i = 0; i < 3; ++i) Jt[i] = qq[4 + i];
    } else if (kind[b] == 0) {  // fixed
      for (int i = 0; i < 9; ++i) JR[i] = I[i];
    } else {
      return FSDF_ERR_ARG;
    }
    double AJ[9], LR[9], Lt[3], u[3], v[3];
    mul33(AR + 9 * b, JR, AJ);
    mul33(AJ, BR + 9 * b, LR);
    mul3(AR + 9 * b, Jt, At + 3 * b, u);  // joint_to_parent applied to the joint's translation
    mul3(AJ, Bt + 3 * b, u, Lt);
    const double* Rp = R + 9 * p;
    mul33(Rp, LR, R + 9 * b);
    mul3(Rp, Lt, t + 3 * p, t + 3 * b);
    mul33(Rp, AR + 9 * b, Rb + 9 * b);
    mul3(Rp, At + 3 * b, t + 3 * p, v);
    for (int i = 0; i < 3; ++i) tb[3 * b + i] = v[i];
  }
  return FSDF_OK;
}

// ∂c/∂q from per-surface wrenches (the accumulator's hull rows) and optional
// extra per-body wrenches (the RBF chain's), the chain rule of
// flash/mechanism.py config_gradient: body wrenches summed over each subtree
// (children before parents: reverse topological order), then per joint with
// the world motion subspace of its frame before the motion (Rb, tb of
// fsdf_tree_transforms): revolute ω = Rb·axis, v = tb × ω, ∂c/∂q = −(ω·M + v·F);
// quaternion-floating (w, x, y, z, t): the four rotation columns through
// E(q̂) and the normalization projection 1/|q| (src/gradientdescent.jl:30), the
// translation columns −(Rb e_j)·F. F, M are about the world origin.
extern "C" int fsdf_config_gradient(int32_t nb, const int32_t* parent, const int32_t* kind, const int32_t* qoff,
                                    const double* axis, const double* Rb, const double* tb, const double* q,
                                    int32_t nsurf, const int32_t* surface_body, const double* surface_wrench,
                                    const double* body_wrench, double* work, double* gq) {
  if (nb < 1 || !parent || !kind || !qoff || !axis || !Rb || !tb || !q || !work || !gq || nsurf < 0 ||
      (nsurf > 0 && (!surface_body || !surface_wrench)))
    return FSDF_ERR_ARG;
  double* sub = work;  // [nb][6]
  for (int i = 0; i < 6 * nb; ++i) sub[i] = body_wrench ? body_wrench[i] : 0.0;
  for (int k = 0; k < nsurf; ++k) {
    const int b = surface_body[k];
    if (b < 0) continue;  // surface without a rigid body wrench (RBF skins: body_wrench)
    if (b >= nb) return FSDF_ERR_ARG;
    for (int j = 0; j < 6; ++j) sub[6 * b + j] += surface_wrench[6 * k + j];
  }
  for (int b = nb - 1; b >= 1; --b) {
    const int p = parent[b];
    if (p < 0 || p >= b) return FSDF_ERR_ARG;
    for (int j = 0; j < 6; ++j) sub[6 * p + j] += sub[6 * b + j];
  }
  for (int b = 1; b < nb; ++b) {
    const double* F = sub + 6 * b;
    const double* M = F + 3;
    const double* R = Rb + 9 * b;
    const double* o = tb + 3 * b;
    if (kind[b] == 1) {
      const double* a = axis + 3 * b;
      double w[3], v[3];
      for (int i = 0; i < 3; ++i) w[i] = R[3 * i] * a[0] + R[3 * i + 1] * a[1] + R[3 * i + 2] * a[2];
      v[0] = o[1] * w[2] - o[2] * w[1];
      v[1] = o[2] * w[0] - o[0] * w[2];
      v[2] = o[0] * w[1] - o[1] * w[0];
      gq[qoff[b]] = -((w[0] * M[0] + w[1] * M[1] + w[2] * M[2]) + (v[0] * F[0] + v[1] * F[1] + v[2] * F[2]));
    } else if (kind[b] == 2) {
      const double* qq = q + qoff[b];
      const double nrm = sqrt(qq[0] * qq[0] + qq[1] * qq[1] + qq[2] * qq[2] + qq[3] * qq[3]);
      if (!(nrm > 0)) return FSDF_ERR_ARG;
      const double W = qq[0] / nrm, X = qq[1] / nrm, Y = qq[2] / nrm, Z = qq[3] / nrm;
      const double E[3][4] = {{-X, W, -Z, Y}, {-Y, Z, W, -X}, {-Z, -Y, X, W}};
      double org[3];  // world origin of the frame after the joint
      for (int i = 0; i < 3; ++i) org[i] = (R[3 * i] * qq[4] + R[3 * i + 1] * qq[5] + R[3 * i + 2] * qq[6]) + o[i];
      for (int j = 0; j < 4; ++j) {
        double w[3], v[3];
        for (int i = 0; i < 3; ++i)
          w[i] = R[3 * i] * (2.0 * E[0][j]) + R[3 * i + 1] * (2.0 * E[1][j]) + R[3 * i + 2] * (2.0 * E[2][j]);
        v[0] = org[1] * w[2] - org[2] * w[1];
        v[1] = org[2] * w[0] - org[0] * w[2];
        v[2] = org[0] * w[1] - org[1] * w[0];
        gq[qoff[b] + j] =
            -((w[0] * M[0] + w[1] * M[1] + w[2] * M[2]) + (v[0] * F[0] + v[1] * F[1] + v[2] * F[2])) / nrm;
      }
      for (int j = 0; j < 3; ++j) gq[qoff[b] + 4 + j] = -(R[j] * F[0] + R[3 + j] * F[1] + R[6 + j] * F[2]);
    } else if (kind[b] != 0) {
      return FSDF_ERR_ARG;
    }
  }
  return FSDF_OK;
}
