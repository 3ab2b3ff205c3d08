// kinematics.cpp — host forward kinematics of the mechanism tree (no device).
//
// transform_to_root of every body, the poses the residual pass consumes
// (src/Flash.jl:248, RigidBodyDynamics.transform_to_root). The Python host
// (flash/mechanism.py body_transform_arrays) batched this per tree level in
// numpy, ~0.2 ms for M64's 64 bodies — more than the GPU pass it feeds; here it
// is one loop over the bodies in topological order (parent[b] < b).
//
// The per-body arithmetic (joint motion, composition, chain rule) is
// kin_impl.h's, shared with the device solver step (solver.hip) so that the
// host and device iterations agree bit for bit.

#include <math.h>
#include <stdint.h>

#include "flashsdf.h"
#include "kin_impl.h"

using namespace fsdf::kin;

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
    double LR[9], Lt[3];
    if (!joint_local(kind[b], axis + 3 * b, AR + 9 * b, At + 3 * b, BR + 9 * b, Bt + 3 * b,
                     kind[b] ? q + qoff[b] : q, LR, Lt))
      return FSDF_ERR_ARG;
    compose(R + 9 * p, t + 3 * p, LR, Lt, AR + 9 * b, At + 3 * b, R + 9 * b, t + 3 * b, Rb + 9 * b, tb + 3 * b);
  }
  return FSDF_OK;
}

// ∂c/∂q from per-surface wrenches (the accumulator's hull rows) and optional
// extra per-body wrenches (the RBF chain's), the chain rule of
// flash/mechanism.py config_gradient: body wrenches summed over each subtree
// (children before parents: reverse topological order), then per joint with
// the world motion subspace of its frame before the motion (Rb, tb of
// fsdf_tree_transforms; kin_impl.h joint_gradient). F, M are about the world
// origin. The device solver step (solver.hip) adds in the same order.
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
    if (!joint_gradient(kind[b], axis + 3 * b, Rb + 9 * b, tb + 3 * b, kind[b] ? q + qoff[b] : q, sub + 6 * b,
                        kind[b] ? gq + qoff[b] : nullptr))
      return FSDF_ERR_ARG;
  }
  return FSDF_OK;
}
