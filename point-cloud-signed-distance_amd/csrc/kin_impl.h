// kin_impl.h — the per-body arithmetic of forward kinematics, the surface
// poses and the chain rule, shared by the host loop (kinematics.cpp, capi.hip
// iteration_prepare / fsdf_config_gradient) and the device solver step
// (solver.hip). Every function is one body's (or one surface's) work with a
// fixed operation order, so the host's sequential loop over bodies and the
// device's level-parallel loop produce the same bits (both translation units
// are built with -ffp-contract=off; device sqrt and division are correctly
// rounded). sin/cos are this file's own (kin::sincos) for the same reason: a
// libm on the host and the device library on the GPU may round differently.
//
// Conventions (RigidBodyDynamics as the reference uses it, src/Flash.jl:248,
// src/gradientdescent.jl:19-30): per body b >= 1
//   J   = joint motion: fixed I; revolute I + sin(a) K + (1 - cos(a)) K^2
//         (K = [axis]x, unit axis); quaternion-floating R(q/|q|), t = q[4:7]
//   L   = joint_to_parent · J · body_to_joint
//   T_b = T_parent(b) · L
//   Tb_b = T_parent(b) · joint_to_parent   (the joint frame before its motion)
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define FSDF_HD __host__ __device__ inline
#else
#define FSDF_HD inline
#endif

namespace fsdf {
namespace kin {

// Every helper reads all of its inputs into locals before it writes an
// output: the device compiler cannot prove that an output (often LDS, seen
// through a generic pointer) does not alias an input, and otherwise orders
// every later load after every store — one memory round trip per matrix entry
// (measured: 1.5 us per FK level of M64, 12 us of a 24 us solver step). The
// arithmetic, and so the bits, are unchanged.
FSDF_HD void load(const double* p, double* v, int n) {
  for (int i = 0; i < n; ++i) v[i] = p[i];
}
FSDF_HD void store(double* p, const double* v, int n) {
  for (int i = 0; i < n; ++i) p[i] = v[i];
}

// C = A · B (3x3, row-major, locals), each entry summed in k order
FSDF_HD void mul33(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
// y = A · x + c (locals)
FSDF_HD void mul3(const double* A, const double* x, const double* c, double* y) {
  for (int i = 0; i < 3; ++i) y[i] = (A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2]) + c[i];
}

// ---- sin / cos --------------------------------------------------------------
// The classic minimax kernels on [-pi/4, pi/4] (coefficients of the public
// fdlibm / openlibm polynomials, which Julia's own sin and cos follow) after a
// Cody-Waite reduction by pi/2 in three parts (exact products: each part has
// few enough bits). |x| beyond 2^19 pi/2 is first folded by fmod(x, 2 pi),
// which is exact; joint angles never get there.
FSDF_HD uint64_t bits_of(double v) {
  uint64_t b;
  memcpy(&b, &v, sizeof b);
  return b;
}
FSDF_HD int biased_exp(double v) { return (int)((bits_of(v) >> 52) & 0x7ff); }

// x + y on [-pi/4, pi/4], |y| << |x|; iy = 0: y is exactly 0
FSDF_HD double sin_poly(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double z = x * x, v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
FSDF_HD double cos_poly(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double ax = fabs(x);
  if (ax < 7.450580596923828125e-9) return 1.0;  // 2^-27
  const double z = x * x;
  const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ax < 0.3) return 1.0 - (0.5 * z - (z * r - x * y));
  // 1 - z/2 as (1 - qx) - (z/2 - qx), qx = |x|/4 cut to its high word (so
  // that 1 - qx is exact), 0.28125 above 0.78125
  double qx = 0.28125;
  if (ax <= 0.78125) {
    const uint64_t b = bits_of(ax * 0.25) & 0xFFFFFFFF00000000ull;
    memcpy(&qx, &b, sizeof qx);
  }
  const double hz = 0.5 * z - qx, a = 1.0 - qx;
  return a - (hz - (z * r - x * y));
}
// n = the quadrant, x = y0 + y1 reduced to [-pi/4, pi/4] (about); |x| < 2^19 pi/2
FSDF_HD int rem_pio2(double x, double* y0, double* y1) {
  const double invpio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
  const double pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21;
  const double pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
  const double t = fabs(x);
  const int n = (int)(t * invpio2 + 0.5);
  const double fn = (double)n;
  double r = t - fn * pio2_1;
  double w = fn * pio2_1t;  // first round: good to 85 bits
  double y = r - w;
  const int j = biased_exp(t);
  if (j - biased_exp(y) > 16) {  // cancellation: the second part of pi/2 (118 bits)
    const double tt = r;
    w = fn * pio2_2;
    r = tt - w;
    w = fn * pio2_2t - ((tt - r) - w);
    y = r - w;
    if (j - biased_exp(y) > 49) {  // and the third (151 bits)
      const double t2 = r;
      w = fn * pio2_3;
      r = t2 - w;
      w = fn * pio2_3t - ((t2 - r) - w);
      y = r - w;
    }
  }
  const double lo = (r - y) - w;
  if (x < 0.0) {
    *y0 = -y;
    *y1 = -lo;
    return -n;
  }
  *y0 = y;
  *y1 = lo;
  return n;
}
FSDF_HD void sincos(double x, double* s, double* c) {
  if (fabs(x) <= 7.85398163397448278999e-01) {  // pi/4
    *s = fabs(x) < 7.450580596923828125e-9 ? x : sin_poly(x, 0.0, 0);
    *c = cos_poly(x, 0.0);
    return;
  }
  if (!(fabs(x) < 8.23549136e5)) {  // 2^19 pi/2 (or not finite)
    if (!isfinite(x)) {
      *s = *c = x - x;
      return;
    }
    x = fmod(x, 6.28318530717958623200);  // exact
  }
  double y0, y1;
  const int n = rem_pio2(x, &y0, &y1);
  const double sv = sin_poly(y0, y1, 1), cv = cos_poly(y0, y1);
  switch (n & 3) {
    case 0: *s = sv; *c = cv; break;
    case 1: *s = cv; *c = -sv; break;
    case 2: *s = -sv; *c = -cv; break;
    default: *s = -cv; *c = sv; break;
  }
}

// ---- forward kinematics -----------------------------------------------------
// L = joint_to_parent · J(q) · body_to_joint of body b: LR (3x3), Lt. Returns
// false for a zero quaternion or an unknown kind.
FSDF_HD bool joint_local(int kind, const double* a_, const double* AR_, const double* At_, const double* BR_,
                         const double* Bt_, const double* q_, double* LR_, double* Lt_) {
  const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  double a[3], AR[9], At[3], BR[9], Bt[3], q[7];
  load(a_, a, 3);
  load(AR_, AR, 9);
  load(At_, At, 3);
  load(BR_, BR, 9);
  load(Bt_, Bt, 3);
  if (kind == 2) load(q_, q, 7);  // (constant counts: the copies stay in registers)
  else if (kind == 1) q[0] = q_[0];
  double JR[9], Jt[3] = {0, 0, 0};
  if (kind == 1) {  // revolute
    double s, c;
    sincos(q[0], &s, &c);
    const double c1 = 1.0 - c;
    const double K[9] = {0, -a[2], a[1], a[2], 0, -a[0], -a[1], a[0], 0};
    double KK[9];
    mul33(K, K, KK);
    for (int i = 0; i < 9; ++i) JR[i] = (I[i] + s * K[i]) + c1 * KK[i];
  } else if (kind == 2) {  // quaternion floating: (w, x, y, z, tx, ty, tz)
    const double nrm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (!(nrm > 0)) return false;
    const double w = q[0] / nrm, x = q[1] / nrm, y = q[2] / nrm, z = q[3] / nrm;
    JR[0] = 1 - 2 * (y * y + z * z);
    JR[1] = 2 * (x * y - w * z);
    JR[2] = 2 * (x * z + w * y);
    JR[3] = 2 * (x * y + w * z);
    JR[4] = 1 - 2 * (x * x + z * z);
    JR[5] = 2 * (y * z - w * x);
    JR[6] = 2 * (x * z - w * y);
    JR[7] = 2 * (y * z + w * x);
    JR[8] = 1 - 2 * (x * x + y * y);
    for (int i = 0; i < 3; ++i) Jt[i] = q[4 + i];
  } else if (kind == 0) {  // fixed
    for (int i = 0; i < 9; ++i) JR[i] = I[i];
  } else {
    return false;
  }
  double AJ[9], u[3], LR[9], Lt[3];
  mul33(AR, JR, AJ);
  mul33(AJ, BR, LR);
  mul3(AR, Jt, At, u);  // joint_to_parent applied to the joint's translation
  mul3(AJ, Bt, u, Lt);
  store(LR_, LR, 9);
  store(Lt_, Lt, 3);
  return true;
}

// One output entry of compose (e = 0..8: R, 9..11: t, 12..20: Rb, 21..23: tb)
// — the expression mul33 / mul3 evaluate for it: the device composes a body's
// 24 entries on 24 lanes, the host in a loop, the same bits.
FSDF_HD double compose_entry(int e, const double* Rp, const double* tp, const double* LR, const double* Lt,
                             const double* AR, const double* At) {
  if (e < 9) {
    const int i = e / 3, j = e - 3 * (e / 3);
    return Rp[3 * i] * LR[j] + Rp[3 * i + 1] * LR[3 + j] + Rp[3 * i + 2] * LR[6 + j];
  }
  if (e < 12) {
    const int i = e - 9;
    return (Rp[3 * i] * Lt[0] + Rp[3 * i + 1] * Lt[1] + Rp[3 * i + 2] * Lt[2]) + tp[i];
  }
  if (e < 21) {
    const int i = (e - 12) / 3, j = (e - 12) - 3 * ((e - 12) / 3);
    return Rp[3 * i] * AR[j] + Rp[3 * i + 1] * AR[3 + j] + Rp[3 * i + 2] * AR[6 + j];
  }
  const int i = e - 21;
  return (Rp[3 * i] * At[0] + Rp[3 * i + 1] * At[1] + Rp[3 * i + 2] * At[2]) + tp[i];
}

// T_b = T_p · L and the joint frame Tb_b = T_p · joint_to_parent
FSDF_HD void compose(const double* Rp_, const double* tp_, const double* LR_, const double* Lt_, const double* AR_,
                     const double* At_, double* R_, double* t_, double* Rb_, double* tb_) {
  double Rp[9], tp[3], LR[9], Lt[3], AR[9], At[3];
  load(Rp_, Rp, 9);
  load(tp_, tp, 3);
  load(LR_, LR, 9);
  load(Lt_, Lt, 3);
  load(AR_, AR, 9);
  load(At_, At, 3);
  double v[24];
  for (int e = 0; e < 24; ++e) v[e] = compose_entry(e, Rp, tp, LR, Lt, AR, At);
  store(R_, v, 9);
  store(t_, v + 9, 3);
  store(Rb_, v + 12, 9);
  store(tb_, v + 21, 3);
}

// One entry of a surface's pose T_world_body · T_body_geometry (e = 0..8: R
// row-major, 9..11: t)
FSDF_HD double surface_pose_entry(int e, const double* Rw, const double* tw, const double* FR, const double* Ft) {
  if (e < 9) {
    const int i = e / 3, j = e - 3 * (e / 3);
    return Rw[3 * i] * FR[j] + Rw[3 * i + 1] * FR[3 + j] + Rw[3 * i + 2] * FR[6 + j];
  }
  const int i = e - 9;
  return (Rw[3 * i] * Ft[0] + Rw[3 * i + 1] * Ft[1] + Rw[3 * i + 2] * Ft[2]) + tw[i];
}

// a surface's pose P = [R (3x3) | t]
FSDF_HD void surface_pose(const double* Rw_, const double* tw_, const double* FR_, const double* Ft_, double* P_) {
  double Rw[9], tw[3], FR[9], Ft[3], P[12];
  load(Rw_, Rw, 9);
  load(tw_, tw, 3);
  load(FR_, FR, 9);
  load(Ft_, Ft, 3);
  for (int e = 0; e < 12; ++e) P[e] = surface_pose_entry(e, Rw, tw, FR, Ft);
  store(P_, P, 12);
}

// ---- chain rule -------------------------------------------------------------
// ∂c/∂q of body b's joint from its subtree wrench (F = w[0..2], M = w[3..5],
// about the world origin) and its joint frame (Rb, tb): revolute
// ω = Rb·axis, v = tb × ω, ∂c/∂q = −(ω·M + v·F); quaternion-floating
// (w, x, y, z, t): the four rotation columns through E(q̂) and the
// normalization projection 1/|q| (src/gradientdescent.jl:30), the translation
// columns −(Rb e_j)·F. gq: the joint's entries. Returns false on a zero
// quaternion / unknown kind.
FSDF_HD bool joint_gradient(int kind, const double* a_, const double* R_, const double* o_, const double* q_,
                            const double* wr_, double* gq) {
  if (kind == 0) return true;
  if (kind != 1 && kind != 2) return false;
  double a[3], R[9], o[3], q[7], wr[6];
  load(a_, a, 3);
  load(R_, R, 9);
  load(o_, o, 3);
  if (kind == 2) load(q_, q, 7);
  else q[0] = q_[0];
  load(wr_, wr, 6);
  const double* F = wr;
  const double* M = wr + 3;
  if (kind == 1) {
    double w[3], v[3];
    for (int i = 0; i < 3; ++i) w[i] = R[3 * i] * a[0] + R[3 * i + 1] * a[1] + R[3 * i + 2] * a[2];
    v[0] = o[1] * w[2] - o[2] * w[1];
    v[1] = o[2] * w[0] - o[0] * w[2];
    v[2] = o[0] * w[1] - o[1] * w[0];
    gq[0] = -((w[0] * M[0] + w[1] * M[1] + w[2] * M[2]) + (v[0] * F[0] + v[1] * F[1] + v[2] * F[2]));
    return true;
  }
  const double nrm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (!(nrm > 0)) return false;
  const double W = q[0] / nrm, X = q[1] / nrm, Y = q[2] / nrm, Z = q[3] / nrm;
  const double E[3][4] = {{-X, W, -Z, Y}, {-Y, Z, W, -X}, {-Z, -Y, X, W}};
  double org[3];  // world origin of the frame after the joint
  for (int i = 0; i < 3; ++i) org[i] = (R[3 * i] * q[4] + R[3 * i + 1] * q[5] + R[3 * i + 2] * q[6]) + o[i];
  double g[7];
  for (int j = 0; j < 4; ++j) {
    double w[3], v[3];
    for (int i = 0; i < 3; ++i)
      w[i] = R[3 * i] * (2.0 * E[0][j]) + R[3 * i + 1] * (2.0 * E[1][j]) + R[3 * i + 2] * (2.0 * E[2][j]);
    v[0] = org[1] * w[2] - org[2] * w[1];
    v[1] = org[2] * w[0] - org[0] * w[2];
    v[2] = org[0] * w[1] - org[1] * w[0];
    g[j] = -((w[0] * M[0] + w[1] * M[1] + w[2] * M[2]) + (v[0] * F[0] + v[1] * F[1] + v[2] * F[2])) / nrm;
  }
  for (int j = 0; j < 3; ++j) g[4 + j] = -(R[j] * F[0] + R[3 + j] * F[1] + R[6 + j] * F[2]);
  store(gq, g, 7);
  return true;
}

// NaiveSolver's component step (flash/tracking.py): clamp(-rate g, ±max_step)
FSDF_HD double clipped_step(double rate, double g, double max_step) {
  const double s = -rate * g;
  const double lo = s < -max_step ? -max_step : s;  // std::max(s, -max_step)
  return max_step < lo ? max_step : lo;             // std::min(lo, max_step)
}

}  // namespace kin
}  // namespace fsdf
