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
static inline void cross3(const double* a, const double* b, double* o) {
  o[0] = fma(a[1], b[2], -(a[2] * b[1]));
  o[1] = fma(a[2], b[0], -(a[0] * b[2]));
  o[2] = fma(a[0], b[1], -(a[1] * b[0]));
}
static inline double dot3(const double* a, const double* b) { return fma(a[0], b[0], fma(a[1], b[1], a[2] * b[2])); }

/* World-frame planes, per-face records, vertices and certificate scales for
 * every hull (src/Flash.jl:248: the surface pose is transform_to_root of the
 * geometry frame). Same formulas as pose_kernel. */
void oracle_pose_model(int32_t F, int32_t V, int32_t K, const double* verts_l, const int32_t* faces,
                       const double* planes_l, const int32_t* face_hull, const int32_t* vert_hull,
                       const int32_t* vert_off, const double* poses, double* planes_w, double* facex_w,
                       double* verts_w, double* hscale) {
  for (int f = 0; f < F; ++f) {
    const double* P = poses + 12 * face_hull[f];
    const double* pl = planes_l + 4 * f;
    double nw[3];
    rot_vec(P, pl, nw);
    const double dw = fma(nw[0], P[9], fma(nw[1], P[10], fma(nw[2], P[11], pl[3])));
    double a[3], b[3], c[3];
    xf_point(P, verts_l + 3 * faces[3 * f + 0], a);
    xf_point(P, verts_l + 3 * faces[3 * f + 1], b);
    xf_point(P, verts_l + 3 * faces[3 * f + 2], c);
    const double e0[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    const double e1[3] = {c[0] - b[0], c[1] - b[1], c[2] - b[2]};
    const double e2[3] = {a[0] - c[0], a[1] - c[1], a[2] - c[2]};
    double m0[3], m1[3], m2[3];
    cross3(nw, e0, m0);
    cross3(nw, e1, m1);
    cross3(nw, e2, m2);
    double* pw = planes_w + 4 * f;
    pw[0] = nw[0]; pw[1] = nw[1]; pw[2] = nw[2]; pw[3] = dw;
    double* fx = facex_w + FX * f;
    fx[0] = m0[0]; fx[1] = m0[1]; fx[2] = m0[2]; fx[3] = dot3(m0, a);
    fx[4] = m1[0]; fx[5] = m1[1]; fx[6] = m1[2]; fx[7] = dot3(m1, b);
    fx[8] = m2[0]; fx[9] = m2[1]; fx[10] = m2[2]; fx[11] = dot3(m2, c);
    fx[12] = a[0]; fx[13] = a[1]; fx[14] = a[2];
    fx[15] = b[0]; fx[16] = b[1]; fx[17] = b[2];
    fx[18] = c[0]; fx[19] = c[1]; fx[20] = c[2];
    fx[21] = 0; fx[22] = 0; fx[23] = 0;
  }
  for (int v = 0; v < V; ++v) {
    double* o = verts_w + 4 * v;
    xf_point(poses + 12 * vert_hull[v], verts_l + 3 * v, o);
    o[3] = 0;
  }
  for (int k = 0; k < K; ++k) {
    double sc = 0;
    for (int v = vert_off[k]; v < vert_off[k + 1]; ++v) {
      double w[3];
      xf_point(poses + 12 * k, verts_l + 3 * v, w);
      const double l1 = fabs(w[0]) + fabs(w[1]) + fabs(w[2]);
      sc = l1 > sc ? l1 : sc;
    }
    hscale[k] = sc;
  }
}

/* The posed model as the kernel sees it. Surfaces (the k* index space) are
 * hulls or RBF skins: surf_index[k] = hull index (>= 0) or -(rbf index) - 1. */
typedef struct {
  int32_t K; /* hulls */
  const int32_t* face_off;
  const int32_t* vert_off;
  const int32_t* nbr;
  const double* planes_w;
  const double* facex_w;
  const double* verts_w;
  const double* hscale;
  int32_t S; /* surfaces */
  const int32_t* surf_index;
  const int32_t* rbf_row_off; /* [R+1] rows (n centres + 1 polynomial row) */
  const int32_t* rbf_acc_off; /* [R+1] offsets in the RBF accumulator block */
  const double* rbf_rows;     /* [rows][4]: (c, w) ... then (a, b) */
  const int32_t* faces;       /* [F][3] global vertex indices (CCW from outside) */
} oracle_posed;

/* RBF interpolating skin (src/Flash.jl:207-213, SpatialFields XCubed + affine):
 * f(x) = Σ w_i |x-c_i|^3 + a + b·x, s = f/|∇f|, ∇s = ∇f/|∇f| − f H∇f/|∇f|^3.
 * F = {f, gx, gy, gz, hxx, hyy, hzz, hxy, hxz, hyz}; same order as the kernel. */
static void rbf_field(const double* rows, int nc, const double* p, double* F) {
  const double* poly = rows + 4 * nc;
  F[0] = fma(poly[1], p[0], fma(poly[2], p[1], fma(poly[3], p[2], poly[0])));
  F[1] = poly[1]; F[2] = poly[2]; F[3] = poly[3];
  for (int j = 4; j < 10; ++j) F[j] = 0.0;
  for (int i = 0; i < nc; ++i) {
    const double* c = rows + 4 * i;
    const double dx = p[0] - c[0], dy = p[1] - c[1], dz = p[2] - c[2];
    const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
    const double r = sqrt(r2);
    const double wr = c[3] * r;
    F[0] = fma(wr, r2, F[0]);
    const double t3 = 3.0 * wr;
    F[1] = fma(t3, dx, F[1]); F[2] = fma(t3, dy, F[2]); F[3] = fma(t3, dz, F[3]);
    const double hq = r2 > 0 ? (3.0 * c[3]) / r : 0.0;
    F[4] = fma(hq * dx, dx, F[4] + t3);
    F[5] = fma(hq * dy, dy, F[5] + t3);
    F[6] = fma(hq * dz, dz, F[6] + t3);
    F[7] = fma(hq * dx, dy, F[7]);
    F[8] = fma(hq * dx, dz, F[8]);
    F[9] = fma(hq * dy, dz, F[9]);
  }
}

static void rbf_skin_from_field(const double* F, double* s, double* g, double* c, double* invG) {
  const double G2 = fma(F[1], F[1], fma(F[2], F[2], F[3] * F[3]));
  const double G = sqrt(G2);
  *s = F[0] / G;
  *invG = 1.0 / G;
  *c = F[0] / (G2 * G);
  const double hgx = fma(F[4], F[1], fma(F[7], F[2], F[8] * F[3]));
  const double hgy = fma(F[7], F[1], fma(F[5], F[2], F[9] * F[3]));
  const double hgz = fma(F[8], F[1], fma(F[9], F[2], F[6] * F[3]));
  g[0] = fma(-*c, hgx, F[1] * *invG);
  g[1] = fma(-*c, hgy, F[2] * *invG);
  g[2] = fma(-*c, hgz, F[3] * *invG);
}

void oracle_rbf_skin(const double* rows, int32_t nc, const double* p, double* s, double* g) {
  double F[10], c, invG;
  rbf_field(rows, nc, p, F);
  rbf_skin_from_field(F, s, g, &c, &invG);
}

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

/* Closest point on triangle v = (a, b, c) to p, Voronoi-region walk. *reg:
 * 0, 1, 2 vertex a, b, c; 3, 4, 5 edge a->b, b->c, c->a; 6 interior. */
static void closest_on_triangle(const double* p, const double* v, double* q, int* reg) {
  const double ax = v[0], ay = v[1], az = v[2];
  const double bx = v[3], by = v[4], bz = v[5];
  const double cx = v[6], cy = v[7], cz = v[8];
  const double abx = bx - ax, aby = by - ay, abz = bz - az;
  const double acx = cx - ax, acy = cy - ay, acz = cz - az;
  const double apx = p[0] - ax, apy = p[1] - ay, apz = p[2] - az;
  const double d1 = fma(abx, apx, fma(aby, apy, abz * apz));
  const double d2 = fma(acx, apx, fma(acy, apy, acz * apz));
  if (d1 <= 0 && d2 <= 0) { q[0] = ax; q[1] = ay; q[2] = az; *reg = 0; return; }
  const double bpx = p[0] - bx, bpy = p[1] - by, bpz = p[2] - bz;
  const double d3 = fma(abx, bpx, fma(aby, bpy, abz * bpz));
  const double d4 = fma(acx, bpx, fma(acy, bpy, acz * bpz));
  if (d3 >= 0 && d4 <= d3) { q[0] = bx; q[1] = by; q[2] = bz; *reg = 1; return; }
  const double vc = fma(d1, d4, -(d3 * d2));
  if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    const double t = d1 / (d1 - d3);
    q[0] = fma(t, abx, ax); q[1] = fma(t, aby, ay); q[2] = fma(t, abz, az);
    *reg = 3;
    return;
  }
  const double cpx = p[0] - cx, cpy = p[1] - cy, cpz = p[2] - cz;
  const double d5 = fma(abx, cpx, fma(aby, cpy, abz * cpz));
  const double d6 = fma(acx, cpx, fma(acy, cpy, acz * cpz));
  if (d6 >= 0 && d5 <= d6) { q[0] = cx; q[1] = cy; q[2] = cz; *reg = 2; return; }
  const double vb = fma(d5, d2, -(d1 * d6));
  if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    const double t = d2 / (d2 - d6);
    q[0] = fma(t, acx, ax); q[1] = fma(t, acy, ay); q[2] = fma(t, acz, az);
    *reg = 5;
    return;
  }
  const double va = fma(d3, d6, -(d5 * d4));
  const double e43 = d4 - d3, e56 = d5 - d6;
  if (va <= 0 && e43 >= 0 && e56 >= 0) {
    const double t = e43 / (e43 + e56);
    q[0] = fma(t, cx - bx, bx); q[1] = fma(t, cy - by, by); q[2] = fma(t, cz - bz, bz);
    *reg = 4;
    return;
  }
  const double inv = 1.0 / (va + vb + vc);
  const double vv = vb * inv, ww = vc * inv;
  q[0] = fma(ww, acx, fma(vv, abx, ax));
  q[1] = fma(ww, acy, fma(vv, aby, ay));
  q[2] = fma(ww, acz, fma(vv, abz, az));
  *reg = 6;
}

static inline double plane_value(const double* pl, const double* p) {
  return fma(pl[0], p[0], fma(pl[1], p[1], fma(pl[2], p[2], -pl[3])));
}

static inline double dist2_to(const double* p, const double* q) {
  const double dx = p[0] - q[0], dy = p[1] - q[1], dz = p[2] - q[2];
  return fma(dx, dx, fma(dy, dy, dz * dz));
}

static inline double edge_val(const double* fx, int e, const double* p) {
  const double* m = fx + 4 * e;
  return fma(m[0], p[0], fma(m[1], p[1], fma(m[2], p[2], -m[3])));
}

/* Local optimality certificate of q = closest point of triangle f (Voronoi
 * region reg) to p, as the kernel's cert_step: w = p - q in the normal cone
 * of the hull at q. Edge u->v shared with g: both in-plane edge values of p
 * <= tol; vertex v: w.(u - v) <= tol for every neighbour u, walking the fan of
 * faces around v through the neighbour table (<= 32 steps). On failure *n1,
 * *n2 name the faces of the descent step (-1 = none). */
static int cert_step(const oracle_posed* m, const double* p, int f, int reg, double scale, int* n1, int* n2) {
  *n1 = -1;
  *n2 = -1;
  if (reg == 6) return plane_value(m->planes_w + 4 * f, p) > 0; /* projection: optimal iff p above f */
  const int32_t* fv = m->faces + 3 * f;
  if (reg >= 3) {
    const int e = reg - 3;
    const int g = m->nbr[3 * f + e];
    const int32_t w = fv[e == 2 ? 0 : e + 1];
    const int32_t* gv = m->faces + 3 * g;
    const int eg = gv[0] == w ? 0 : (gv[1] == w ? 1 : 2); /* g's edge w -> u */
    const double sf = edge_val(m->facex_w + FX * f, e, p);
    const double sg = edge_val(m->facex_w + FX * g, eg, p);
    const double* U = m->verts_w + 4 * fv[e];
    const double* W = m->verts_w + 4 * w;
    const double tol = 1e-13 * (((fabs(p[0]) + fabs(p[1])) + fabs(p[2])) + scale) *
                       ((fabs(W[0] - U[0]) + fabs(W[1] - U[1])) + fabs(W[2] - U[2]));
    if (sf <= tol && sg <= tol) return 1;
    if (sg > tol && g != f) *n1 = g;
    return 0;
  }
  const int32_t v = fv[reg];
  const double* V = m->verts_w + 4 * v;
  const double wx = p[0] - V[0], wy = p[1] - V[1], wz = p[2] - V[2];
  const double tol = 1e-13 * ((fabs(wx) + fabs(wy)) + fabs(wz)) * scale;
  int g = f, j = reg;
  for (int it = 0; it < 32; ++it) {
    const double* U = m->verts_w + 4 * m->faces[3 * g + (j == 2 ? 0 : j + 1)];
    const double dot = fma(wx, U[0] - V[0], fma(wy, U[1] - V[1], wz * (U[2] - V[2])));
    const int g2 = m->nbr[3 * g + j];
    if (dot > tol) {
      *n1 = g != f ? g : g2;
      *n2 = (g != f && g2 != f) ? g2 : -1;
      return 0;
    }
    if (g2 == f) return 1;
    const int32_t* gv = m->faces + 3 * g2;
    j = gv[0] == v ? 0 : (gv[1] == v ? 1 : 2);
    g = g2;
  }
  return 0;
}

/* Signed distance of p to posed hull k, with its unit gradient. Restates
 * ConvexSurface(x) (src/Flash.jl:238-243) as the exact polytope SDF:
 *   inside / on the surface: max_f h_f (first max face's normal);
 *   outside: h_{f*} when p projects into triangle f*; else the closest point on
 *   triangle f*, certified by the normal cone at its feature (cert_step); a
 *   failed certificate names the faces of a strictly descending step (<= 24
 *   steps); a stalled walk -> exhaustive scan of the visible faces whose plane
 *   distance is below the best so far (strict < keeps the walk's point). */
void oracle_hull_sdf(const oracle_posed* m, int32_t k, const double* p, double* d, double* g) {
  const int f0 = m->face_off[k], f1 = m->face_off[k + 1];
  double hmax = -INFINITY;
  int fs = f0;
  for (int f = f0; f < f1; ++f) {
    const double h = plane_value(m->planes_w + 4 * f, p);
    if (h > hmax) { hmax = h; fs = f; }
  }
  const double* pls = m->planes_w + 4 * fs;
  *d = hmax;
  g[0] = pls[0]; g[1] = pls[1]; g[2] = pls[2];
  if (!(hmax > 0)) return;
  const double* fx = m->facex_w + FX * fs;
  const double s[3] = {fma(fx[0], p[0], fma(fx[1], p[1], fma(fx[2], p[2], -fx[3]))),
                       fma(fx[4], p[0], fma(fx[5], p[1], fma(fx[6], p[2], -fx[7]))),
                       fma(fx[8], p[0], fma(fx[9], p[1], fma(fx[10], p[2], -fx[11])))};
  if (s[0] >= 0 && s[1] >= 0 && s[2] >= 0) return;
  const double scale = m->hscale[k];
  double q[3];
  int rA;
  closest_on_triangle(p, fx + 12, q, &rA);
  double best2 = dist2_to(p, q);
  /* stage B: descent walk (<= 24 steps), each step to a face the failed
   * certificate names, accepted only if strictly closer */
  int cf = fs, cr = rA, todo = 1;
  for (int step = 0; step < 24; ++step) {
    int n1, n2;
    if (cert_step(m, p, cf, cr, scale, &n1, &n2)) { todo = 0; break; }
    int moved = 0;
    for (int t = 0; t < 2; ++t) {
      const int g = t == 0 ? n1 : n2;
      if (g >= 0) {
        double c[3];
        int rg;
        closest_on_triangle(p, m->facex_w + FX * g + 12, c, &rg);
        const double d2 = dist2_to(p, c);
        if (d2 < best2) { best2 = d2; q[0] = c[0]; q[1] = c[1]; q[2] = c[2]; cf = g; cr = rg; moved = 1; }
      }
    }
    if (!moved) break;
  }
  if (todo) {
    /* stage C: continues from the walk's point; only a strictly closer face replaces it */
    double b2 = best2, b[3] = {q[0], q[1], q[2]};
    for (int f = f0; f < f1; ++f) {
      const double h = plane_value(m->planes_w + 4 * f, p);
      if (h > 0 && h * h < b2) {
        double c[3];
        int rg;
        closest_on_triangle(p, m->facex_w + FX * f + 12, c, &rg);
        const double d2 = dist2_to(p, c);
        if (d2 < b2) { b2 = d2; b[0] = c[0]; b[1] = c[1]; b[2] = c[2]; }
      }
    }
    best2 = b2;
    q[0] = b[0]; q[1] = b[1]; q[2] = b[2];
  }
  if (best2 > 0) {
    *d = sqrt(best2);
    const double inv = 1.0 / *d;
    g[0] = (p[0] - q[0]) * inv;
    g[1] = (p[1] - q[1]) * inv;
    g[2] = (p[2] - q[2]) * inv;
  } else {
    *d = 0.0; /* p on the boundary: subgradient = normal of the max face */
  }
}

/* Scene SDF: brute-force minimum over ALL surfaces in index order, strict <,
 * i.e. exactly the reference's `minimum(s(x) for s in all_surfaces)`. */
static void skin_one(const oracle_posed* m, const double* p, double* d, int32_t* k, double* g) {
  double best = INFINITY, gb[3] = {0, 0, 0};
  int32_t bk = 0;
  for (int32_t kk = 0; kk < m->S; ++kk) {
    double dk, gk[3];
    const int32_t si = m->surf_index[kk];
    if (si >= 0) {
      oracle_hull_sdf(m, si, p, &dk, gk);
    } else {
      const int r = -si - 1, r0 = m->rbf_row_off[r];
      oracle_rbf_skin(m->rbf_rows + 4 * r0, m->rbf_row_off[r + 1] - r0 - 1, p, &dk, gk);
    }
    if (dk < best) { best = dk; bk = kk; gb[0] = gk[0]; gb[1] = gk[1]; gb[2] = gk[2]; }
  }
  *d = best;
  *k = bk;
  g[0] = gb[0]; g[1] = gb[1]; g[2] = gb[2];
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

/* Per-point skin over a cloud. Any output may be NULL. threads <= 0: all. */
void oracle_skin(const oracle_posed* m, const double* pts, int64_t n, double* d_out, int32_t* k_out,
                 double* g_out, int32_t threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 256)
#endif
  for (int64_t i = 0; i < n; ++i) {
    double d, g[3];
    int32_t k;
    skin_one(m, pts + 3 * i, &d, &k, g);
    if (d_out) d_out[i] = d;
    if (k_out) k_out[i] = k;
    if (g_out) { g_out[3 * i] = g[0]; g_out[3 * i + 1] = g[1]; g_out[3 * i + 2] = g[2]; }
  }
  (void)threads;
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
