// hull.cpp — convex hull of a mesh's vertex set (host side of fsdf_set_model).
//
// The reference never builds a hull: EnhancedGJK.NeighborMesh(mesh)
// (src/models.jl:152) walks the mesh vertices with a support function, so the
// shape it measures is conv(vertices). The STL triangulations shipped with the
// IRB140 (examples/data/IRB140/urdf/meshes/*_chull.stl) are NOT that hull
// (concave edges, inconsistent windings), so the face
// planes used by the exact polytope SDF are rebuilt here from the vertex set.
//
// Incremental hull, O(n·F): fine for the ~52-vertex link hulls and anything up
// to a few thousand points. Output faces are triangles, outward, CCW.

#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <utility>
#include <vector>

#include "flashsdf.h"

namespace {

struct HFace {
  int v[3];
  double n[3];
  double d;
  bool alive;
};

inline void sub3(const double* a, const double* b, double* o) {
  o[0] = a[0] - b[0];
  o[1] = a[1] - b[1];
  o[2] = a[2] - b[2];
}
inline void cross3(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline double norm3(const double* a) { return sqrt(dot3(a, a)); }

// Outward unit plane of triangle (a, b, c) given CCW order.
bool make_plane(const double* P, HFace& f) {
  const double* a = P + 3 * f.v[0];
  const double* b = P + 3 * f.v[1];
  const double* c = P + 3 * f.v[2];
  double ab[3], ac[3], n[3];
  sub3(b, a, ab);
  sub3(c, a, ac);
  cross3(ab, ac, n);
  const double len = norm3(n);
  if (!(len > 0.0)) return false;
  f.n[0] = n[0] / len;
  f.n[1] = n[1] / len;
  f.n[2] = n[2] / len;
  // d from the three vertices' mean offset (symmetric in the vertices)
  f.d = (dot3(f.n, a) + dot3(f.n, b) + dot3(f.n, c)) / 3.0;
  return true;
}

inline double plane_dist(const HFace& f, const double* p) { return dot3(f.n, p) - f.d; }

}  // namespace

extern "C" int fsdf_convex_hull(const double* points, int32_t n, int32_t* n_vertices_out, double* vertices_out,
                                int32_t* n_faces_out, int32_t* faces_out, double* planes_out) {
  if (!points || !n_vertices_out || !vertices_out || !n_faces_out || !faces_out || !planes_out) return FSDF_ERR_ARG;
  if (n < 4) return FSDF_ERR_DEGENERATE;
  for (int i = 0; i < 3 * n; ++i)
    if (!std::isfinite(points[i])) return FSDF_ERR_ARG;
  const double* P = points;

  double lo[3] = {P[0], P[1], P[2]}, hi[3] = {P[0], P[1], P[2]};
  for (int i = 1; i < n; ++i)
    for (int j = 0; j < 3; ++j) {
      lo[j] = std::min(lo[j], P[3 * i + j]);
      hi[j] = std::max(hi[j], P[3 * i + j]);
    }
  const double scale = std::max(std::max(hi[0] - lo[0], hi[1] - lo[1]), hi[2] - lo[2]);
  if (!(scale > 0.0)) return FSDF_ERR_DEGENERATE;
  const double eps = 1e-11 * scale;

  // initial tetrahedron
  int i0 = 0;
  for (int i = 1; i < n; ++i)
    if (P[3 * i] < P[3 * i0]) i0 = i;
  int i1 = -1;
  double best = -1.0;
  for (int i = 0; i < n; ++i) {
    double e[3];
    sub3(P + 3 * i, P + 3 * i0, e);
    const double l = norm3(e);
    if (l > best) { best = l; i1 = i; }
  }
  if (best <= eps) return FSDF_ERR_DEGENERATE;
  int i2 = -1;
  best = -1.0;
  {
    double u[3];
    sub3(P + 3 * i1, P + 3 * i0, u);
    for (int i = 0; i < n; ++i) {
      double e[3], c[3];
      sub3(P + 3 * i, P + 3 * i0, e);
      cross3(u, e, c);
      const double l = norm3(c) / norm3(u);
      if (l > best) { best = l; i2 = i; }
    }
  }
  if (best <= eps) return FSDF_ERR_DEGENERATE;
  int i3 = -1;
  best = -1.0;
  double nrm[3];
  {
    double u[3], v[3];
    sub3(P + 3 * i1, P + 3 * i0, u);
    sub3(P + 3 * i2, P + 3 * i0, v);
    cross3(u, v, nrm);
    const double l = norm3(nrm);
    for (int j = 0; j < 3; ++j) nrm[j] /= l;
    for (int i = 0; i < n; ++i) {
      double e[3];
      sub3(P + 3 * i, P + 3 * i0, e);
      const double h = fabs(dot3(nrm, e));
      if (h > best) { best = h; i3 = i; }
    }
  }
  if (best <= eps) return FSDF_ERR_DEGENERATE;

  std::vector<HFace> faces;
  faces.reserve(4 * n);
  std::map<std::pair<int, int>, int> edge_face;  // directed edge -> face
  auto add_face = [&](int a, int b, int c) -> bool {
    HFace f;
    f.v[0] = a; f.v[1] = b; f.v[2] = c;
    f.alive = true;
    if (!make_plane(P, f)) return false;
    const int id = (int)faces.size();
    faces.push_back(f);
    edge_face[{a, b}] = id;
    edge_face[{b, c}] = id;
    edge_face[{c, a}] = id;
    return true;
  };
  {
    // orient so that i3 is behind (i0, i1, i2)
    double e[3];
    sub3(P + 3 * i3, P + 3 * i0, e);
    int a = i0, b = i1, c = i2;
    if (dot3(nrm, e) > 0) std::swap(b, c);
    if (!add_face(a, b, c) || !add_face(a, c, i3) || !add_face(c, b, i3) || !add_face(b, a, i3))
      return FSDF_ERR_DEGENERATE;
  }

  // Insert the remaining points farthest-first from the tetrahedron's centroid:
  // extreme points enter before points on edges/faces, which then test as not
  // visible (within eps) and never become (coplanar) hull vertices.
  std::vector<int> order;
  {
    double c0[3];
    for (int j = 0; j < 3; ++j) c0[j] = 0.25 * (P[3 * i0 + j] + P[3 * i1 + j] + P[3 * i2 + j] + P[3 * i3 + j]);
    std::vector<double> r(n);
    for (int i = 0; i < n; ++i) {
      double e[3];
      sub3(P + 3 * i, c0, e);
      r[i] = dot3(e, e);
    }
    for (int i = 0; i < n; ++i)
      if (i != i0 && i != i1 && i != i2 && i != i3) order.push_back(i);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return r[a] > r[b]; });
  }
  std::vector<int> visible;
  for (int p : order) {
    const double* pp = P + 3 * p;
    visible.clear();
    for (int f = 0; f < (int)faces.size(); ++f)
      if (faces[f].alive && plane_dist(faces[f], pp) > eps) visible.push_back(f);
    if (visible.empty()) continue;
    // horizon: directed edges (a,b) of visible faces whose twin (b,a) is on a
    // non-visible face
    std::vector<std::pair<int, int>> horizon;
    for (int f : visible) faces[f].alive = false;
    for (int f : visible) {
      for (int e = 0; e < 3; ++e) {
        const int a = faces[f].v[e], b = faces[f].v[(e + 1) % 3];
        auto it = edge_face.find({b, a});
        if (it != edge_face.end() && faces[it->second].alive) horizon.push_back({a, b});
      }
    }
    for (int f : visible)
      for (int e = 0; e < 3; ++e) edge_face.erase({faces[f].v[e], faces[f].v[(e + 1) % 3]});
    for (auto& hb : horizon)
      if (!add_face(hb.first, hb.second, p)) return FSDF_ERR_DEGENERATE;
  }

  // compact vertices in ascending input order
  std::vector<int> used(n, 0);
  int nf = 0;
  for (auto& f : faces)
    if (f.alive) {
      ++nf;
      for (int j = 0; j < 3; ++j) used[f.v[j]] = 1;
    }
  if (nf > 2 * n - 4) return FSDF_ERR_DEGENERATE;
  std::vector<int> remap(n, -1);
  int nv = 0;
  for (int i = 0; i < n; ++i)
    if (used[i]) {
      remap[i] = nv;
      for (int j = 0; j < 3; ++j) vertices_out[3 * nv + j] = P[3 * i + j];
      ++nv;
    }
  int o = 0;
  for (auto& f : faces) {
    if (!f.alive) continue;
    for (int j = 0; j < 3; ++j) faces_out[3 * o + j] = remap[f.v[j]];
    for (int j = 0; j < 3; ++j) planes_out[4 * o + j] = f.n[j];
    planes_out[4 * o + 3] = f.d;
    ++o;
  }
  *n_vertices_out = nv;
  *n_faces_out = nf;
  return FSDF_OK;
}
