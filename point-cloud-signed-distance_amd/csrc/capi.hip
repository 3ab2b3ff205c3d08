// capi.hip — the C-ABI of include/flashsdf.h: context, resident model and
// cloud, and the three-launch residual pass (pose -> pass -> reduce).
//
// Ownership mirrors the reference: the cloud is held for a whole frame
// (CostFunctor keeps sensed_points by reference, src/gradientdescent.jl:41-47)
// and every evaluation only ships the K poses (what set_configuration! +
// transform_to_root produce in src/Flash.jl:248). No CPU fallback exists: a
// context cannot be created without a HIP device.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <map>
#include <utility>
#include <string>
#include <vector>

#include "flashsdf.h"
#include "fsdf_internal.h"
#include "kin_impl.h"

#ifndef FSDF_POSE_OVERLAP
#define FSDF_POSE_OVERLAP 0  // (pose_model: measured slower, off)
#endif
#ifndef FSDF_PRIOR_SEEDS
#define FSDF_PRIOR_SEEDS 1
#endif
#ifndef FSDF_ORDER_EVERY
#define FSDF_ORDER_EVERY 16
#endif
static constexpr int kOrderEvery = FSDF_ORDER_EVERY;

namespace {

constexpr int kPoseRing = 8;
#ifndef FSDF_CHUNK_WS
#define FSDF_CHUNK_WS 1  // passes over the resident cloud read the chunk spheres of set_points
#endif

template <typename P>
hipError_t dalloc(P** p, size_t bytes) {
  *p = nullptr;
  if (bytes == 0) return hipSuccess;
  return hipMalloc((void**)p, bytes);
}
template <typename P>
void dfree(P*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

}  // namespace

// default plan composition: chunks split over 4 / 2 waves (fsdf_set_plan shares < 0)
static constexpr int64_t kPlanDefault4 = 96, kPlanDefault2 = 192;

struct fsdf_ctx {
  int device = 0;
  int precision = 64;
  int sort_points = 0;
  int cull = 1;
  int out_order = FSDF_ORDER_CALLER;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  std::string pass_kernel;  // the pass-kernel variant of the last pass (fsdf_pass_kernel_name)

  // local model
  fsdf::LocalModel lm;
  double* d_verts_l = nullptr;
  int32_t* d_faces = nullptr;
  double* d_planes_l = nullptr;
  int32_t* d_face_hull = nullptr;
  double* d_sphere_l = nullptr;
  double* d_box_l = nullptr;
  int32_t* d_face_off = nullptr;
  int32_t* d_vert_hull = nullptr;
  int32_t* d_vert_off = nullptr;
  int32_t* d_face_rows = nullptr;
  int32_t* d_hull_surface = nullptr;
  int32_t* d_item_meta = nullptr;  // LocalModel::item_meta
  int32_t* d_surface_kind = nullptr;
  int32_t* d_rbf_surface = nullptr;
  int32_t* d_rbf_row_off = nullptr;
  int32_t* d_rbf_acc_off = nullptr;
  double* d_rbf64 = nullptr;     // per-pass RBF rows (f64)
  double* h_rbf[kPoseRing] = {}; // pinned staging ring for RBF rows (own slots and events,
  hipEvent_t rbf_ev[kPoseRing] = {};  // independent of the pose ring: poses of <= 64
  std::vector<int32_t> h_surface_kind, h_n_centers;  // host copy of the surface list (set_surfaces)
  int rbf_slot = 0;                   // surfaces never touch theirs)
  bool rbf_ready = false;
  // posed model, double-buffered: pass i poses into buffer i % 2 on its own
  // stream while the context stream still runs pass i-1 / its reduce
  // (FSDF_POSE_OVERLAP); ev_pm_free[b] marks the last read of buffer b
  fsdf::PosedModel pm;
  fsdf::PosedModel pm_alt;
  int pm_next = 0;
  hipStream_t pose_stream = nullptr;
  hipEvent_t ev_pose = nullptr;
  hipEvent_t ev_pm_free[2] = {};
  // poses: pinned ring + device copy
  double* h_poses[kPoseRing] = {};
  hipEvent_t pose_ev[kPoseRing] = {};
  int pose_slot = 0;
  double* d_poses = nullptr;
  // pinned read-back of the accumulator (fetch): a pageable destination makes
  // the D2H copy go through the runtime's staging buffer
  double* h_acc = nullptr;
  int h_acc_cap = 0;
  // resident cloud (precision-typed AoS)
  int64_t n = 0;
  void* d_pts = nullptr;
  int64_t pts_cap = 0;
  int32_t* d_perm = nullptr;        // resident i -> caller index (sorted clouds)
  int64_t perm_cap = 0;
  float* d_chunk_ws = nullptr;       // [ceil(n/64)][4] bounding sphere per 64-point chunk
  uint8_t* d_prior = nullptr;        // [n] each resident point's nearest surface in the last pass (seed hint)
  int64_t prior_cap = 0;
  bool prior_ok = false;             // d_prior was written by a pass over the current resident cloud
  // regroup (fsdf_regroup_points): mode (fsdf_set_regroup), whether the
  // resident cloud has been regrouped since its set_points, whether its first
  // iteration pass is still to come (the auto regroup follows that pass), and
  // the shape of the last resident pass (the auto rule's input)
  int regroup_mode = FSDF_REGROUP_AUTO;
  bool regrouped = false;
  bool regroup_pending = false;
  int last_pass_shape = 0;           // 0 none, 1 one wave per chunk, 2 hull-partitioned tiers, 3 planned
  int64_t chunk_ws_cap = 0;          // chunks
  fsdf::SortScratch sort;            // per-frame sort scratch (grown only)
  double* d_staging = nullptr;       // host-source clouds land here first
  int64_t staging_cap = 0;
  // the next frame's cloud, copied ahead on a stream of its own (fsdf_prefetch_points)
  double* d_prefetch = nullptr;
  int64_t prefetch_cap = 0, prefetch_n = -1;  // -1: none pending
  // a prefetch is queued on the next pass's launch (its host-side work then
  // overlaps that pass instead of delaying the frame's first launch): the
  // caller's cloud, whether it is still to be issued, and the issue's result
  const double* prefetch_src = nullptr;
  bool prefetch_deferred = false;
  int prefetch_rc = 0;
  // ... and its resident form, sorted there too (swapped in by fsdf_set_points_prefetched)
  bool prefetch_sorted = false;
  void* d_pts_next = nullptr;
  int32_t* d_perm_next = nullptr;
  float* d_chunk_ws_next = nullptr;
  int64_t pts_cap_next = 0, perm_cap_next = 0, chunk_ws_cap_next = 0;
  fsdf::SortScratch sort_next;
  // seeds carried from one cloud to the next (a voxel grid of the last pass's k*)
  uint8_t* d_vox = nullptr;
  bool vox_ok = false, seed_pending = false;
  fsdf::VoxBox vox;
  hipStream_t copy_stream = nullptr;
  hipEvent_t ev_prefetch = nullptr;
  bool ranged = false;               // the resident cloud is a range of a larger one (fsdf_set_points_range)
  void* d_range_pts = nullptr;       // fsdf_set_points_range: the whole cloud, sorted (scratch)
  int32_t* d_range_perm = nullptr;
  int64_t range_cap = 0;
  // work
  double* d_partials = nullptr;
  size_t partials_cap = 0;
  // cost-ordered schedule of resident-cloud passes (fsdf::PassOutputs::order)
  uint32_t* d_block_cost = nullptr;  // [kMaxBlocks]
  // the one-wave grid's heaviest-first block orders, one per layout of a frame's
  // cloud: [0] its Hilbert order (the frame's first pass), [1] regrouped (the
  // rest of the frame) — each rebuilt from the costs of a pass in its layout, so
  // a frame's passes run the order the previous frame left for the same layout
  int32_t* d_block_order[2] = {nullptr, nullptr};  // [kMaxBlocks]
  int order_nblocks[2] = {0, 0};  // grid the order was built for (0: none yet)
  int order_age[2] = {0, 0};      // passes since the order was rebuilt
  // planned pass (fsdf::planned_pass_kernel): per-chunk partial rows, chunk
  // durations and the workgroup plan built from them (fsdf_set_plan)
  fsdf::ChunkOutputs co;             // device arrays, [co_cap] chunks
  int64_t co_cap = 0;
  int co_s = 0;                      // surfaces the dense rows of co were sized for
  int32_t* d_plan = nullptr;         // [plan_cap][4]
  int32_t* d_plan_order = nullptr;   // [co_cap] plan_kernel scratch
  int64_t plan_cap = 0;
  int plan_grid = 0;                 // workgroups of the current plan (0: none — the default shape)
  int64_t plan_nc = -1;              // chunks the plan was built for
  int plan_age = 0;                  // planned passes since the plan was rebuilt
  int plan_enable = 1;
  double plan_f4 = -1.0, plan_f2 = -1.0;  // shares of the chunks split over 4 / 2 waves (< 0: default counts)
  int wave_slots = 0;                // device wave slots at the pass's occupancy (0: not queried yet)
  int64_t plan_max_points = -1;      // planned pass up to this cloud size (per device; -1: the model's default)
  double* d_accum = nullptr;
  int32_t* d_kstar = nullptr;
  double* d_d = nullptr;
  double* d_grad = nullptr;
  int64_t out_cap = 0;
  // query scratch (fsdf_skin)
  void* d_q = nullptr;
  int64_t q_cap = 0;
  double* d_q64 = nullptr;
  int64_t q64_cap = 0;
  // pass-kernel timing (fsdf_profile_pass)
  bool profiling = false;
  std::vector<hipEvent_t> prof_ev;  // pairs
  size_t prof_used = 0;             // events recorded (2 per pass)
  unsigned long long* d_stats = nullptr;  // fsdf_kernel_stats
  bool stats_on = false;
  // mechanism of fsdf_set_mechanism (host arrays; fsdf_value_and_gradient)
  struct Mechanism {
    int nb = 0, nq = 0;
    std::vector<int32_t> parent, kind, qoff, surface_body;
    std::vector<double> axis, AR, At, BR, Bt, frame_R, frame_t;
    std::vector<double> R, t, Rb, tb, poses, accum, work;  // scratch
    // RBF surfaces (fsdf_set_rbf_centres), in surface order; n == 0: undeclared
    struct Rbf {
      int n_sp = 0, n = 0;
      std::vector<int32_t> body, drow, piv;
      std::vector<double> local, values, centres, u, lu, G, work;
    };
    std::vector<Rbf> rbf;
    int n_deform = 0;
    double weight = 10.0;  // default_deformation_cost_weight (src/gradientdescent.jl:7)
    std::vector<double> rows, body_wrench, x_prepared;
    // the x of the last two fsdf_eval_state_device passes (their accumulators
    // may still be in flight): fsdf_state_gradient accepts only these (or the
    // last prepared x) and refuses any other with FSDF_ERR_STATE
    std::vector<double> x_pass[2];
    int x_pass_next = 0;
  } mech;
  // device solver loop of fsdf_descend (solver.hip): the mechanism's device
  // arrays (built on the first device descend after fsdf_set_mechanism) and
  // one frame's state; pinned staging for x / divisors in and x, f, flags out
  int solver_device = 1;             // fsdf_set_solver: 1 device where possible (default), 0 host loop,
                                     // 2 device required
  bool solver_tree_ok = false;
  fsdf::SolverTree stree;
  double* d_stree_d = nullptr;       // the tree blob (fsdf::SolverTree::blob)
  double* d_solver = nullptr;        // x | div | Rb | tb | poses | f
  int* d_solver_flags = nullptr;
  double* h_solver = nullptr;        // pinned: x | div | f | flags (as doubles)
  size_t solver_cap = 0, h_solver_cap = 0;
};

static int fail(fsdf_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIPCHECK(ctx, expr)                                                                             \
  do {                                                                                                  \
    hipError_t e_ = (expr);                                                                             \
    if (e_ != hipSuccess) return fail((ctx), FSDF_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

static void free_model(fsdf_ctx* c) {
  dfree(c->d_verts_l);
  dfree(c->d_faces);
  dfree(c->d_planes_l);
  dfree(c->d_face_hull);
  dfree(c->d_sphere_l);
  dfree(c->d_box_l);
  dfree(c->d_face_off);
  dfree(c->d_vert_hull);
  dfree(c->d_vert_off);
  dfree(c->d_face_rows);
  dfree(c->d_hull_surface);
  dfree(c->d_item_meta);
  dfree(c->d_surface_kind);
  dfree(c->d_rbf_surface);
  dfree(c->d_rbf_row_off);
  dfree(c->d_rbf_acc_off);
  if (c->pm.rbf_rows != (void*)c->d_rbf64) dfree(c->pm.rbf_rows);
  c->pm.rbf_rows = nullptr;
  dfree(c->d_rbf64);
  for (int i = 0; i < kPoseRing; ++i) {
    if (c->rbf_ev[i]) (void)hipEventSynchronize(c->rbf_ev[i]);
    if (c->h_rbf[i]) (void)hipHostFree(c->h_rbf[i]);
    c->h_rbf[i] = nullptr;
  }
  c->rbf_slot = 0;
  c->rbf_ready = false;
  if (c->pose_stream) (void)hipStreamSynchronize(c->pose_stream);
  for (fsdf::PosedModel* P : {&c->pm, &c->pm_alt}) {
    dfree(P->verts_w);
    dfree(P->hscale_w);
    dfree(P->planes_w);
    dfree(P->spheres_w);
    dfree(P->screen_w);
    dfree(P->image_w);
  }
  c->pm_alt.rbf_rows = nullptr;
  c->pm_next = 0;
  dfree(c->d_poses);
  dfree(c->d_accum);
  // (the partition tiers are a context setting: they survive a model change)
  const int64_t h4 = c->lm.hpart4_points, h2 = c->lm.hpart2_points;
  c->plan_nc = -1;
  c->prior_ok = false;        // seeds name surfaces of the old model
  c->solver_tree_ok = false;  // (its surface list)
  c->last_pass_shape = 0;
  c->lm = fsdf::LocalModel();
  c->lm.hpart4_points = h4;
  c->lm.hpart2_points = h2;
}

extern "C" int fsdf_create(fsdf_ctx** out, const fsdf_opts* opts) {
  if (!out) return FSDF_ERR_ARG;
  *out = nullptr;
  fsdf_ctx* c = new (std::nothrow) fsdf_ctx();
  if (!c) return FSDF_ERR_NOMEM;
  if (opts) {
    c->device = opts->device;
    c->precision = opts->precision ? opts->precision : 64;
    c->sort_points = opts->sort_points;
    c->cull = opts->cull;
  }
  if (c->precision != 64 && c->precision != 32) {
    delete c;
    return FSDF_ERR_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || c->device < 0 || c->device >= ndev) {
    delete c;
    return FSDF_ERR_HIP;
  }
  if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return FSDF_ERR_HIP;
  }
  c->stream = c->own_stream;
  // the prefetch copy stream right after the context stream: HIP hands out its
  // hardware queues round robin by stream creation, so the two land on
  // different queues (on a shared one the copy would serialise with the passes)
  if (hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_prefetch, hipEventDisableTiming) != hipSuccess) {
    (void)hipStreamDestroy(c->own_stream);
    delete c;
    return FSDF_ERR_HIP;
  }
  for (int i = 0; i < kPoseRing; ++i) c->pose_ev[i] = nullptr;
  // (the pose stream only where the pose overlap is built in: every stream of a
  // process shares its few hardware queues — GPU_MAX_HW_QUEUES, 4 by default —
  // and a stream sharing the context stream's queue serialises with it)
  if ((FSDF_POSE_OVERLAP && hipStreamCreateWithFlags(&c->pose_stream, hipStreamNonBlocking) != hipSuccess) ||
      hipEventCreateWithFlags(&c->ev_pose, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_pm_free[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_pm_free[1], hipEventDisableTiming) != hipSuccess) {
    (void)hipStreamDestroy(c->own_stream);
    delete c;
    return FSDF_ERR_HIP;
  }
  *out = c;
  return FSDF_OK;
}

extern "C" int fsdf_destroy(fsdf_ctx* c) {
  if (!c) return FSDF_ERR_ARG;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->pose_stream) (void)hipStreamSynchronize(c->pose_stream);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  free_model(c);
  dfree(c->d_pts);
  dfree(c->d_perm);
  dfree(c->d_chunk_ws);
  dfree(c->d_prior);
  dfree(c->d_staging);
  dfree(c->d_prefetch);
  dfree(c->d_pts_next);
  dfree(c->d_perm_next);
  dfree(c->d_chunk_ws_next);
  fsdf::free_sort_scratch(c->sort_next);
  dfree(c->d_vox);
  if (c->ev_prefetch) (void)hipEventDestroy(c->ev_prefetch);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  dfree(c->d_range_pts);
  dfree(c->d_range_perm);
  fsdf::free_sort_scratch(c->sort);
  dfree(c->d_partials);
  dfree(c->d_kstar);
  dfree(c->d_d);
  dfree(c->d_grad);
  dfree(c->d_q);
  dfree(c->d_q64);
  dfree(c->d_stats);
  dfree(c->d_block_cost);
  dfree(c->d_block_order[0]);
  dfree(c->d_block_order[1]);
  dfree(c->co.hdr);
  dfree(c->co.ent);  // (csum, dense: the same allocation)
  dfree(c->co.dur);
  dfree(c->d_plan);
  dfree(c->d_plan_order);
  dfree(c->d_stree_d);
  dfree(c->d_solver);
  dfree(c->d_solver_flags);
  if (c->h_solver) (void)hipHostFree(c->h_solver);
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  for (int i = 0; i < kPoseRing; ++i) {
    if (c->pose_ev[i]) (void)hipEventDestroy(c->pose_ev[i]);
    if (c->rbf_ev[i]) (void)hipEventDestroy(c->rbf_ev[i]);
    if (c->h_poses[i]) (void)hipHostFree(c->h_poses[i]);
  }
  if (c->h_acc) (void)hipHostFree(c->h_acc);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  if (c->pose_stream) (void)hipStreamDestroy(c->pose_stream);
  if (c->ev_pose) (void)hipEventDestroy(c->ev_pose);
  for (hipEvent_t e : c->ev_pm_free)
    if (e) (void)hipEventDestroy(e);
  delete c;
  return FSDF_OK;
}

extern "C" const char* fsdf_last_error(const fsdf_ctx* c) {
  if (!c) return "null context";
  return c->err.c_str();
}

extern "C" int fsdf_set_stream(fsdf_ctx* c, void* s) {
  if (!c) return FSDF_ERR_ARG;
  c->stream = s == FSDF_HIP_NULL_STREAM ? (hipStream_t)0 : (s ? (hipStream_t)s : c->own_stream);
  return FSDF_OK;
}

extern "C" int fsdf_num_hulls(const fsdf_ctx* c, int32_t* k) {
  if (!c || !k) return FSDF_ERR_ARG;
  *k = c->lm.S;  // surfaces of every kind = poses expected per pass
  return FSDF_OK;
}

static int accum_len(const fsdf_ctx* c) { return 1 + 6 * c->lm.S + c->lm.rbf_acc; }

extern "C" int fsdf_accum_len(const fsdf_ctx* c, int32_t* len) {
  if (!c || !len) return FSDF_ERR_ARG;
  *len = accum_len(c);
  return FSDF_OK;
}

extern "C" int fsdf_num_points(const fsdf_ctx* c, int64_t* n) {
  if (!c || !n) return FSDF_ERR_ARG;
  *n = c->n;
  return FSDF_OK;
}

static decltype(fsdf_ctx::mech) fresh_mechanism() { return {}; }

extern "C" int fsdf_set_surfaces(fsdf_ctx* c, const fsdf_surface* surfs, int32_t S) {
  if (!c) return FSDF_ERR_ARG;
  if (!surfs || S < 1) return fail(c, FSDF_ERR_ARG, "set_surfaces: need at least one surface");
  if (S > fsdf::kMaxHulls) return fail(c, FSDF_ERR_ARG, "set_surfaces: %d surfaces exceeds the limit %d", S, fsdf::kMaxHulls);
  std::vector<fsdf_hull> hulls;
  std::vector<int32_t> hull_surface, surface_kind, rbf_surface, rbf_row_off{0}, rbf_acc_off{0};
  for (int k = 0; k < S; ++k) {
    surface_kind.push_back(surfs[k].kind);
    if (surfs[k].kind == FSDF_SURFACE_HULL) {
      hulls.push_back(surfs[k].hull);
      hull_surface.push_back(k);
    } else if (surfs[k].kind == FSDF_SURFACE_RBF) {
      if (surfs[k].n_centers < 1) return fail(c, FSDF_ERR_ARG, "set_surfaces: RBF surface %d has no centres", k);
      rbf_surface.push_back(k);
      rbf_row_off.push_back(rbf_row_off.back() + surfs[k].n_centers + 1);
      rbf_acc_off.push_back(rbf_acc_off.back() + 4 * surfs[k].n_centers + 4);
    } else {
      return fail(c, FSDF_ERR_ARG, "set_surfaces: surface %d has unknown kind %d", k, surfs[k].kind);
    }
  }
  if (rbf_acc_off.back() > fsdf::kMaxRbfAccum)
    return fail(c, FSDF_ERR_ARG, "set_surfaces: RBF skins need %d accumulators, limit %d", rbf_acc_off.back(),
                fsdf::kMaxRbfAccum);
  const int K = (int)hulls.size();
  std::vector<double> verts, planes, sph, box;
  std::vector<int32_t> faces, face_hull, face_off, vert_hull, vert_off, face_rows;
  int stage_bytes = 0, stage_p64 = 0;
  const int tsz_ = c->precision == 64 ? (int)sizeof(double) : (int)sizeof(float);
  face_off.push_back(0);
  vert_off.push_back(0);
  for (int k = 0; k < K; ++k) {
    const fsdf_hull& h = hulls[(size_t)k];
    if (h.n_vertices < 4 || h.n_faces < 4 || !h.vertices || !h.faces)
      return fail(c, FSDF_ERR_ARG, "set_model: hull %d has %d vertices / %d faces", k, h.n_vertices, h.n_faces);
    const int vbase = (int)(verts.size() / 3);
    double cen[3] = {0, 0, 0};
    for (int i = 0; i < h.n_vertices; ++i)
      for (int j = 0; j < 3; ++j) {
        const double v = h.vertices[3 * i + j];
        if (!std::isfinite(v)) return fail(c, FSDF_ERR_ARG, "set_model: hull %d vertex %d not finite", k, i);
        verts.push_back(v);
        cen[j] += v;
      }
    for (int j = 0; j < 3; ++j) cen[j] /= h.n_vertices;
    for (int i = 0; i < h.n_vertices; ++i) vert_hull.push_back(k);
    vert_off.push_back((int32_t)vert_hull.size());
    double r2 = 0;
    for (int i = 0; i < h.n_vertices; ++i) {
      double s = 0;
      for (int j = 0; j < 3; ++j) {
        const double e = h.vertices[3 * i + j] - cen[j];
        s += e * e;
      }
      r2 = std::max(r2, s);
    }
    // radius padded and rounded up to float: the culling bound stays exact-safe
    float rf = (float)(sqrt(r2) * (1.0 + 1e-9) + 1e-12);
    rf = nextafterf(rf, INFINITY);
    sph.push_back(cen[0]);
    sph.push_back(cen[1]);
    sph.push_back(cen[2]);
    sph.push_back((double)rf);
    // body-frame bounding box, half extents padded and rounded up to float
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < h.n_vertices; ++i)
      for (int j = 0; j < 3; ++j) {
        lo[j] = std::min(lo[j], h.vertices[3 * i + j]);
        hi[j] = std::max(hi[j], h.vertices[3 * i + j]);
      }
    for (int j = 0; j < 3; ++j) box.push_back(0.5 * (lo[j] + hi[j]));
    box.push_back(0.0);
    for (int j = 0; j < 3; ++j) {
      const double c = 0.5 * (lo[j] + hi[j]);
      const double e = std::max(hi[j] - c, c - lo[j]);
      box.push_back((double)nextafterf((float)(e * (1.0 + 1e-9) + 1e-12), INFINITY));
    }
    box.push_back(0.0);
    for (int f = 0; f < h.n_faces; ++f) {
      for (int j = 0; j < 3; ++j) {
        const int vi = h.faces[3 * f + j];
        if (vi < 0 || vi >= h.n_vertices)
          return fail(c, FSDF_ERR_ARG, "set_model: hull %d face %d vertex index %d out of range", k, f, vi);
        faces.push_back(vbase + vi);
      }
      double pl[4];
      if (h.planes) {
        for (int j = 0; j < 4; ++j) pl[j] = h.planes[4 * f + j];
      } else {
        const double* a = h.vertices + 3 * h.faces[3 * f];
        const double* b = h.vertices + 3 * h.faces[3 * f + 1];
        const double* cc = h.vertices + 3 * h.faces[3 * f + 2];
        const double ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
        const double ac[3] = {cc[0] - a[0], cc[1] - a[1], cc[2] - a[2]};
        double nn[3] = {ab[1] * ac[2] - ab[2] * ac[1], ab[2] * ac[0] - ab[0] * ac[2], ab[0] * ac[1] - ab[1] * ac[0]};
        const double l = sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
        if (!(l > 0)) return fail(c, FSDF_ERR_DEGENERATE, "set_model: hull %d face %d degenerate", k, f);
        for (int j = 0; j < 3; ++j) pl[j] = nn[j] / l;
        pl[3] = pl[0] * a[0] + pl[1] * a[1] + pl[2] * a[2];
      }
      for (int j = 0; j < 4; ++j) planes.push_back(pl[j]);
      face_hull.push_back(k);
    }
    // face adjacency across each edge v_i -> v_{i+1} (the twin edge's face);
    // an open mesh edge points back at its own face (the certificate then
    // simply fails over to the exhaustive scan). Packed with the face's
    // hull-local vertex indices into one 16-byte row (fsdf_internal.h).
    {
      if (h.n_vertices > 0xffff || h.n_faces > 0xffff)
        return fail(c, FSDF_ERR_ARG, "set_model: hull %d has %d vertices / %d faces (limit 65535)", k,
                    h.n_vertices, h.n_faces);
      std::map<std::pair<int, int>, int> owner;
      for (int f = 0; f < h.n_faces; ++f)
        for (int e = 0; e < 3; ++e) owner[{h.faces[3 * f + e], h.faces[3 * f + (e + 1) % 3]}] = f;
      // exact duplicate planes (coplanar triangles of one facet): a later face
      // with the bitwise plane of an earlier one can never be the first-index
      // maximum, so the fp32 screen leaves it out (no near-tie fallbacks)
      std::map<std::array<uint64_t, 4>, int> seen_plane;
      for (int f = 0; f < h.n_faces; ++f) {
        std::array<uint64_t, 4> key;
        memcpy(key.data(), planes.data() + planes.size() - 4 * (size_t)(h.n_faces - f), sizeof(key));
        const bool dup = !seen_plane.emplace(key, f).second;
        int nb[3];
        for (int e = 0; e < 3; ++e) {
          auto it = owner.find({h.faces[3 * f + (e + 1) % 3], h.faces[3 * f + e]});
          nb[e] = it == owner.end() ? f : it->second;
        }
        const int* fv = h.faces + 3 * f;
        face_rows.push_back((int32_t)((uint32_t)fv[0] | ((uint32_t)fv[1] << 16)));
        face_rows.push_back((int32_t)((uint32_t)fv[2] | ((uint32_t)nb[0] << 16)));
        face_rows.push_back((int32_t)((uint32_t)nb[1] | ((uint32_t)nb[2] << 16)));
        face_rows.push_back(dup ? 1 : 0);
      }
      // per-wave LDS stage: plane rows (f64 contexts: the fp32 screening
      // pairs, 32 B per two faces) and vertex rows of 4 T, one 16-byte face row
      // per face (M64 f64: 4864 B; 4 waves + the wrench rows + the hull table
      // stay under 40 KiB, i.e. 4 workgroups per CU)
      const int plane_bytes = (tsz_ == 8 && FSDF_SCREEN32) ? 32 * ((h.n_faces + 1) / 2) : h.n_faces * 4 * tsz_;
      stage_bytes = std::max(stage_bytes, plane_bytes + h.n_vertices * 4 * tsz_ + 16 * h.n_faces);
      // (+ the fp64 planes, 32 B per face, when they are staged too; the
      // stage is then a copy of the hull's stage image, whose pair region is
      // nf + 1 chunks as in screen_w)
      stage_p64 = std::max(stage_p64, 16 * (h.n_faces + 1) + h.n_faces * 32 + h.n_vertices * 4 * tsz_ +
                                          16 * h.n_faces);
    }
    face_off.push_back((int32_t)(face_hull.size()));
  }
  // the RBF centre rows are staged through the same buffer, 64 rows at a time
  // at least; the resident-order gradient store transposes 64 x 3 doubles in it
  auto finish_stage = [&](int b) {
    b = (std::max(b, 64 * 4 * std::max(tsz_, 8)) + 15) & ~15;
    if (FSDF_RED_IN_STAGE && S <= 64 && rbf_surface.empty())
      b = std::max(b, fsdf::kRedInStageMinBytes);  // wrench rows + transpose after the evaluation
    return b;
  };
  stage_bytes = finish_stage(stage_bytes);
  stage_p64 = finish_stage(stage_p64);
  // f64 hull-only scenes of <= 64 surfaces also stage the fp64 planes when the
  // one-chunk-per-wave pass (wrench rows in the stage) then still runs 4
  // workgroups per CU
  int planes64 = 0;
  if (FSDF_STAGE_PLANES64 && tsz_ == 8 && FSDF_SCREEN32 && FSDF_RED_IN_STAGE && S <= 64 && rbf_surface.empty()) {
    fsdf::LocalModel probe;
    probe.K = K;
    probe.S = S;
    probe.stage_bytes = stage_p64;
    // (4 waves per SIMD: 16 waves per CU = 16·64/kPassBlock workgroups)
    if (fsdf::pass_lds_bytes(probe, false, true) <= (size_t)fsdf::kLdsPerCu * fsdf::kPassBlock / 1024 &&
        fsdf::pass_lds_bytes(probe, false) <= (size_t)fsdf::kMaxLds) {
      planes64 = 1;
      stage_bytes = stage_p64;
    }
  }
  {
    fsdf::LocalModel probe;
    probe.K = K;
    probe.S = S;
    probe.R = (int)rbf_surface.size();
    probe.stage_bytes = stage_bytes;
    const size_t lds = fsdf::pass_lds_bytes(probe, false);
    if (lds > (size_t)fsdf::kMaxLds)
      return fail(c, FSDF_ERR_ARG,
                  "set_model: the largest hull needs %d bytes of LDS stage per wave (%zu per workgroup, limit %d); "
                  "decimate it",
                  stage_bytes, lds, fsdf::kMaxLds);
  }
  HIPCHECK(c, hipSetDevice(c->device));
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  free_model(c);
  const int F = (int)face_hull.size(), V = (int)(verts.size() / 3);
  const size_t tsz = c->precision == 64 ? sizeof(double) : sizeof(float);
  HIPCHECK(c, dalloc(&c->d_verts_l, verts.size() * sizeof(double)));
  HIPCHECK(c, dalloc(&c->d_faces, faces.size() * sizeof(int32_t)));
  HIPCHECK(c, dalloc(&c->d_planes_l, planes.size() * sizeof(double)));
  HIPCHECK(c, dalloc(&c->d_face_hull, face_hull.size() * sizeof(int32_t)));
  HIPCHECK(c, dalloc(&c->d_sphere_l, sph.size() * sizeof(double)));
  HIPCHECK(c, dalloc(&c->d_box_l, box.size() * sizeof(double)));
  HIPCHECK(c, dalloc(&c->d_face_off, face_off.size() * sizeof(int32_t)));
  HIPCHECK(c, dalloc(&c->d_vert_hull, vert_hull.size() * sizeof(int32_t)));
  HIPCHECK(c, dalloc(&c->d_vert_off, vert_off.size() * sizeof(int32_t)));
  HIPCHECK(c, dalloc(&c->d_face_rows, std::max<size_t>(4, face_rows.size()) * sizeof(int32_t)));
  std::vector<int32_t> item_meta;  // (LocalModel::item_meta)
  item_meta.reserve((size_t)(F + V) * 4);
  auto meta = [&](int h) {
    const int nf = face_off[h + 1] - face_off[h];
    item_meta.insert(item_meta.end(), {hull_surface[h] | (nf << 16), h, face_off[h], vert_off[h]});
  };
  for (int f = 0; f < F; ++f) meta(face_hull[f]);
  for (int v = 0; v < V; ++v) meta(vert_hull[v]);
  HIPCHECK(c, dalloc(&c->d_item_meta, std::max<size_t>(4, item_meta.size()) * sizeof(int32_t)));
  if (!item_meta.empty())
    HIPCHECK(c, hipMemcpy(c->d_item_meta, item_meta.data(), item_meta.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  for (fsdf::PosedModel* P : {&c->pm, &c->pm_alt}) {
    HIPCHECK(c, dalloc((char**)&P->verts_w, (size_t)V * 4 * tsz));
    HIPCHECK(c, dalloc((char**)&P->hscale_w, (size_t)K * tsz));
    HIPCHECK(c, dalloc((char**)&P->planes_w, (size_t)std::max(F, 1) * 4 * tsz));
    HIPCHECK(c, dalloc(&P->spheres_w, (size_t)K * fsdf::kBoundFloats * sizeof(float)));
    HIPCHECK(c, dalloc(&P->screen_w, (size_t)std::max(F + K, 1) * 4 * sizeof(float)));
  }
  if (planes64) {
    // per-hull stage images (fsdf_internal.h PosedModel::image_w): the pose
    // kernel rewrites the pairs, planes and vertex rows every pass; the face
    // rows are static and written here
    const size_t chunks = (size_t)4 * F + K + 2 * (size_t)V;
    std::vector<int32_t> img(chunks * 4, 0);
    for (int h = 0; h < K; ++h) {
      const int nf = face_off[h + 1] - face_off[h], nv = vert_off[h + 1] - vert_off[h];
      const size_t base = (size_t)4 * face_off[h] + h + 2 * (size_t)vert_off[h] + 3 * (size_t)nf + 1 + 2 * (size_t)nv;
      memcpy(img.data() + 4 * base, face_rows.data() + 4 * (size_t)face_off[h], (size_t)nf * 4 * sizeof(int32_t));
    }
    for (fsdf::PosedModel* P : {&c->pm, &c->pm_alt}) {
      HIPCHECK(c, dalloc((char**)&P->image_w, chunks * 16));
      HIPCHECK(c, hipMemcpy(P->image_w, img.data(), chunks * 16, hipMemcpyHostToDevice));
    }
  }
  HIPCHECK(c, dalloc(&c->d_poses, (size_t)S * 12 * sizeof(double)));
  const int R = (int)rbf_surface.size();
  HIPCHECK(c, dalloc(&c->d_accum, (size_t)(1 + 6 * S + rbf_acc_off.back()) * sizeof(double)));
  HIPCHECK(c, dalloc(&c->d_hull_surface, std::max<size_t>(1, hull_surface.size()) * sizeof(int32_t)));
  HIPCHECK(c, dalloc(&c->d_surface_kind, surface_kind.size() * sizeof(int32_t)));
  HIPCHECK(c, dalloc(&c->d_rbf_surface, std::max<size_t>(1, rbf_surface.size()) * sizeof(int32_t)));
  HIPCHECK(c, dalloc(&c->d_rbf_row_off, rbf_row_off.size() * sizeof(int32_t)));
  HIPCHECK(c, dalloc(&c->d_rbf_acc_off, rbf_acc_off.size() * sizeof(int32_t)));
  if (!hull_surface.empty())
    HIPCHECK(c, hipMemcpy(c->d_hull_surface, hull_surface.data(), hull_surface.size() * sizeof(int32_t),
                          hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_surface_kind, surface_kind.data(), surface_kind.size() * sizeof(int32_t),
                        hipMemcpyHostToDevice));
  if (R > 0)
    HIPCHECK(c, hipMemcpy(c->d_rbf_surface, rbf_surface.data(), rbf_surface.size() * sizeof(int32_t),
                          hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_rbf_row_off, rbf_row_off.data(), rbf_row_off.size() * sizeof(int32_t),
                        hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_rbf_acc_off, rbf_acc_off.data(), rbf_acc_off.size() * sizeof(int32_t),
                        hipMemcpyHostToDevice));
  const int nrows = rbf_row_off.back();
  if (R > 0) {
    HIPCHECK(c, dalloc(&c->d_rbf64, (size_t)nrows * 4 * sizeof(double)));
    if (c->precision == 64) c->pm.rbf_rows = c->d_rbf64;
    else HIPCHECK(c, dalloc((char**)&c->pm.rbf_rows, (size_t)nrows * 4 * sizeof(float)));
    for (int i = 0; i < kPoseRing; ++i) {
      HIPCHECK(c, hipHostMalloc((void**)&c->h_rbf[i], (size_t)nrows * 4 * sizeof(double), hipHostMallocDefault));
      if (!c->rbf_ev[i]) HIPCHECK(c, hipEventCreateWithFlags(&c->rbf_ev[i], hipEventDisableTiming | hipEventDisableSystemFence));
    }
  }
  HIPCHECK(c, hipMemcpy(c->d_verts_l, verts.data(), verts.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_faces, faces.data(), faces.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_planes_l, planes.data(), planes.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_face_hull, face_hull.data(), face_hull.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_sphere_l, sph.data(), sph.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_box_l, box.data(), box.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_face_off, face_off.data(), face_off.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_vert_hull, vert_hull.data(), vert_hull.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHECK(c, hipMemcpy(c->d_vert_off, vert_off.data(), vert_off.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  if (!face_rows.empty())
    HIPCHECK(c, hipMemcpy(c->d_face_rows, face_rows.data(), face_rows.size() * sizeof(int32_t),
                          hipMemcpyHostToDevice));
  for (int i = 0; i < kPoseRing; ++i) {
    if (c->h_poses[i]) (void)hipHostFree(c->h_poses[i]);
    c->h_poses[i] = nullptr;
    HIPCHECK(c, hipHostMalloc((void**)&c->h_poses[i], (size_t)S * 12 * sizeof(double), hipHostMallocDefault));
    if (!c->pose_ev[i]) HIPCHECK(c, hipEventCreateWithFlags(&c->pose_ev[i], hipEventDisableTiming | hipEventDisableSystemFence));
  }
  c->lm.K = K;
  c->lm.F = F;
  c->lm.V = V;
  c->lm.verts_l = c->d_verts_l;
  c->lm.faces = c->d_faces;
  c->lm.planes_l = c->d_planes_l;
  c->lm.face_hull = c->d_face_hull;
  c->lm.sphere_l = c->d_sphere_l;
  c->lm.box_l = c->d_box_l;
  c->lm.face_off = c->d_face_off;
  c->lm.vert_hull = c->d_vert_hull;
  c->lm.vert_off = c->d_vert_off;
  c->lm.face_rows = c->d_face_rows;
  c->lm.item_meta = c->d_item_meta;
  c->lm.stage_bytes = stage_bytes;
  c->lm.planes64 = planes64;
  c->lm.S = S;
  c->lm.R = R;
  c->h_surface_kind = surface_kind;
  c->h_n_centers.assign(S, 0);
  for (int k = 0; k < S; ++k) c->h_n_centers[k] = surfs[k].kind == FSDF_SURFACE_RBF ? surfs[k].n_centers : 0;
  // the mechanism's surface bodies / frames / poses and the RBF centre
  // declarations refer to the previous surface list: drop them all (the
  // caller re-registers with fsdf_set_mechanism; iterations fail until then)
  c->mech = fresh_mechanism();
  c->lm.rbf_rows = nrows;
  c->lm.rbf_acc = rbf_acc_off.back();
  c->lm.hull_surface = c->d_hull_surface;
  c->lm.surface_kind = c->d_surface_kind;
  c->lm.rbf_surface = c->d_rbf_surface;
  c->lm.rbf_row_off = c->d_rbf_row_off;
  c->lm.rbf_acc_off = c->d_rbf_acc_off;
  return FSDF_OK;
}

extern "C" int fsdf_set_model(fsdf_ctx* c, const fsdf_hull* hulls, int32_t K) {
  if (!c) return FSDF_ERR_ARG;
  if (!hulls || K < 1) return fail(c, FSDF_ERR_ARG, "set_model: need at least one hull");
  std::vector<fsdf_surface> s((size_t)K);
  for (int k = 0; k < K; ++k) {
    s[(size_t)k].kind = FSDF_SURFACE_HULL;
    s[(size_t)k].n_centers = 0;
    s[(size_t)k].hull = hulls[k];
  }
  return fsdf_set_surfaces(c, s.data(), K);
}

extern "C" int fsdf_set_rbf_params(fsdf_ctx* c, const double* params, int64_t n) {
  if (!c) return FSDF_ERR_ARG;
  if (c->lm.R == 0) return fail(c, FSDF_ERR_STATE, "set_rbf_params: the scene has no RBF surface");
  if (!params || n != 4LL * c->lm.rbf_rows)
    return fail(c, FSDF_ERR_ARG, "set_rbf_params: expected %d doubles, got %lld", 4 * c->lm.rbf_rows, (long long)n);
  for (int64_t i = 0; i < n; ++i)
    if (!std::isfinite(params[i])) return fail(c, FSDF_ERR_ARG, "set_rbf_params: entry %lld not finite", (long long)i);
  HIPCHECK(c, hipSetDevice(c->device));
  // own ring: the slot is reused only after the copy that last read it ran
  // (the ring events only mark a copy's completion: no system-scope fence)
  // (an asynchronous caller may queue several passes with different rows)
  const int sl = c->rbf_slot;
  c->rbf_slot = (sl + 1) % kPoseRing;
  HIPCHECK(c, hipEventSynchronize(c->rbf_ev[sl]));
  memcpy(c->h_rbf[sl], params, (size_t)n * sizeof(double));
  HIPCHECK(c, hipMemcpyAsync(c->d_rbf64, c->h_rbf[sl], (size_t)n * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPCHECK(c, hipEventRecord(c->rbf_ev[sl], c->stream));
  if (c->precision != 64) HIPCHECK(c, fsdf::launch_to_f32(c->d_rbf64, (float*)c->pm.rbf_rows, n, c->stream));
  c->rbf_ready = true;
  return FSDF_OK;
}

// Convert/copy AoS f64 points already on the device into a resident buffer of
// the context precision, growing it when needed.
static int adopt_points_device(fsdf_ctx* c, const double* d_src, int64_t n, void** d_dst, int64_t* cap) {
  const size_t tsz = c->precision == 64 ? sizeof(double) : sizeof(float);
  if (*cap < n || !*d_dst) {
    dfree(*d_dst);
    *cap = 0;
    HIPCHECK(c, hipMalloc(d_dst, (size_t)std::max<int64_t>(n, 1) * 3 * tsz));
    *cap = std::max<int64_t>(n, 1);
  }
  if (n == 0) return FSDF_OK;
  if (c->precision == 64) {
    HIPCHECK(c, hipMemcpyAsync(*d_dst, d_src, (size_t)n * 3 * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  } else {
    HIPCHECK(c, fsdf::launch_to_f32(d_src, (float*)*d_dst, n * 3, c->stream));
  }
  return FSDF_OK;
}

static int finish_resident(fsdf_ctx* c, int64_t n, bool ranged, bool spheres_done = false);

// Seeds for a new cloud's first pass from the last pass over the previous one
// (fsdf_set_points / fsdf_set_points_prefetched of sorting hull-only contexts):
// before the cloud is replaced its points write their k* into a coarse voxel
// grid (carry_seeds_out), after it the new points read theirs into the seed
// buffer (finish_resident). The grid's box is the first cloud's box grown by
// a quarter of its extent each way, fixed for the context. Seeds only order
// the search — the pass's bits do not depend on them (tests/test_gpu_tracking.py).
static bool seeds_apply(const fsdf_ctx* c) {
  return FSDF_PRIOR_SEEDS && c->sort_points && c->lm.R == 0 && c->lm.S <= 64 && c->lm.K > 0;
}

static int ensure_vox_box(fsdf_ctx* c, const double* d_src, int64_t n) {
  if (c->vox_ok || n <= 0 || !seeds_apply(c)) return FSDF_OK;
  double* d_box = nullptr;
  hipError_t e = fsdf::cloud_box(d_src, n, c->sort, c->stream, &d_box);
  if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "set_points (seed box): %s", hipGetErrorString(e));
  double box[6];
  HIPCHECK(c, hipMemcpyAsync(box, d_box, sizeof box, hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(c, hipStreamSynchronize(c->stream));  // (once per context)
  for (int j = 0; j < 3; ++j) {
    const double ext = std::max(box[3 + j] - box[j], 1e-3);
    if (!std::isfinite(ext)) return FSDF_OK;  // (no seeds)
    c->vox.lo[j] = box[j] - 0.25 * ext;
    c->vox.inv[j] = fsdf::kVoxDim / (1.5 * ext);
  }
  if (!c->d_vox) HIPCHECK(c, hipMalloc(&c->d_vox, (size_t)fsdf::kVoxDim * fsdf::kVoxDim * fsdf::kVoxDim));
  c->vox_ok = true;
  return FSDF_OK;
}

static int carry_seeds_out(fsdf_ctx* c) {
  c->seed_pending = false;
  if (!c->vox_ok || !seeds_apply(c) || c->n <= 0 || !c->prior_ok || !c->d_prior || c->prior_cap < c->n || c->ranged)
    return FSDF_OK;
  HIPCHECK(c, hipMemsetAsync(c->d_vox, 0xFF, (size_t)fsdf::kVoxDim * fsdf::kVoxDim * fsdf::kVoxDim, c->stream));
  hipError_t e = fsdf::vox_scatter(c->precision, c->d_pts, c->n, c->d_prior, c->vox, c->d_vox, c->stream);
  if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "set_points (seeds): %s", hipGetErrorString(e));
  c->seed_pending = true;
  return FSDF_OK;
}

// [begin, end): the resident cloud is that range of the whole cloud's order
// (the Hilbert order of all n points with sort_points, else the caller's);
// the permutation then holds the points' indices in the whole cloud
// (fsdf_set_points_range). begin = 0, end = n: the whole cloud.
static int set_points_impl(fsdf_ctx* c, const double* src, int64_t n, bool device_src, int64_t begin, int64_t end,
                           bool range_call = false) {
  if (!c) return FSDF_ERR_ARG;
  if (n < 0 || (n > 0 && !src)) return fail(c, FSDF_ERR_ARG, "set_points: bad buffer (n=%lld)", (long long)n);
  if (begin < 0 || end < begin || end > n)
    return fail(c, FSDF_ERR_ARG, "set_points_range: bad range [%lld, %lld) of %lld points", (long long)begin,
                (long long)end, (long long)n);
  if ((c->sort_points || begin > 0 || end < n) && n > INT32_MAX)
    return fail(c, FSDF_ERR_ARG, "set_points: sorted or ranged clouds support < 2^31 points (n=%lld)", (long long)n);
  const bool ranged = begin > 0 || end < n;
  HIPCHECK(c, hipSetDevice(c->device));
  // the previous frame's work may still read the staging buffer / the cloud
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  int rc0 = ranged ? FSDF_OK : carry_seeds_out(c);  // (the previous cloud, still resident)
  if (rc0) return rc0;
  c->n = 0;
  const double* d_src = src;
  if (!device_src && n > 0) {
    if (c->staging_cap < n) {
      dfree(c->d_staging);
      c->staging_cap = 0;
      HIPCHECK(c, hipMalloc(&c->d_staging, (size_t)n * 3 * sizeof(double)));
      c->staging_cap = n;
    }
    HIPCHECK(c, hipMemcpyAsync(c->d_staging, src, (size_t)n * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    d_src = c->d_staging;
  }
  const int64_t nr = end - begin;  // resident points
  const size_t tsz = c->precision == 64 ? sizeof(double) : sizeof(float);
  auto ensure_res = [&]() -> int {
    if (c->pts_cap < nr || !c->d_pts) {
      dfree(c->d_pts);
      c->pts_cap = 0;
      HIPCHECK(c, hipMalloc(&c->d_pts, (size_t)std::max<int64_t>(nr, 1) * 3 * tsz));
      c->pts_cap = std::max<int64_t>(nr, 1);
    }
    if (c->perm_cap < nr || !c->d_perm) {
      dfree(c->d_perm);
      c->perm_cap = 0;
      HIPCHECK(c, hipMalloc(&c->d_perm, (size_t)std::max<int64_t>(nr, 1) * sizeof(int32_t)));
      c->perm_cap = std::max<int64_t>(nr, 1);
    }
    return FSDF_OK;
  };
  if (c->sort_points && n > 0) {
    // spatially coherent resident order + permutation back to caller order
    int rc = ensure_res();
    if (rc) return rc;
    if (!ranged) {
      rc = ensure_vox_box(c, d_src, n);
      if (rc) return rc;
    }
    if (!ranged) {
      hipError_t e = fsdf::sort_points_spatial(d_src, n, c->precision, c->d_pts, c->d_perm, c->sort, c->stream);
      if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "set_points (sort): %s", hipGetErrorString(e));
    } else {
      // the whole cloud sorted into scratch, then the range kept
      if (c->range_cap < n) {
        dfree(c->d_range_pts);
        dfree(c->d_range_perm);
        c->range_cap = 0;
        HIPCHECK(c, hipMalloc(&c->d_range_pts, (size_t)n * 3 * tsz));
        HIPCHECK(c, hipMalloc(&c->d_range_perm, (size_t)n * sizeof(int32_t)));
        c->range_cap = n;
      }
      hipError_t e =
          fsdf::sort_points_spatial(d_src, n, c->precision, c->d_range_pts, c->d_range_perm, c->sort, c->stream);
      if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "set_points_range (sort): %s", hipGetErrorString(e));
      if (nr > 0) {
        HIPCHECK(c, hipMemcpyAsync(c->d_pts, (const char*)c->d_range_pts + (size_t)begin * 3 * tsz,
                                   (size_t)nr * 3 * tsz, hipMemcpyDeviceToDevice, c->stream));
        HIPCHECK(c, hipMemcpyAsync(c->d_perm, c->d_range_perm + begin, (size_t)nr * sizeof(int32_t),
                                   hipMemcpyDeviceToDevice, c->stream));
      }
    }
  } else if (ranged) {
    // a slice of the caller's order; the permutation names the slice's indices
    int rc = ensure_res();
    if (rc) return rc;
    rc = adopt_points_device(c, d_src + 3 * begin, nr, &c->d_pts, &c->pts_cap);
    if (rc) return rc;
    std::vector<int32_t> idx((size_t)std::max<int64_t>(nr, 0));
    for (int64_t i = 0; i < nr; ++i) idx[(size_t)i] = (int32_t)(begin + i);
    if (nr > 0)
      HIPCHECK(c, hipMemcpyAsync(c->d_perm, idx.data(), (size_t)nr * sizeof(int32_t), hipMemcpyHostToDevice,
                                 c->stream));
    HIPCHECK(c, hipStreamSynchronize(c->stream));  // (idx is a host temporary)
  } else {
    dfree(c->d_perm);
    c->perm_cap = 0;
    int rc = adopt_points_device(c, d_src, n, &c->d_pts, &c->pts_cap);
    if (rc) return rc;
  }
  return finish_resident(c, nr, ranged || range_call);
}

// the per-cloud state of a new resident cloud of n points (d_pts / d_perm
// written, stream-ordered): chunk spheres (unless spheres_done: a prefetched
// cloud's came with it), seed buffer, plan and regroup state
static int finish_resident(fsdf_ctx* c, int64_t n, bool ranged, bool spheres_done) {
  if (n > 0 && !spheres_done) {  // per-chunk bounding spheres of the resident order (pose-independent)
    // (padded to whole 4-chunk pass workgroups: every wave of a hull-partitioned
    // pass reads its chunk's row, also past the cloud's end)
    const int64_t nc = ((n + 63) / 64 + 3) & ~(int64_t)3;
    if (c->chunk_ws_cap < nc) {
      HIPCHECK(c, hipStreamSynchronize(c->stream));
      dfree(c->d_chunk_ws);
      c->chunk_ws_cap = 0;
      HIPCHECK(c, hipMalloc(&c->d_chunk_ws, (size_t)nc * 4 * sizeof(float)));
      c->chunk_ws_cap = nc;
    }
    HIPCHECK(c, fsdf::launch_chunk_spheres(c->precision, c->d_pts, n, nc, c->d_chunk_ws, c->stream));
  }
  if (n > 0) {
    if (c->prior_cap < n) {  // (the previous frame's passes are done: synchronised above)
      HIPCHECK(c, hipStreamSynchronize(c->stream));  // (the seed scatter may still read it)
      dfree(c->d_prior);
      c->prior_cap = 0;
      HIPCHECK(c, hipMalloc(&c->d_prior, (size_t)n));
      c->prior_cap = n;
    }
  }
  // a new cloud: its first pass seeds from the previous cloud's voxels, else from the bounds
  c->prior_ok = false;
  if (c->seed_pending && n > 0 && !ranged && c->d_prior && c->prior_cap >= n) {
    hipError_t e = fsdf::vox_gather(c->precision, c->d_pts, n, c->vox, c->d_vox, c->d_prior, c->stream);
    if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "set_points (seeds): %s", hipGetErrorString(e));
    c->prior_ok = true;
  }
  c->seed_pending = false;
  c->regrouped = false;
  c->regroup_pending = true;  // (the auto regroup follows the new cloud's first iteration pass)
  c->last_pass_shape = 0;
  // the caller may reuse its buffer once this returns
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  c->n = n;
  // (a range call keeps resident-order outputs even when its range is the
  // whole cloud: the caller indexes them through the permutation)
  c->ranged = ranged;
  c->plan_nc = -1;  // a new cloud: its first planned pass runs the default shape and measures
  // and its first one-wave pass runs the previous cloud's Hilbert-layout
  // order and rebuilds it from its own costs (left to age, a stale order cost
  // the next passes 0.094 -> 0.111 ms, tools/seed_probe.py)
  c->order_age[0] = kOrderEvery;
  return FSDF_OK;
}

// ---- exchanged spatial shards (O(N/W) ingest per rank) ------------------------
extern "C" int fsdf_cloud_box_device(fsdf_ctx* c, const double* d_xyz, int64_t n, double* box_out) {
  if (!c) return FSDF_ERR_ARG;
  if (n < 0 || (n > 0 && !d_xyz) || !box_out) return fail(c, FSDF_ERR_ARG, "cloud_box_device: bad arguments");
  HIPCHECK(c, hipSetDevice(c->device));
  if (n == 0) {
    for (int j = 0; j < 3; ++j) {
      box_out[j] = HUGE_VAL;
      box_out[3 + j] = -HUGE_VAL;
    }
    return FSDF_OK;
  }
  double* d_box = nullptr;
  hipError_t e = fsdf::cloud_box(d_xyz, n, c->sort, c->stream, &d_box);
  if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "cloud_box_device: %s", hipGetErrorString(e));
  HIPCHECK(c, hipMemcpyAsync(box_out, d_box, 6 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  return FSDF_OK;
}

extern "C" int fsdf_curve_keys_device(fsdf_ctx* c, const double* d_xyz, int64_t n, const double* box,
                                      uint32_t* d_keys) {
  if (!c) return FSDF_ERR_ARG;
  if (n < 0 || (n > 0 && (!d_xyz || !d_keys)) || !box) return fail(c, FSDF_ERR_ARG, "curve_keys_device: bad arguments");
  for (int j = 0; j < 6; ++j)
    if (!std::isfinite(box[j])) return fail(c, FSDF_ERR_ARG, "curve_keys_device: box not finite");
  HIPCHECK(c, hipSetDevice(c->device));
  if (n == 0) return FSDF_OK;
  double* d_box = nullptr;  // (the scratch's box slot, filled from the host)
  hipError_t e = fsdf::cloud_box(d_xyz, 0, c->sort, c->stream, &d_box);
  if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "curve_keys_device: %s", hipGetErrorString(e));
  HIPCHECK(c, hipStreamSynchronize(c->stream));  // (an earlier sort may still read the slot)
  HIPCHECK(c, hipMemcpy(d_box, box, 6 * sizeof(double), hipMemcpyHostToDevice));
  e = fsdf::curve_keys(d_xyz, n, d_box, d_keys, c->stream);
  if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "curve_keys_device: %s", hipGetErrorString(e));
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  return FSDF_OK;
}

extern "C" int fsdf_set_points_keyed_device(fsdf_ctx* c, const double* d_xyz, const uint32_t* d_keys,
                                            const int64_t* d_index, int64_t n) {
  if (!c) return FSDF_ERR_ARG;
  if (n < 0 || (n > 0 && (!d_xyz || !d_keys || !d_index)))
    return fail(c, FSDF_ERR_ARG, "set_points_keyed_device: bad arguments");
  if (n > INT32_MAX) return fail(c, FSDF_ERR_ARG, "set_points_keyed_device: < 2^31 points per shard");
  HIPCHECK(c, hipSetDevice(c->device));
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  c->n = 0;
  const size_t tsz = c->precision == 64 ? sizeof(double) : sizeof(float);
  if (c->pts_cap < n || !c->d_pts) {
    dfree(c->d_pts);
    c->pts_cap = 0;
    HIPCHECK(c, hipMalloc(&c->d_pts, (size_t)std::max<int64_t>(n, 1) * 3 * tsz));
    c->pts_cap = std::max<int64_t>(n, 1);
  }
  if (c->perm_cap < n || !c->d_perm) {
    dfree(c->d_perm);
    c->perm_cap = 0;
    HIPCHECK(c, hipMalloc(&c->d_perm, (size_t)std::max<int64_t>(n, 1) * sizeof(int32_t)));
    c->perm_cap = std::max<int64_t>(n, 1);
  }
  if (n > 0) {
    hipError_t e = fsdf::sort_points_keyed(d_xyz, d_keys, d_index, n, c->precision, c->d_pts, c->d_perm, c->sort,
                                           c->stream);
    if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "set_points_keyed_device (sort): %s", hipGetErrorString(e));
  }
  return finish_resident(c, n, true);
}

extern "C" int fsdf_set_points(fsdf_ctx* c, const double* xyz, int64_t n) {
  return set_points_impl(c, xyz, n, false, 0, n);
}

extern "C" int fsdf_set_points_device(fsdf_ctx* c, const double* d_xyz, int64_t n) {
  return set_points_impl(c, d_xyz, n, true, 0, n);
}

// The next frame's cloud ahead of time: its host-to-device copy runs on a
// stream of the context's own while the current frame's passes run on the
// context stream (the copy engine beside the compute units), and
// fsdf_set_points_prefetched then makes it resident from the device copy —
// the per-frame ingest loses its host-link transfer (25 MB at 2^20 points).
// The copy overlaps only from page-locked host memory; the caller keeps xyz
// unchanged until fsdf_set_points_prefetched returns. A second prefetch
// replaces a pending one. fsdf_prefetch_points only records the cloud;
// prefetch_issue enqueues the copy and sort on the copy stream, from the next
// pass's launch (run_pass) or from fsdf_set_points_prefetched when no pass
// came between.
static int prefetch_issue(fsdf_ctx* c) {
  c->prefetch_deferred = false;
  const double* xyz = c->prefetch_src;
  const int64_t n = c->prefetch_n;
  HIPCHECK(c, hipSetDevice(c->device));
  // (an earlier prefetch's copy may still write the buffer; a consumed one's
  // sort has finished: fsdf_set_points_prefetched returns after it)
  HIPCHECK(c, hipStreamSynchronize(c->copy_stream));
  if (c->prefetch_cap < n) {
    dfree(c->d_prefetch);
    c->prefetch_cap = 0;
    HIPCHECK(c, hipMalloc(&c->d_prefetch, (size_t)n * 3 * sizeof(double)));
    c->prefetch_cap = n;
  }
  if (n > 0)
    HIPCHECK(c, hipMemcpyAsync(c->d_prefetch, xyz, (size_t)n * 3 * sizeof(double), hipMemcpyHostToDevice,
                               c->copy_stream));
  // the next resident cloud, Hilbert-sorted on the copy stream as well (its own
  // buffers and sort scratch: the current frame's cloud is untouched), so the
  // next frame's set_points_prefetched only swaps buffers
  c->prefetch_sorted = false;
  if (n > 0 && c->sort_points && n <= INT32_MAX) {
    const size_t tsz = c->precision == 64 ? sizeof(double) : sizeof(float);
    const int64_t nc = ((n + 63) / 64 + 3) & ~(int64_t)3;  // (finish_resident's padding)
    if (c->pts_cap_next < n) {
      dfree(c->d_pts_next);
      c->pts_cap_next = 0;
      HIPCHECK(c, hipMalloc(&c->d_pts_next, (size_t)n * 3 * tsz));
      c->pts_cap_next = n;
    }
    if (c->perm_cap_next < n) {
      dfree(c->d_perm_next);
      c->perm_cap_next = 0;
      HIPCHECK(c, hipMalloc(&c->d_perm_next, (size_t)n * sizeof(int32_t)));
      c->perm_cap_next = n;
    }
    if (c->chunk_ws_cap_next < nc) {
      dfree(c->d_chunk_ws_next);
      c->chunk_ws_cap_next = 0;
      HIPCHECK(c, hipMalloc(&c->d_chunk_ws_next, (size_t)nc * 4 * sizeof(float)));
      c->chunk_ws_cap_next = nc;
    }
    hipError_t e = fsdf::sort_points_spatial(c->d_prefetch, n, c->precision, c->d_pts_next, c->d_perm_next,
                                             c->sort_next, c->copy_stream);
    if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "prefetch_points (sort): %s", hipGetErrorString(e));
    HIPCHECK(c, fsdf::launch_chunk_spheres(c->precision, c->d_pts_next, n, nc, c->d_chunk_ws_next, c->copy_stream));
    c->prefetch_sorted = true;
  }
  HIPCHECK(c, hipEventRecord(c->ev_prefetch, c->copy_stream));
  return FSDF_OK;
}

extern "C" int fsdf_prefetch_points(fsdf_ctx* c, const double* xyz, int64_t n) {
  if (!c) return FSDF_ERR_ARG;
  if (n < 0 || (n > 0 && !xyz)) return fail(c, FSDF_ERR_ARG, "prefetch_points: bad buffer (n=%lld)", (long long)n);
  c->prefetch_src = xyz;
  c->prefetch_n = n;
  c->prefetch_deferred = true;
  c->prefetch_rc = FSDF_OK;
  return FSDF_OK;
}

extern "C" int fsdf_set_points_prefetched(fsdf_ctx* c) {
  if (!c) return FSDF_ERR_ARG;
  if (c->prefetch_n < 0) return fail(c, FSDF_ERR_STATE, "set_points_prefetched: no prefetch pending");
  const int64_t n = c->prefetch_n;
  int rc = c->prefetch_deferred ? prefetch_issue(c) : c->prefetch_rc;
  c->prefetch_n = -1;
  c->prefetch_rc = FSDF_OK;
  if (rc) return rc;
  HIPCHECK(c, hipSetDevice(c->device));
  HIPCHECK(c, hipStreamWaitEvent(c->stream, c->ev_prefetch, 0));  // (the copy, and the sort when done there)
  if (!c->prefetch_sorted) return set_points_impl(c, c->d_prefetch, n, true, 0, n);
  // the sorted next cloud becomes resident: the current frame's work is done
  // (synchronised), its buffers become the next prefetch's
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  rc = ensure_vox_box(c, c->d_prefetch, n);  // (a first cloud: the seed box)
  if (rc) return rc;
  rc = carry_seeds_out(c);  // (the previous cloud, still resident)
  if (rc) return rc;
  c->n = 0;
  std::swap(c->d_pts, c->d_pts_next);
  std::swap(c->pts_cap, c->pts_cap_next);
  std::swap(c->d_perm, c->d_perm_next);
  std::swap(c->perm_cap, c->perm_cap_next);
  std::swap(c->d_chunk_ws, c->d_chunk_ws_next);
  std::swap(c->chunk_ws_cap, c->chunk_ws_cap_next);
  return finish_resident(c, n, false, true);
}

extern "C" int fsdf_set_points_range(fsdf_ctx* c, const double* xyz, int64_t n, int64_t begin, int64_t end) {
  return set_points_impl(c, xyz, n, false, begin, end, true);
}

extern "C" int fsdf_set_points_range_device(fsdf_ctx* c, const double* d_xyz, int64_t n, int64_t begin,
                                            int64_t end) {
  return set_points_impl(c, d_xyz, n, true, begin, end, true);
}

// Regroup the resident cloud by each point's nearest surface in the last pass
// (a stable device sort on PassOutputs::prior_out's bytes: the Hilbert order
// kept within each group), so that a chunk's points share their surface and
// the seeded passes evaluate fewer hulls per chunk. Per-point results do not
// change; sums change in rounding only (other chunks). Stream-ordered after
// the passes already queued.
extern "C" int fsdf_regroup_points(fsdf_ctx* c) {
  if (!c) return FSDF_ERR_ARG;
  if (c->n == 0) return FSDF_OK;
  if (!c->d_perm)
    return fail(c, FSDF_ERR_STATE, "regroup_points: needs a sorted (sort_points) or ranged resident cloud");
  if (!c->prior_ok || !c->d_prior || c->prior_cap < c->n)
    return fail(c, FSDF_ERR_STATE, "regroup_points: run a pass over the resident cloud first (hull-only scenes)");
  HIPCHECK(c, hipSetDevice(c->device));
  void* pts = c->d_pts;
  hipError_t e = fsdf::regroup_points(&pts, &c->pts_cap, c->n, c->precision, c->d_perm, c->d_prior, c->sort, c->stream);
  c->d_pts = pts;
  if (e != hipSuccess) return fail(c, FSDF_ERR_HIP, "regroup_points: %s", hipGetErrorString(e));
  const int64_t nc = ((c->n + 63) / 64 + 3) & ~(int64_t)3;
  HIPCHECK(c, fsdf::launch_chunk_spheres(c->precision, c->d_pts, c->n, nc, c->d_chunk_ws, c->stream));
  c->plan_nc = -1;  // other chunks: the next planned pass measures anew
  // the one-wave grid's heaviest-first block order: the next pass runs the
  // regrouped layout's order (the previous frame's) and rebuilds it from its
  // own costs — unordered, that pass took 163 us, with the Hilbert layout's
  // order 177, with the previous regrouped one 122 (M64 2^20, profiles/r06/regroup_order/)
  c->order_age[1] = kOrderEvery;
  c->regrouped = true;
  c->regroup_pending = false;
  return FSDF_OK;
}

// The auto rule (FSDF_REGROUP_AUTO): regroup where the pass is bound by its
// summed work — the last resident pass ran one wave per chunk (the grid above
// the planned window) — and not where the planned pass or a hull-partitioned
// tier is bound by its heaviest chunk, which grouping makes heavier (2^17 step
// 0.0612 -> 0.0677 ms and worse). Needs a pass over the
// cloud (its k* are the groups) and a sorted or ranged cloud.
static bool regroup_wanted(const fsdf_ctx* c) {
  return c->n > 0 && c->d_perm && c->prior_ok && !c->regrouped && c->last_pass_shape == 1;
}

extern "C" int fsdf_regroup_auto(fsdf_ctx* c, int32_t* applied_out) {
  if (!c) return FSDF_ERR_ARG;
  if (applied_out) *applied_out = 0;
  if (!regroup_wanted(c)) return FSDF_OK;
  const int rc = fsdf_regroup_points(c);
  if (rc) return rc;
  if (applied_out) *applied_out = 1;
  return FSDF_OK;
}

extern "C" int fsdf_set_regroup(fsdf_ctx* c, int32_t mode) {
  if (!c) return FSDF_ERR_ARG;
  if (mode != FSDF_REGROUP_OFF && mode != FSDF_REGROUP_AUTO)
    return fail(c, FSDF_ERR_ARG, "set_regroup: unknown mode %d", mode);
  c->regroup_mode = mode;
  return FSDF_OK;
}

// after an iteration pass (value_and_gradient, eval_state_device, descend):
// the new cloud's first one regroups it when the auto rule says so
static int iteration_regroup(fsdf_ctx* c) {
  if (!c->regroup_pending) return FSDF_OK;
  c->regroup_pending = false;
  if (c->regroup_mode != FSDF_REGROUP_AUTO) return FSDF_OK;
  return fsdf_regroup_auto(c, nullptr);
}

static int ensure_partials(fsdf_ctx* c, int nblocks) {
  // (rounded up to whole 8-entry tiles: FSDF_PARTIALS_LAYOUT 2)
  const size_t need = (size_t)((accum_len(c) + 7) & ~7) * nblocks;
  if (c->partials_cap < need) {
    dfree(c->d_partials);
    c->partials_cap = 0;
    HIPCHECK(c, hipMalloc(&c->d_partials, need * sizeof(double)));
    c->partials_cap = need;
  }
  return FSDF_OK;
}

static int upload_poses(fsdf_ctx* c, const double* poses, hipStream_t st) {
  for (int i = 0; i < 12 * c->lm.S; ++i)
    if (!std::isfinite(poses[i])) return fail(c, FSDF_ERR_ARG, "poses: entry %d is not finite", i);
  if (c->lm.S <= fsdf::kPoseArgMax) return FSDF_OK;  // they ride in the pose kernel's arguments
  const int s = c->pose_slot;
  c->pose_slot = (s + 1) % kPoseRing;
  HIPCHECK(c, hipEventSynchronize(c->pose_ev[s]));  // slot free once its last copy ran
  memcpy(c->h_poses[s], poses, (size_t)c->lm.S * 12 * sizeof(double));
  HIPCHECK(c, hipMemcpyAsync(c->d_poses, c->h_poses[s], (size_t)c->lm.S * 12 * sizeof(double),
                             hipMemcpyHostToDevice, st));
  HIPCHECK(c, hipEventRecord(c->pose_ev[s], st));
  return FSDF_OK;
}

// Pose the model for one pass into the next posed buffer. With
// FSDF_POSE_OVERLAP the upload and pose kernel run on the context's pose
// stream — behind the last reader of that buffer (two passes back), ahead of
// the current pass's kernels on the context stream, which waits for them — so
// the pose kernel overlaps the previous pass's tail and reduce. *buf: the
// buffer index to release with release_posed() after its last reader.
// Measured: the cross-stream event waits cost more than the overlap saves
// (+10 us per step on M64), so it is off and the pose kernel runs in order.
// posed: the model is already posed on the device (the device solver loop's
// step poses the next pass's model itself, solver.hip): no pose launch.
static int pose_model(fsdf_ctx* c, const double* poses, fsdf::PosedModel** out, int* buf, bool posed = false) {
  const int b = FSDF_POSE_OVERLAP ? c->pm_next : 0;
  c->pm_next ^= FSDF_POSE_OVERLAP ? 1 : 0;
  fsdf::PosedModel* P = b ? &c->pm_alt : &c->pm;
  P->rbf_rows = c->pm.rbf_rows;  // per-pass RBF rows: one buffer, context-stream ordered
  const hipStream_t ps = FSDF_POSE_OVERLAP ? c->pose_stream : c->stream;
  if (FSDF_POSE_OVERLAP) HIPCHECK(c, hipStreamWaitEvent(ps, c->ev_pm_free[b], 0));
  if (!posed) {
    int rc = upload_poses(c, poses, ps);
    if (rc) return rc;
    HIPCHECK(c, fsdf::launch_pose(c->precision, c->lm, c->d_poses, *P, ps,
                                  c->lm.S <= fsdf::kPoseArgMax ? poses : nullptr));
  }
  if (FSDF_POSE_OVERLAP) {
    HIPCHECK(c, hipEventRecord(c->ev_pose, ps));
    HIPCHECK(c, hipStreamWaitEvent(c->stream, c->ev_pose, 0));
  }
  *out = P;
  *buf = b;
  return FSDF_OK;
}

static int release_posed(fsdf_ctx* c, int buf) {
  if (FSDF_POSE_OVERLAP) HIPCHECK(c, hipEventRecord(c->ev_pm_free[buf], c->stream));
  return FSDF_OK;
}


static int ensure_chunk_outputs(fsdf_ctx* c, int64_t nc) {
  if (c->co_cap >= nc && c->co_s >= c->lm.S) return FSDF_OK;
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  dfree(c->co.hdr);
  dfree(c->co.ent);  // (csum and dense live in the same allocation)
  dfree(c->co.dur);
  dfree(c->d_plan_order);
  c->co.csum = c->co.dense = nullptr;
  c->co_cap = 0;
  c->plan_nc = -1;
  HIPCHECK(c, hipMalloc(&c->co.hdr, (size_t)nc * 4 * sizeof(int32_t)));
  // one allocation: entries [nc][24] | Σ d² [nc] | dense rows [nc][S][6] (sized by the surface count:
  // (25 + 6 S) doubles per chunk, 1.6 KB at S = 64 — per context, so two in flight hold it twice)
  HIPCHECK(c, hipMalloc(&c->co.ent, (size_t)nc * (24 + 1 + 6 * (size_t)c->lm.S) * sizeof(double)));
  c->co_s = c->lm.S;
  c->co.csum = c->co.ent + (size_t)nc * 24;
  c->co.dense = c->co.ent + (size_t)nc * 25;
  c->co.cap = nc;
  HIPCHECK(c, hipMalloc(&c->co.dur, (size_t)nc * sizeof(uint32_t)));
  HIPCHECK(c, hipMalloc(&c->d_plan_order, (size_t)nc * sizeof(int32_t)));
  c->co_cap = nc;
  return FSDF_OK;
}

// the plan's composition for nc chunks: n4 chunks over 4 waves, n2 over 2,
// the rest one wave each. The heaviest `plan_f4` / `plan_f2` shares are split,
// and at least as many chunks over 4 waves as the device's idle wave slots
// allow (slots - nc, 3 extra waves per split chunk): a strong-scaling shard
// that leaves slots free splits its heavy third, a full machine only its tail.
static int wave_slots(fsdf_ctx* c) {
  if (c->wave_slots == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus <= 0)
      cus = 256;
    c->wave_slots = cus * 4 * 4;  // 4 SIMDs x 4 waves (the pass's register budget)
  }
  return c->wave_slots;
}

static void plan_shape(fsdf_ctx* c, int64_t nc, int* n4, int* n2) {
  wave_slots(c);
  const int64_t spare = std::max<int64_t>(0, (int64_t)c->wave_slots - nc);
  // default (shares < 0): fixed counts — the heavy tail that outlasts the rest
  // of a pass is ~100 chunks at 2^18 and at 2^19 points alike (measured)
  const int64_t want4 = c->plan_f4 < 0 ? kPlanDefault4 : llround(c->plan_f4 * (double)nc);
  const int64_t want2 = c->plan_f2 < 0 ? kPlanDefault2 : llround(c->plan_f2 * (double)nc);
  const int64_t a = std::min<int64_t>(nc, std::max<int64_t>(want4, spare / 3));
  *n4 = (int)a;
  *n2 = (int)std::min<int64_t>(nc - a, want2);
}

// The planned pass of a resident cloud: per-chunk partial rows, the
// two-level chunk reduction (16-chunk groups, then the tile reduce), and a
// plan rebuilt from this pass's chunk durations on the first pass of a cloud
// and then every kOrderEvery passes.
static int run_planned(fsdf_ctx* c, const fsdf::PosedModel& P, const void* d_pts, int64_t n, double* d_accum,
                       fsdf::PassOutputs& out, hipEvent_t* pe, const int* skip) {
  const int64_t nc = (n + 63) / 64;
  int rc = ensure_chunk_outputs(c, nc);
  if (rc) return rc;
  rc = ensure_partials(c, (int)std::max<int64_t>(fsdf::pass_blocks(n, c->lm), fsdf::reduce_chunk_groups(nc)));
  if (rc) return rc;
  out.partials = c->d_partials;
  out.cost = nullptr;
  out.order = nullptr;
  fsdf::ChunkOutputs co = c->co;
  // the split speed-ups behind the serial-equivalent durations (plan order,
  // fsdf_chunk_costs, the shard rebalance): M64-class scenes (>= 32 hulls)
  // measured 1.82-1.87x at 4 waves and 1.28-1.33x at 2 (tools/split_speedup.py,
  // profiles/r05/split_speedup.jsonl); IRB140-class measurements scattered
  // (4-way 1.22-1.53x) and their plan ran slower with them (profiles/r05/
  // keyed_plan), so those keep round 4's 5/2 and 8/5
  if (c->lm.K >= 32) {
    co.r4n = 15; co.r4d = 8; co.r2n = 4; co.r2d = 3;
  }
  const bool planned = c->plan_nc == nc && c->plan_grid > 0;
  co.plan = planned ? c->d_plan : nullptr;
  const int dparts = fsdf::hpart_parts(c->lm, n);
  co.dparts = dparts ? dparts : 1;
  const int grid = planned ? c->plan_grid : (int)((nc * co.dparts + 3) / 4);
  HIPCHECK(c, fsdf::launch_planned_pass(c->precision, c->cull != 0, c->lm, P, d_pts, n, grid, out, co, c->stream,
                                        pe ? pe[0] : nullptr, pe ? pe[1] : nullptr));
  c->pass_kernel = fsdf::last_pass_kernel();
  HIPCHECK(c, fsdf::launch_reduce_chunks(co, nc, c->lm.S, c->d_partials, d_accum, c->stream, pe ? pe[2] : nullptr,
                                         skip));
  if (!planned || ++c->plan_age >= kOrderEvery) {
    int n4, n2;
    plan_shape(c, nc, &n4, &n2);
    const int64_t g = n4 + (n2 + 1) / 2 + (nc - n4 - n2 + 3) / 4;
    if (c->plan_cap < g) {
      HIPCHECK(c, hipStreamSynchronize(c->stream));
      dfree(c->d_plan);
      c->plan_cap = 0;
      HIPCHECK(c, hipMalloc(&c->d_plan, (size_t)g * 4 * sizeof(int32_t)));
      c->plan_cap = g;
    }
    HIPCHECK(c, fsdf::launch_plan(c->co.dur, nc, n4, n2, c->d_plan_order, c->d_plan, c->stream));
    c->plan_grid = (int)g;
    c->plan_nc = nc;
    c->plan_age = 0;
  }
  return FSDF_OK;
}

// schedule: resident-cloud passes (repeated over the same cloud) launch their
// workgroups heaviest-first by the previous pass's durations
// posed / skip: the device solver loop's pass — its model posed by the
// previous step (pose_model), its done flag
static int run_pass_impl(fsdf_ctx* c, const double* poses, const void* d_pts, int64_t n, double* d_accum,
                         int32_t* d_kstar, double* d_d, double* d_grad, const int32_t* d_perm, bool schedule,
                         bool posed, const int* skip) {
  if (c->lm.R > 0 && !c->rbf_ready)
    return fail(c, FSDF_ERR_STATE, "eval: the scene has RBF surfaces: call fsdf_set_rbf_params first");
  fsdf::PosedModel* P = nullptr;
  int pbuf = 0;
  int rc = pose_model(c, poses, &P, &pbuf, posed);
  if (rc) return rc;
  const bool resident = d_pts == c->d_pts && n == c->n;
  const int nblocks = fsdf::pass_blocks(n, c->lm);
  rc = ensure_partials(c, nblocks);
  if (rc) return rc;
  fsdf::PassOutputs out;
  out.partials = c->d_partials;
  out.kstar = d_kstar;
  out.d = d_d;
  out.grad = d_grad;
  out.perm = d_perm;
  out.stats = c->stats_on ? c->d_stats : nullptr;
  out.skip = skip;
  out.chunk_ws = FSDF_CHUNK_WS && resident ? c->d_chunk_ws : nullptr;  // resident cloud only
  // the previous pass's nearest surfaces as seeds (resident cloud, hull-only
  // scenes of <= 64 surfaces; fsdf_internal.h PassOutputs::prior_in); marked
  // written (prior_ok) once the pass is launched — stream-ordered, the next
  // pass reads what this one writes
  const bool prior = FSDF_PRIOR_SEEDS && resident && n > 0 && c->d_prior && c->prior_cap >= n && c->lm.R == 0 &&
                     c->lm.S <= 64;
  out.prior_out = prior ? c->d_prior : nullptr;
  out.prior_in = prior && c->prior_ok ? c->d_prior : nullptr;
  // planned window: (default min, model's default max], or (0, max_points] when set
  const int64_t plan_max = c->plan_max_points >= 0 ? c->plan_max_points : fsdf::planned_default_max_points(c->lm);
  const int64_t plan_min = c->plan_max_points >= 0 ? 0 : fsdf::planned_default_min_points();
  if (schedule && n > plan_min && c->plan_enable && n <= plan_max && c->precision == 64 &&
      fsdf::planned_pass(c->lm, n)) {
    const bool prof = c->profiling && c->prof_used + 3 <= c->prof_ev.size();
    hipEvent_t* pe = prof ? &c->prof_ev[c->prof_used] : nullptr;
    rc = run_planned(c, *P, d_pts, n, d_accum, out, pe, skip);
    if (rc) return rc;
    if (prior) c->prior_ok = true;
    if (resident) c->last_pass_shape = 3;
    if (prof) c->prof_used += 3;
    return release_posed(c, pbuf);
  }
  const int ol = c->regrouped ? 1 : 0;  // (the layout's block order)
  if (schedule && n > 0) {
    if (!c->d_block_cost) {
      HIPCHECK(c, hipMalloc(&c->d_block_cost, fsdf::kMaxBlocks * sizeof(uint32_t)));
      HIPCHECK(c, hipMalloc(&c->d_block_order[0], fsdf::kMaxBlocks * sizeof(int32_t)));
      HIPCHECK(c, hipMalloc(&c->d_block_order[1], fsdf::kMaxBlocks * sizeof(int32_t)));
    }
    out.cost = c->d_block_cost;
    out.order = c->order_nblocks[ol] == nblocks ? c->d_block_order[ol] : nullptr;
  }
  if (n > 0) {
    // profiling: the pass kernel's start / end and the reduce's end, stamped
    // by the dispatches themselves (no packets of their own between kernels)
    const bool prof = c->profiling && c->prof_used + 3 <= c->prof_ev.size();
    hipEvent_t* pe = prof ? &c->prof_ev[c->prof_used] : nullptr;
    HIPCHECK(c, fsdf::launch_pass(c->precision, c->cull != 0, c->lm, *P, d_pts, n, nblocks, out, c->stream,
                                  pe ? pe[0] : nullptr, pe ? pe[1] : nullptr));
    c->pass_kernel = fsdf::last_pass_kernel();
    if (prior) c->prior_ok = true;
    if (resident) c->last_pass_shape = fsdf::hpart_pass(c->lm, n) ? 2 : 1;
    rc = release_posed(c, pbuf);
    if (rc) return rc;
    if (prof) c->prof_used += 3;
    // the order is rebuilt on the first scheduled pass of a grid and then every
    // kOrderEvery passes (the heavy blocks of a cloud stay heavy from pass to
    // pass; the rebuild is a ~7 us single-workgroup sort on the reduce launch)
    const bool rebuild = out.cost && (c->order_nblocks[ol] != nblocks || ++c->order_age[ol] >= kOrderEvery);
    HIPCHECK(c, fsdf::launch_reduce(c->d_partials, nblocks, accum_len(c), d_accum, c->stream,
                                    rebuild ? out.cost : nullptr, rebuild ? c->d_block_order[ol] : nullptr,
                                    pe ? pe[2] : nullptr, skip));
    if (rebuild) {
      c->order_nblocks[ol] = nblocks;
      c->order_age[ol] = 0;
    }
  } else {
    rc = release_posed(c, pbuf);
    if (rc) return rc;
    HIPCHECK(c, hipMemsetAsync(d_accum, 0, (size_t)accum_len(c) * sizeof(double), c->stream));
  }
  return FSDF_OK;
}

// A pass, then a prefetch still to be issued (fsdf_prefetch_points): its copy,
// sort launches and their host-side cost go behind this pass, which the device
// is already running (profiles/r06/prefetch_defer/). Its result waits for
// fsdf_set_points_prefetched.
static int run_pass(fsdf_ctx* c, const double* poses, const void* d_pts, int64_t n, double* d_accum,
                    int32_t* d_kstar, double* d_d, double* d_grad, const int32_t* d_perm, bool schedule,
                    bool posed = false, const int* skip = nullptr) {
  const int rc = run_pass_impl(c, poses, d_pts, n, d_accum, d_kstar, d_d, d_grad, d_perm, schedule, posed, skip);
  if (!rc && c->prefetch_deferred) c->prefetch_rc = prefetch_issue(c);
  return rc;
}

// per-point outputs of resident-cloud passes: scattered to caller order through
// the sort permutation, or written in resident order (coalesced)
// (a ranged cloud, fsdf_set_points_range: always resident order — its
// permutation names indices of the WHOLE cloud, beyond the outputs' length)
static const int32_t* out_perm(const fsdf_ctx* c) {
  return c->out_order == FSDF_ORDER_RESIDENT || c->ranged ? nullptr : c->d_perm;
}

extern "C" int fsdf_set_partition(fsdf_ctx* c, int64_t four_way_max_points, int64_t two_way_max_points) {
  if (!c) return FSDF_ERR_ARG;
  if (four_way_max_points < -1 || two_way_max_points < -1)
    return fail(c, FSDF_ERR_ARG, "set_partition: limits are -1 (model default), 0 (off) or a point count");
  c->lm.hpart4_points = four_way_max_points;
  c->lm.hpart2_points = two_way_max_points;
  return FSDF_OK;
}

extern "C" int fsdf_get_partition(fsdf_ctx* c, int64_t n, int64_t* four_way_max_out, int64_t* two_way_max_out,
                                  int32_t* parts_out) {
  if (!c) return FSDF_ERR_ARG;
  int64_t f4, f2;
  fsdf::hpart_default_limits(c->lm, &f4, &f2);
  if (c->lm.hpart4_points >= 0) f4 = c->lm.hpart4_points;
  if (c->lm.hpart2_points >= 0) f2 = c->lm.hpart2_points;
  if (four_way_max_out) *four_way_max_out = f4;
  if (two_way_max_out) *two_way_max_out = f2;
  if (parts_out) *parts_out = c->lm.K > 0 ? fsdf::hpart_parts(c->lm, n) : 0;
  return FSDF_OK;
}

extern "C" const char* fsdf_pass_kernel_name(const fsdf_ctx* c) { return c ? c->pass_kernel.c_str() : ""; }

extern "C" int fsdf_chunk_costs(fsdf_ctx* c, uint32_t* costs_out, int64_t* count_out) {
  if (!c || !count_out) return FSDF_ERR_ARG;
  // a regrouped range's chunks are no longer the whole cloud's Hilbert chunks:
  // costs balanced as if they were would place the cut by wrong prefix sums
  if (c->ranged && c->regrouped)
    return fail(c, FSDF_ERR_STATE, "chunk_costs: the ranged cloud was regrouped (its chunks are not the whole "
                                   "cloud's order); gather costs before fsdf_regroup_points");
  const int64_t nc = c->plan_nc > 0 ? c->plan_nc : 0;
  *count_out = nc;
  if (!costs_out || nc == 0) return FSDF_OK;
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  HIPCHECK(c, hipMemcpy(costs_out, c->co.dur, (size_t)nc * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return FSDF_OK;
}

extern "C" int fsdf_set_plan(fsdf_ctx* c, int32_t enable, double four_way_share, double two_way_share,
                             int64_t max_points) {
  if (!c) return FSDF_ERR_ARG;
  if (!(four_way_share <= 1.0 && two_way_share <= 1.0) || four_way_share != four_way_share || two_way_share != two_way_share)
    return fail(c, FSDF_ERR_ARG, "set_plan: shares must lie in [0, 1] (or < 0: the default counts)");
  if (max_points < -1) return fail(c, FSDF_ERR_ARG, "set_plan: max_points is -1 (default) or a point count");
  c->plan_enable = enable != 0;
  c->plan_f4 = four_way_share;
  c->plan_f2 = two_way_share;
  c->plan_max_points = max_points < 0 ? -1 : max_points;
  c->plan_nc = -1;  // rebuilt on the next pass
  return FSDF_OK;
}

extern "C" int fsdf_set_output_order(fsdf_ctx* c, int32_t order) {
  if (!c) return FSDF_ERR_ARG;
  if (order != FSDF_ORDER_CALLER && order != FSDF_ORDER_RESIDENT)
    return fail(c, FSDF_ERR_ARG, "set_output_order: unknown order %d", order);
  c->out_order = order;
  return FSDF_OK;
}

static int get_perm(fsdf_ctx* c, int64_t* out, bool device) {
  if (!c) return FSDF_ERR_ARG;
  if (c->n > 0 && !out) return fail(c, FSDF_ERR_ARG, "get_permutation: null output");
  HIPCHECK(c, hipSetDevice(c->device));
  if (c->n == 0) return FSDF_OK;
  if (c->d_perm) {
    std::vector<int32_t> p32;
    if (device) {
      HIPCHECK(c, fsdf::widen_permutation(c->d_perm, c->n, out, c->stream));
    } else {
      p32.resize((size_t)c->n);
      HIPCHECK(c, hipMemcpyAsync(p32.data(), c->d_perm, (size_t)c->n * sizeof(int32_t), hipMemcpyDeviceToHost,
                                 c->stream));
    }
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    for (size_t i = 0; i < p32.size(); ++i) out[i] = p32[i];
  } else if (device) {
    std::vector<int64_t> id((size_t)c->n);
    for (int64_t i = 0; i < c->n; ++i) id[(size_t)i] = i;
    HIPCHECK(c, hipMemcpy(out, id.data(), (size_t)c->n * sizeof(int64_t), hipMemcpyHostToDevice));
  } else {
    for (int64_t i = 0; i < c->n; ++i) out[i] = i;
  }
  return FSDF_OK;
}

extern "C" int fsdf_get_permutation(fsdf_ctx* c, int64_t* perm_out) { return get_perm(c, perm_out, false); }
extern "C" int fsdf_get_permutation_device(fsdf_ctx* c, int64_t* d_perm_out) { return get_perm(c, d_perm_out, true); }

extern "C" int fsdf_eval_device(fsdf_ctx* c, const double* poses, double* d_accum, int32_t* d_kstar, double* d_d,
                                double* d_grad) {
  if (!c) return FSDF_ERR_ARG;
  if (c->lm.S == 0) return fail(c, FSDF_ERR_STATE, "eval: no model (call fsdf_set_model first)");
  if (!poses || !d_accum) return fail(c, FSDF_ERR_ARG, "eval_device: poses and d_accum are required");
  HIPCHECK(c, hipSetDevice(c->device));
  return run_pass(c, poses, c->d_pts, c->n, d_accum, d_kstar, d_d, d_grad, out_perm(c), true);
}

static int ensure_outputs(fsdf_ctx* c, int64_t n) {
  if (c->out_cap >= n) return FSDF_OK;
  dfree(c->d_kstar);
  dfree(c->d_d);
  dfree(c->d_grad);
  c->out_cap = 0;
  HIPCHECK(c, hipMalloc(&c->d_kstar, (size_t)std::max<int64_t>(n, 1) * sizeof(int32_t)));
  HIPCHECK(c, hipMalloc(&c->d_d, (size_t)std::max<int64_t>(n, 1) * sizeof(double)));
  HIPCHECK(c, hipMalloc(&c->d_grad, (size_t)std::max<int64_t>(n, 1) * 3 * sizeof(double)));
  c->out_cap = n;
  return FSDF_OK;
}

// fsdf_value_and_gradient: the reduction kernel stores the accumulator into
// the pinned host buffer itself (no D2H copy command before the sync). Same
// results; full iteration -1.5 to -2.5 us against the pinned copy
// (profiles/r02/experiments/r02zc).
#ifndef FSDF_ZERO_COPY_ACCUM
#define FSDF_ZERO_COPY_ACCUM 1
#endif

static int ensure_host_acc(fsdf_ctx* c, int len) {
  if (len <= c->h_acc_cap) return FSDF_OK;
  if (c->h_acc) HIPCHECK(c, hipHostFree(c->h_acc));
  c->h_acc = nullptr;
  c->h_acc_cap = 0;
  HIPCHECK(c, hipHostMalloc((void**)&c->h_acc, (size_t)len * sizeof(double), hipHostMallocDefault));
  c->h_acc_cap = len;
  return FSDF_OK;
}

static int fetch(fsdf_ctx* c, int64_t n, double* cost_out, double* accum_out, int32_t* kstar_out, double* d_out,
                 double* grad_out, bool want_pp) {
  const int len = accum_len(c);
  int rc = ensure_host_acc(c, len);
  if (rc) return rc;
  double* acc = c->h_acc;
  HIPCHECK(c, hipMemcpyAsync(acc, c->d_accum, len * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (want_pp && n > 0) {
    if (kstar_out)
      HIPCHECK(c, hipMemcpyAsync(kstar_out, c->d_kstar, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    if (d_out) HIPCHECK(c, hipMemcpyAsync(d_out, c->d_d, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (grad_out)
      HIPCHECK(c, hipMemcpyAsync(grad_out, c->d_grad, n * 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  if (cost_out) *cost_out = acc[0];
  if (accum_out) memcpy(accum_out, acc, len * sizeof(double));
  return FSDF_OK;
}

extern "C" int fsdf_eval(fsdf_ctx* c, const double* poses, double* cost_out, double* accum_out, int32_t* kstar_out,
                         double* d_out, double* grad_out) {
  if (!c) return FSDF_ERR_ARG;
  if (c->lm.S == 0) return fail(c, FSDF_ERR_STATE, "eval: no model (call fsdf_set_model first)");
  if (!poses) return fail(c, FSDF_ERR_ARG, "eval: poses required");
  HIPCHECK(c, hipSetDevice(c->device));
  const bool want_pp = kstar_out || d_out || grad_out;
  if (want_pp) {
    int rc = ensure_outputs(c, c->n);
    if (rc) return rc;
  }
  int rc = run_pass(c, poses, c->d_pts, c->n, c->d_accum, want_pp ? c->d_kstar : nullptr,
                    want_pp ? c->d_d : nullptr, want_pp ? c->d_grad : nullptr, out_perm(c), true);
  if (rc) return rc;
  return fetch(c, c->n, cost_out, accum_out, kstar_out, d_out, grad_out, want_pp);
}

extern "C" int fsdf_set_mechanism(fsdf_ctx* c, int32_t nb, const int32_t* parent, const int32_t* kind,
                                  const int32_t* qoff, const double* axis, const double* AR, const double* At,
                                  const double* BR, const double* Bt, int32_t nq, const int32_t* surface_body,
                                  const double* frame_R, const double* frame_t) {
  if (!c) return FSDF_ERR_ARG;
  if (c->lm.S == 0) return fail(c, FSDF_ERR_STATE, "set_mechanism: set the surfaces first");
  if (nb < 1 || nq < 0 || !parent || !kind || !qoff || !axis || !AR || !At || !BR || !Bt || !surface_body ||
      !frame_R || !frame_t)
    return fail(c, FSDF_ERR_ARG, "set_mechanism: bad arguments");
  const int S = c->lm.S;
  for (int b = 1; b < nb; ++b) {
    if (parent[b] < 0 || parent[b] >= b) return fail(c, FSDF_ERR_ARG, "set_mechanism: bodies not in topological order");
    if (kind[b] < 0 || kind[b] > 2) return fail(c, FSDF_ERR_ARG, "set_mechanism: joint kind %d", kind[b]);
    const int width = kind[b] == 1 ? 1 : (kind[b] == 2 ? 7 : 0);
    if (width && (qoff[b] < 0 || qoff[b] + width > nq)) return fail(c, FSDF_ERR_ARG, "set_mechanism: q offset");
  }
  for (int k = 0; k < S; ++k)
    if (surface_body[k] < -1 || surface_body[k] >= nb) return fail(c, FSDF_ERR_ARG, "set_mechanism: surface body");
  auto& M = c->mech;
  M.nb = nb;
  M.nq = nq;
  M.parent.assign(parent, parent + nb);
  M.kind.assign(kind, kind + nb);
  M.qoff.assign(qoff, qoff + nb);
  M.surface_body.assign(surface_body, surface_body + S);
  M.axis.assign(axis, axis + 3 * nb);
  M.AR.assign(AR, AR + 9 * nb);
  M.At.assign(At, At + 3 * nb);
  M.BR.assign(BR, BR + 9 * nb);
  M.Bt.assign(Bt, Bt + 3 * nb);
  M.frame_R.assign(frame_R, frame_R + 9 * S);
  M.frame_t.assign(frame_t, frame_t + 3 * S);
  M.R.resize(9 * nb);
  M.t.resize(3 * nb);
  M.Rb.resize(9 * nb);
  M.tb.resize(3 * nb);
  M.poses.resize(12 * S);
  M.work.resize(6 * nb);
  M.rbf.clear();  // centre declarations name bodies of the previous tree
  M.x_prepared.clear();
  c->solver_tree_ok = false;
  return FSDF_OK;
}

extern "C" int fsdf_set_rbf_centres(fsdf_ctx* c, int32_t surface, int32_t n_sp, const int32_t* body_sp,
                                    const double* local_sp, const int32_t* deform_row_sp, int32_t n_sk,
                                    const int32_t* body_sk, const double* local_sk) {
  if (!c) return FSDF_ERR_ARG;
  auto& M = c->mech;
  if (M.nb == 0) return fail(c, FSDF_ERR_STATE, "set_rbf_centres: call fsdf_set_mechanism first");
  const int S = c->lm.S;
  if (surface < 0 || surface >= S || c->h_surface_kind[surface] != FSDF_SURFACE_RBF)
    return fail(c, FSDF_ERR_ARG, "set_rbf_centres: surface %d is not an RBF surface", surface);
  if (n_sp < 0 || n_sk < 0 || n_sp + n_sk != c->h_n_centers[surface] || (n_sp && (!body_sp || !local_sp)) ||
      (n_sk && (!body_sk || !local_sk)))
    return fail(c, FSDF_ERR_ARG, "set_rbf_centres: surface %d has %d centres, got %d + %d", surface,
                c->h_n_centers[surface], n_sp, n_sk);
  int r = 0;
  for (int k = 0; k < surface; ++k) r += c->h_surface_kind[k] == FSDF_SURFACE_RBF;
  M.rbf.resize(c->lm.R);
  auto& D = M.rbf[r];
  const int n = n_sp + n_sk;
  D.n_sp = n_sp;
  D.n = n;
  D.body.resize(n);
  D.drow.assign(n, -1);
  D.local.resize(3 * n);
  D.values.resize(n);
  for (int j = 0; j < n; ++j) {
    const bool sp = j < n_sp;
    const int b = sp ? body_sp[j] : body_sk[j - n_sp];
    if (b < -1 || b >= M.nb) return fail(c, FSDF_ERR_ARG, "set_rbf_centres: centre %d body %d", j, b);
    D.body[j] = b;
    if (sp && deform_row_sp) D.drow[j] = deform_row_sp[j];
    if (D.drow[j] < -1) return fail(c, FSDF_ERR_ARG, "set_rbf_centres: centre %d deformation row", j);
    const double* p = sp ? local_sp + 3 * j : local_sk + 3 * (j - n_sp);
    for (int i = 0; i < 3; ++i) D.local[3 * j + i] = p[i];
    D.values[j] = sp ? 0.0 : -1.0;  // src/Flash.jl:208-211
  }
  D.centres.resize(3 * n);
  D.u.resize(n + 4);
  D.lu.resize((size_t)(n + 4) * (n + 4));
  D.piv.resize(n + 4);
  D.G.resize(3 * n);
  D.work.resize(n + 4);
  return FSDF_OK;
}

extern "C" int fsdf_set_deformations(fsdf_ctx* c, int32_t n_deform, double weight) {
  if (!c) return FSDF_ERR_ARG;
  if (n_deform < 0 || !std::isfinite(weight)) return fail(c, FSDF_ERR_ARG, "set_deformations: bad arguments");
  c->mech.n_deform = n_deform;
  c->mech.weight = weight;
  return FSDF_OK;
}

// The host halves of one CostFunctor iteration at x (fsdf_value_and_gradient
// and its device-split form fsdf_eval_state_device + fsdf_state_gradient):
// prepare = FK, RBF centres + weight solve + rows upload, surface poses;
// finish = RBF adjoint, chain rule, regularizer from an accumulator.
// upload = false: the host part only (FK, RBF centres + weight solve, surface
// poses into c->mech) — fsdf_state_gradient re-prepares an earlier x so the
// chain rule runs on that pass's solve (pipelined passes, flash/distributed.py)
static int iteration_prepare(fsdf_ctx* c, const double* x, const char* who, bool upload = true) {
  auto& M = c->mech;
  if (M.nb == 0) return fail(c, FSDF_ERR_STATE, "%s: no mechanism (call fsdf_set_mechanism)", who);
  if ((int)M.surface_body.size() != c->lm.S || (int)M.poses.size() != 12 * c->lm.S)
    return fail(c, FSDF_ERR_STATE, "%s: mechanism registered for another surface list (call fsdf_set_mechanism)", who);
  const int R = c->lm.R;
  if (R > 0) {
    bool all = (int)M.rbf.size() == R;
    for (int r = 0; all && r < R; ++r) all = M.rbf[r].n > 0;
    if (!all) return fail(c, FSDF_ERR_STATE, "%s: declare every RBF surface's centres (fsdf_set_rbf_centres)", who);
    for (const auto& D : M.rbf)
      for (int j = 0; j < D.n; ++j)
        if (D.drow[j] >= M.n_deform)
          return fail(c, FSDF_ERR_STATE, "%s: deformation row %d >= %d (fsdf_set_deformations)", who, D.drow[j],
                      M.n_deform);
  }
  HIPCHECK(c, hipSetDevice(c->device));
  // forward kinematics (quaternion blocks normalized inside: normalize!, src/gradientdescent.jl:30)
  int rc = fsdf_tree_transforms(M.nb, M.parent.data(), M.kind.data(), M.qoff.data(), M.axis.data(), M.AR.data(),
                                M.At.data(), M.BR.data(), M.Bt.data(), x, M.R.data(), M.t.data(), M.Rb.data(),
                                M.tb.data());
  if (rc) return fail(c, rc, "%s: forward kinematics (bad configuration)", who);
  const double* delta = x + M.nq;
  // RBF skins: centres c = R_b (p + δ) + t_b, the weight solve, the rows
  // (flash/rbf.py solve / rows)
  if (R > 0) {
    M.rows.clear();
    for (auto& D : M.rbf) {
      for (int j = 0; j < D.n; ++j) {
        double p[3] = {D.local[3 * j], D.local[3 * j + 1], D.local[3 * j + 2]};
        if (D.drow[j] >= 0)
          for (int i = 0; i < 3; ++i) p[i] += delta[3 * D.drow[j] + i];
        const int b = D.body[j];
        for (int i = 0; i < 3; ++i)
          D.centres[3 * j + i] = b < 0 ? p[i]
                                       : (M.R[9 * b + 3 * i] * p[0] + M.R[9 * b + 3 * i + 1] * p[1] +
                                          M.R[9 * b + 3 * i + 2] * p[2]) + M.t[3 * b + i];
      }
      rc = fsdf_rbf_solve(D.n, D.centres.data(), D.values.data(), D.u.data(), D.lu.data(), D.piv.data());
      if (rc) return fail(c, rc, "%s: singular RBF system", who);
      for (int j = 0; j < D.n; ++j) {
        M.rows.insert(M.rows.end(), D.centres.begin() + 3 * j, D.centres.begin() + 3 * j + 3);
        M.rows.push_back(D.u[j]);
      }
      M.rows.insert(M.rows.end(), D.u.begin() + D.n, D.u.end());
    }
    if (upload) {
      rc = fsdf_set_rbf_params(c, M.rows.data(), (int64_t)M.rows.size());
      if (rc) return rc;
    }
  }
  // surface poses T_world_body · T_body_geometry (identity for surfaces without
  // a body; kin_impl.h, the device solver's arithmetic too)
  const int S = c->lm.S;
  for (int k = 0; k < S; ++k) {
    double* P = M.poses.data() + 12 * k;
    const int b = M.surface_body[k];
    if (b < 0) {
      for (int i = 0; i < 12; ++i) P[i] = (i % 4 == 0 && i < 9) ? 1.0 : 0.0;
      continue;
    }
    fsdf::kin::surface_pose(M.R.data() + 9 * b, M.t.data() + 3 * b, M.frame_R.data() + 9 * k,
                            M.frame_t.data() + 3 * k, P);
  }
  M.x_prepared.assign(x, x + M.nq + 3 * M.n_deform);
  return FSDF_OK;
}

static int iteration_finish(fsdf_ctx* c, const double* x, const double* accum, double* cost_out, double* grad_out,
                            const char* who) {
  auto& M = c->mech;
  const int R = c->lm.R, S = c->lm.S;
  const double* delta = x + M.nq;
  for (int i = 0; i < M.nq + 3 * M.n_deform; ++i) grad_out[i] = 0.0;
  // RBF chain (flash/rbf.py chain): G_j = ∂c/∂c_j through the solve -> body
  // wrenches (F, M about the world origin; δc = -(ω·M + v·F)) and ∂c/∂δ
  if (R > 0) {
    M.body_wrench.assign(6 * M.nb, 0.0);
    const double* block = accum + 1 + 6 * S;
    for (auto& D : M.rbf) {
      const int rc = fsdf_rbf_adjoint(D.n, D.centres.data(), D.u.data(), D.lu.data(), D.piv.data(), block,
                                      D.G.data(), D.work.data());
      if (rc) return fail(c, rc, "%s: RBF adjoint", who);
      block += 4 * D.n + 4;
      for (int j = 0; j < D.n; ++j) {
        const double* G = D.G.data() + 3 * j;
        const double* cj = D.centres.data() + 3 * j;
        const int b = D.body[j];
        if (b >= 0) {
          double* w = M.body_wrench.data() + 6 * b;
          w[0] -= G[0];
          w[1] -= G[1];
          w[2] -= G[2];
          w[3] -= cj[1] * G[2] - cj[2] * G[1];
          w[4] -= cj[2] * G[0] - cj[0] * G[2];
          w[5] -= cj[0] * G[1] - cj[1] * G[0];
        }
        if (D.drow[j] >= 0) {  // c_j = R_b (p_j + δ_j) + t_b
          double* gd = grad_out + M.nq + 3 * D.drow[j];
          for (int i = 0; i < 3; ++i)
            gd[i] += b < 0 ? G[i] : (M.R[9 * b + i] * G[0] + M.R[9 * b + 3 + i] * G[1] + M.R[9 * b + 6 + i] * G[2]);
        }
      }
    }
  }
  const int rc = fsdf_config_gradient(M.nb, M.parent.data(), M.kind.data(), M.qoff.data(), M.axis.data(),
                                      M.Rb.data(), M.tb.data(), x, S, M.surface_body.data(), accum + 1,
                                      R > 0 ? M.body_wrench.data() : nullptr, M.work.data(), grad_out);
  if (rc) return fail(c, rc, "%s: chain rule", who);
  // the deformation regularizer weight Σ|δ|^2 (src/gradientdescent.jl:33-37)
  double reg = 0.0;
  for (int i = 0; i < 3 * M.n_deform; ++i) {
    reg += delta[i] * delta[i];
    grad_out[M.nq + i] += 2.0 * M.weight * delta[i];
  }
  *cost_out = accum[0] + M.weight * reg;
  return FSDF_OK;
}

// diagnostic builds (-DFSDF_HOST_TIMES=1): host-side clocks of the host solver
// loop's iterations — prepare (FK, poses), launches, the wait, the chain rule —
// summed here and printed by fsdf_descend (stderr), to split the GPU's idle
// gap between iterations into host work and synchronisation latency
#if FSDF_HOST_TIMES
#include <chrono>
static double g_host_t[8];
static long g_host_n;
static inline double host_now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define HOST_STAMP(i) const double ht_##i = host_now_us()
#else
#define HOST_STAMP(i)
#endif

extern "C" int fsdf_value_and_gradient(fsdf_ctx* c, const double* x, double* cost_out, double* grad_out) {
  if (!c) return FSDF_ERR_ARG;
  HOST_STAMP(0);
  if (!x || !cost_out || !grad_out) return fail(c, FSDF_ERR_ARG, "value_and_gradient: null argument");
  int rc = iteration_prepare(c, x, "value_and_gradient");
  if (rc) return rc;
  auto& M = c->mech;
#if FSDF_ZERO_COPY_ACCUM
  // the reduction stores the accumulator straight into pinned host memory
  rc = ensure_host_acc(c, accum_len(c));
  if (rc) return rc;
  double* d_acc_host = nullptr;
  HIPCHECK(c, hipHostGetDevicePointer((void**)&d_acc_host, c->h_acc, 0));
  HOST_STAMP(1);
  rc = run_pass(c, M.poses.data(), c->d_pts, c->n, d_acc_host, nullptr, nullptr, nullptr, nullptr, true);
  if (rc) return rc;
  HOST_STAMP(2);
  rc = iteration_regroup(c);  // (stream-ordered after the pass: the sync below covers it)
  if (rc) return rc;
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  HOST_STAMP(3);
  rc = iteration_finish(c, x, c->h_acc, cost_out, grad_out, "value_and_gradient");
#if FSDF_HOST_TIMES
  HOST_STAMP(4);
  g_host_t[0] += ht_1 - ht_0;  // prepare
  g_host_t[1] += ht_2 - ht_1;  // pose + pass + reduce launches
  g_host_t[2] += ht_3 - ht_2;  // wait (device work + wake-up)
  g_host_t[3] += ht_4 - ht_3;  // chain rule
  ++g_host_n;
#endif
  return rc;
#else
  rc = run_pass(c, M.poses.data(), c->d_pts, c->n, c->d_accum, nullptr, nullptr, nullptr, nullptr, true);
  if (rc) return rc;
  rc = iteration_regroup(c);
  if (rc) return rc;
  M.accum.resize(accum_len(c));
  rc = fetch(c, c->n, nullptr, M.accum.data(), nullptr, nullptr, nullptr, false);
  if (rc) return rc;
  return iteration_finish(c, x, M.accum.data(), cost_out, grad_out, "value_and_gradient");
#endif
}

// The solver loop of estimate_state (src/tracking.jl:16-26 with the
// NaiveSolver restated in flash/tracking.py) around fsdf_value_and_gradient,
// without a host-language round trip per iteration: f = c/n, g = (∂c/∂x / n)
// ./ divisors; stop when |g| < tolerance; else x += clamp(-rate g, ±max_step).
// The device arrays of the mechanism for the solver step (solver.hip) and
// the level schedules of its parallel FK (bodies by depth) and subtree sums
// (parents by height, children in descending index: the host's reverse
// topological loop adds them in that order).
static int build_solver_tree(fsdf_ctx* c) {
  auto& M = c->mech;
  const int nb = M.nb, S = c->lm.S;
  std::vector<int> depth(nb, 0), height(nb, 0), nchild(nb, 0);
  for (int b = 1; b < nb; ++b) depth[b] = depth[M.parent[b]] + 1;
  for (int b = nb - 1; b >= 1; --b) {
    const int p = M.parent[b];
    height[p] = std::max(height[p], height[b] + 1);
    ++nchild[p];
  }
  int D = 0, H = 0;
  for (int b = 1; b < nb; ++b) {
    D = std::max(D, depth[b]);
    if (nchild[b]) H = std::max(H, height[b]);
  }
  std::vector<int32_t> iv;  // parent | kind | qoff | depth_order | depth_off | height_order | height_off |
                            // child_off | child_list | surf_off | surf_list | surface_body
  auto put = [&](const std::vector<int32_t>& v) {
    const size_t at = iv.size();
    iv.insert(iv.end(), v.begin(), v.end());
    return at;
  };
  // dord / doff: every body's path from the root, its ancestors of depth 1 .. its own
  // (the device composes a body's chain in registers, one thread per body)
  std::vector<int32_t> dord, doff(1, 0), hord, hoff(1, 0), coff(1, 0), clist, soff(1, 0), slist;
  dord.reserve((size_t)nb * (size_t)(D + 1));
  for (int b = 0; b < nb; ++b) {
    std::vector<int32_t> path;
    for (int a = b; a > 0; a = M.parent[a]) path.push_back(a);
    dord.insert(dord.end(), path.rbegin(), path.rend());
    doff.push_back((int32_t)dord.size());
  }
  int widest = 0;  // the most parents at one height: the subtree sums run in one wave when 6x that fits
  // chains: every body but the root has at most one child (IRB140, M64's arms): body b's
  // subtree is the list b, child, grandchild, ... (dlist / dof), summed in one thread
  bool chains = true;
  for (int b = 1; b < nb; ++b) chains = chains && nchild[b] <= 1;
  std::vector<int32_t> dlist, dof(1, 0);
  if (chains) {
    std::vector<int32_t> child(nb, -1);
    for (int b = 1; b < nb; ++b)
      if (M.parent[b] > 0) child[M.parent[b]] = b;
    for (int b = 0; b < nb; ++b) {
      for (int a = b; b > 0 && a >= 0; a = child[a]) dlist.push_back(a);
      dof.push_back((int32_t)dlist.size());
    }
  }
  for (int h = 1; h <= H; ++h) {
    for (int b = 1; b < nb; ++b)
      if (nchild[b] && height[b] == h) hord.push_back(b);
    widest = std::max(widest, (int)hord.size() - hoff.back());
    hoff.push_back((int32_t)hord.size());
  }
  for (int p = 0; p < nb; ++p) {
    for (int b = nb - 1; b > p; --b)
      if (M.parent[b] == p) clist.push_back(b);
    coff.push_back((int32_t)clist.size());
    for (int k = 0; k < S; ++k)
      if (M.surface_body[k] == p) slist.push_back(k);
    soff.push_back((int32_t)slist.size());
  }
  const size_t o_parent = put(M.parent), o_kind = put(M.kind), o_qoff = put(M.qoff), o_dord = put(dord),
               o_doff = put(doff), o_hord = put(hord), o_hoff = put(hoff), o_coff = put(coff), o_clist = put(clist),
               o_soff = put(soff), o_slist = put(slist), o_sb = put(M.surface_body), o_dlist = put(dlist),
               o_dof = put(dof);
  std::vector<double> dv;
  auto putd = [&](const std::vector<double>& v) {
    const size_t at = dv.size();
    dv.insert(dv.end(), v.begin(), v.end());
    return at;
  };
  const size_t o_axis = putd(M.axis), o_AR = putd(M.AR), o_At = putd(M.At), o_BR = putd(M.BR), o_Bt = putd(M.Bt),
               o_FR = putd(M.frame_R), o_Ft = putd(M.frame_t);
  HIPCHECK(c, hipStreamSynchronize(c->stream));  // (a previous frame's steps may still read the old arrays)
  dfree(c->d_stree_d);
  const size_t bytes = dv.size() * sizeof(double) + iv.size() * sizeof(int32_t);
  const size_t chunks = (bytes + 15) / 16;
  std::vector<char> blob(chunks * 16, 0);
  memcpy(blob.data(), dv.data(), dv.size() * sizeof(double));
  memcpy(blob.data() + dv.size() * sizeof(double), iv.data(), iv.size() * sizeof(int32_t));
  HIPCHECK(c, hipMalloc(&c->d_stree_d, std::max<size_t>(blob.size(), 16)));
  HIPCHECK(c, hipMemcpy(c->d_stree_d, blob.data(), blob.size(), hipMemcpyHostToDevice));
  fsdf::SolverTree& T = c->stree;
  T.nb = nb;
  T.nx = M.nq;
  T.S = S;
  T.D = D;
  T.H = H;
  T.blob = c->d_stree_d;
  T.ni = (int)iv.size();
  T.nd = (int)dv.size();
  T.chunks16 = (int)chunks;
  T.parent = (int)o_parent;
  T.kind = (int)o_kind;
  T.qoff = (int)o_qoff;
  T.path_list = (int)o_dord;
  T.path_off = (int)o_doff;
  T.narrow = 6 * widest <= 64;
  T.chains = chains;
  T.chain_list = (int)o_dlist;
  T.chain_off = (int)o_dof;
  T.height_order = (int)o_hord;
  T.height_off = (int)o_hoff;
  T.child_off = (int)o_coff;
  T.child_list = (int)o_clist;
  T.surf_off = (int)o_soff;
  T.surf_list = (int)o_slist;
  T.surface_body = (int)o_sb;
  T.axis = (int)o_axis;
  T.AR = (int)o_AR;
  T.At = (int)o_At;
  T.BR = (int)o_BR;
  T.Bt = (int)o_Bt;
  T.frame_R = (int)o_FR;
  T.frame_t = (int)o_Ft;
  c->solver_tree_ok = true;
  return FSDF_OK;
}

// fsdf_descend for rigid scenes, every iteration on the device: solver_init
// (FK of x0 -> poses), then per iteration pose -> pass -> reduce -> solver
// step, all enqueued up front; one read-back of x, f and the count at the end.
// Bit-identical to the host loop below (solver.hip).
static int descend_device(fsdf_ctx* c, double* x, int32_t iteration_limit, double rate, double max_step,
                          double tolerance, const double* divisors, double n_points, double* value_out,
                          int32_t* iterations_out) {
  auto& M = c->mech;
  const int nx = M.nq, nb = M.nb;
  HIPCHECK(c, hipSetDevice(c->device));
  if (!c->solver_tree_ok) {
    const int rc = build_solver_tree(c);
    if (rc) return rc;
  }
  // device: x [2][nx] (slots by iteration parity) | div [nx] | Rb|tb [2][12 nb] | f; flags [4] int
  const size_t need = (size_t)3 * nx + 24 * (size_t)nb + 1;
  if (c->solver_cap < need) {
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    dfree(c->d_solver);
    c->solver_cap = 0;
    HIPCHECK(c, hipMalloc(&c->d_solver, need * sizeof(double)));
    c->solver_cap = need;
  }
  if (!c->d_solver_flags) HIPCHECK(c, hipMalloc(&c->d_solver_flags, 4 * sizeof(int)));
  // pinned: x [2][nx] | div [nx] | f | flags [4] (as 2 doubles)
  const size_t hneed = (size_t)3 * nx + 3;
  if (c->h_solver_cap < hneed) {
    if (c->h_solver) HIPCHECK(c, hipHostFree(c->h_solver));
    c->h_solver = nullptr;
    c->h_solver_cap = 0;
    HIPCHECK(c, hipHostMalloc((void**)&c->h_solver, hneed * sizeof(double), hipHostMallocDefault));
    c->h_solver_cap = hneed;
  }
  double* h = c->h_solver;
  HIPCHECK(c, hipStreamSynchronize(c->stream));  // (the pinned staging of an earlier frame is free)
  memcpy(h, x, (size_t)nx * sizeof(double));  // (slot 0)
  if (divisors) memcpy(h + 2 * nx, divisors, (size_t)nx * sizeof(double));
  HIPCHECK(c, hipMemcpyAsync(c->d_solver, h, (size_t)(divisors ? 3 : 1) * nx * sizeof(double),
                             hipMemcpyHostToDevice, c->stream));
  fsdf::SolverState st;
  st.x = c->d_solver;
  st.div = divisors ? c->d_solver + 2 * nx : nullptr;
  st.Rb = c->d_solver + 3 * nx;
  st.f = st.Rb + 24 * nb;
  st.flags = c->d_solver_flags;
  st.rate = rate;
  st.max_step = max_step;
  st.tol = tolerance;
  st.n_points = n_points;
  st.weight = M.weight;
  st.limit = iteration_limit;
  HIPCHECK(c, hipMemsetAsync(c->d_solver_flags, 0, 4 * sizeof(int), c->stream));
  // (the init and every step pose the next pass's model themselves: the
  // passes below launch no pose kernel; FSDF_POSE_OVERLAP is off, c->pm is
  // the one posed model)
  HIPCHECK(c, fsdf::launch_solver_init(c->stree, st, c->lm, c->pm, c->precision, c->stream));
  HOST_STAMP(0);
  for (int it = 0; it < iteration_limit; ++it) {
    int rc = run_pass(c, nullptr, c->d_pts, c->n, c->d_accum, nullptr, nullptr, nullptr, nullptr, true, true,
                      st.flags);
    if (rc) return rc;
    if (it == 0) {
      rc = iteration_regroup(c);
      if (rc) return rc;
    }
    HIPCHECK(c, fsdf::launch_solver_step(c->stree, st, c->d_accum, c->lm, c->pm, c->precision, it, c->stream));
  }
  HOST_STAMP(1);
  HIPCHECK(c, hipMemcpyAsync(h, st.x, (size_t)2 * nx * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(c, hipMemcpyAsync(h + 3 * nx, st.f, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(c, hipMemcpyAsync(h + 3 * nx + 1, st.flags, 4 * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(c, hipStreamSynchronize(c->stream));
#if FSDF_HOST_TIMES
  HOST_STAMP(2);
  fprintf(stderr, "device loop: enqueue %.1f us (%d iterations), then wait %.1f us\n", ht_1 - ht_0, iteration_limit,
          ht_2 - ht_1);
#endif
  int flags[4];
  memcpy(flags, h + 3 * nx + 1, sizeof flags);
#ifdef FSDF_SOLVER_TIMES
  {
    unsigned long long tt[16];
    fsdf::solver_times(tt);
    fprintf(stderr, "solver step phases (10 ns):");
    for (int i = 1; i < 10; ++i) fprintf(stderr, " %lld", (long long)(tt[i] - tt[0]));
    fprintf(stderr, "\n");
  }
#endif
  memcpy(x, h + (size_t)(flags[1] & 1) * nx, (size_t)nx * sizeof(double));  // (the last iteration's slot)
  if (iterations_out) *iterations_out = flags[1];
  if (flags[2] == 2) return fail(c, FSDF_ERR_ARG, "descend: poses not finite (configuration diverged)");
  if (flags[2]) return fail(c, FSDF_ERR_ARG, "descend: forward kinematics / chain rule (bad configuration)");
  if (value_out) *value_out = h[3 * nx];
  return FSDF_OK;
}

extern "C" int fsdf_set_solver(fsdf_ctx* c, int32_t device_loop) {
  if (!c) return FSDF_ERR_ARG;
  if (device_loop < 0 || device_loop > 2) return fail(c, FSDF_ERR_ARG, "set_solver: mode %d", device_loop);
  c->solver_device = device_loop;
  return FSDF_OK;
}

extern "C" int fsdf_descend(fsdf_ctx* c, double* x, int32_t iteration_limit, double rate, double max_step,
                            double tolerance, const double* divisors, double n_points, double* value_out,
                            int32_t* iterations_out) {
  if (!c) return FSDF_ERR_ARG;
  if (iterations_out) *iterations_out = 0;
  if (!x || iteration_limit < 0 || !(n_points > 0.0) || !std::isfinite(rate) || !(max_step >= 0.0))
    return fail(c, FSDF_ERR_ARG, "descend: bad arguments");
  if (c->mech.nb == 0) return fail(c, FSDF_ERR_STATE, "descend: no mechanism (call fsdf_set_mechanism)");
  const auto& Mc = c->mech;
  if ((int)Mc.surface_body.size() != c->lm.S || (int)Mc.poses.size() != 12 * c->lm.S)
    return fail(c, FSDF_ERR_STATE, "descend: mechanism registered for another surface list (call fsdf_set_mechanism)");
  // rigid scenes (no RBF skin, no deformation) iterate on the device when the
  // mechanism's tree and the step's work arrays fit the step's LDS (M64's 65
  // bodies: ~45 KB)
  // (the step poses c->pm itself: not with the double-buffered pose overlap)
  bool device_loop = c->solver_device && iteration_limit > 0 && c->lm.R == 0 && Mc.n_deform == 0 && c->n > 0 &&
                     !FSDF_POSE_OVERLAP;
  if (device_loop && !c->solver_tree_ok) {
    HIPCHECK(c, hipSetDevice(c->device));
    const int rc = build_solver_tree(c);
    if (rc) return rc;
  }
  device_loop = device_loop && fsdf::solver_fits(Mc.nb, Mc.nq, c->lm.S, c->stree.ni);
  if (c->solver_device == 2 && iteration_limit > 0 && !device_loop)
    return fail(c, FSDF_ERR_STATE, "descend: the device loop was required (fsdf_set_solver 2) but the scene %s",
                c->lm.R > 0 || Mc.n_deform > 0 ? "has RBF skins / deformations" :
                c->n == 0 ? "has no resident points" : "does not fit the solver step's LDS");
  if (device_loop)
    return descend_device(c, x, iteration_limit, rate, max_step, tolerance, divisors, n_points, value_out,
                          iterations_out);
  const int ns = c->mech.nq + 3 * c->mech.n_deform;
  std::vector<double> g(ns);
  double f = 0.0;
  int it = 0;
#if FSDF_HOST_TIMES
  for (double& v : g_host_t) v = 0.0;
  g_host_n = 0;
  const double ht_start = host_now_us();
#endif
  while (it < iteration_limit) {
    double cost = 0.0;
    const int rc = fsdf_value_and_gradient(c, x, &cost, g.data());
    if (rc) return rc;
    ++it;
    if (iterations_out) *iterations_out = it;
    f = cost / n_points;
    double nrm2 = 0.0;
    for (int i = 0; i < ns; ++i) {
      double gi = g[i] / n_points;
      if (divisors) gi = gi / divisors[i];
      g[i] = gi;
      nrm2 += gi * gi;
    }
    if (std::sqrt(nrm2) < tolerance) break;
    for (int i = 0; i < ns; ++i) x[i] = x[i] + std::min(std::max(-rate * g[i], -max_step), max_step);
  }
#if FSDF_HOST_TIMES
  if (g_host_n > 0) {
    const double span = host_now_us() - ht_start, k = (double)g_host_n;
    fprintf(stderr, "host loop per iteration (us): prepare %.2f launches %.2f wait %.2f chain %.2f total %.2f (%ld)\n",
            g_host_t[0] / k, g_host_t[1] / k, g_host_t[2] / k, g_host_t[3] / k, span / k, g_host_n);
  }
#endif
  if (value_out) *value_out = f;
  return FSDF_OK;
}

extern "C" int fsdf_eval_state_device(fsdf_ctx* c, const double* x, double* d_accum) {
  if (!c) return FSDF_ERR_ARG;
  if (!x || !d_accum) return fail(c, FSDF_ERR_ARG, "eval_state_device: null argument");
  int rc = iteration_prepare(c, x, "eval_state_device");
  if (rc) return rc;
  rc = run_pass(c, c->mech.poses.data(), c->d_pts, c->n, d_accum, nullptr, nullptr, nullptr, nullptr, true);
  if (rc) return rc;
  rc = iteration_regroup(c);
  if (rc) return rc;
  auto& M = c->mech;
  M.x_pass[M.x_pass_next] = M.x_prepared;
  M.x_pass_next ^= 1;
  return FSDF_OK;
}

extern "C" int fsdf_state_gradient(fsdf_ctx* c, const double* x, const double* accum, double* cost_out,
                                   double* grad_out) {
  if (!c) return FSDF_ERR_ARG;
  if (!x || !accum || !cost_out || !grad_out) return fail(c, FSDF_ERR_ARG, "state_gradient: null argument");
  auto& M = c->mech;
  const size_t nx = (size_t)M.nq + 3 * (size_t)M.n_deform;
  // the chain rule runs on the FK / weight solve of the pass that produced
  // accum; for an x other than the last prepared one (a pipelined earlier
  // pass) that host part is redone — the same arithmetic, the same bits
  if (M.nb == 0) return fail(c, FSDF_ERR_STATE, "state_gradient: no mechanism (call fsdf_set_mechanism)");
  auto same = [&](const std::vector<double>& v) {
    return v.size() == nx && memcmp(v.data(), x, nx * sizeof(double)) == 0;
  };
  if (!same(M.x_prepared)) {
    // an earlier pass of the ring: its FK / weight solve is redone (the same
    // arithmetic, the same bits); any other x cannot belong to an accumulator
    // of this context
    if (!same(M.x_pass[0]) && !same(M.x_pass[1]))
      return fail(c, FSDF_ERR_STATE,
                  "state_gradient: x is not the configuration of either of this context's last two "
                  "eval_state_device passes (nor the last prepared one)");
    const int rc = iteration_prepare(c, x, "state_gradient", false);
    if (rc) return rc;
  }
  return iteration_finish(c, x, accum, cost_out, grad_out, "state_gradient");
}

extern "C" int fsdf_skin(fsdf_ctx* c, const double* poses, const double* xyz, int64_t n, double* d_out,
                         int32_t* kstar_out, double* grad_out) {
  if (!c) return FSDF_ERR_ARG;
  if (c->lm.S == 0) return fail(c, FSDF_ERR_STATE, "skin: no model (call fsdf_set_model first)");
  if (!poses || n < 0 || (n > 0 && !xyz)) return fail(c, FSDF_ERR_ARG, "skin: bad arguments");
  HIPCHECK(c, hipSetDevice(c->device));
  if (n == 0) return FSDF_OK;
  int rc = ensure_outputs(c, n);
  if (rc) return rc;
  // stage the query points (f64 on the device, then the context precision)
  if (c->q64_cap < n) {
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    dfree(c->d_q64);
    c->q64_cap = 0;
    HIPCHECK(c, hipMalloc(&c->d_q64, (size_t)n * 3 * sizeof(double)));
    c->q64_cap = n;
  }
  HIPCHECK(c, hipMemcpyAsync(c->d_q64, xyz, (size_t)n * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
  const void* d_query = c->d_q64;
  if (c->precision != 64) {
    rc = adopt_points_device(c, c->d_q64, n, &c->d_q, &c->q_cap);
    if (rc) return rc;
    d_query = c->d_q;
  }
  rc = run_pass(c, poses, d_query, n, c->d_accum, c->d_kstar, c->d_d, c->d_grad, nullptr, false);
  if (rc) return rc;
  return fetch(c, n, nullptr, nullptr, kstar_out, d_out, grad_out, true);
}

extern "C" int fsdf_synchronize(fsdf_ctx* c) {
  if (!c) return FSDF_ERR_ARG;
  HIPCHECK(c, hipSetDevice(c->device));
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  return FSDF_OK;
}

extern "C" int fsdf_profile_pass(fsdf_ctx* c, int32_t enable) {
  if (!c) return FSDF_ERR_ARG;
  HIPCHECK(c, hipSetDevice(c->device));
  if (enable && c->prof_ev.empty()) {
    c->prof_ev.resize(3 * 4096, nullptr);
    // timing-only events: a default event record is a system-scope release
    // (the whole L2 written back), which put ~10 us between the pass and the
    // reduce of every profiled pass; fsdf_pass_times synchronizes the stream
    // before reading them
    for (auto& e : c->prof_ev) HIPCHECK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  }
  c->profiling = enable != 0;
  c->prof_used = 0;
  return FSDF_OK;
}

extern "C" int fsdf_pass_times(fsdf_ctx* c, double* kernel_ms, double* pass_ms, int64_t* launches) {
  if (!c || !kernel_ms || !pass_ms || !launches) return FSDF_ERR_ARG;
  HIPCHECK(c, hipSetDevice(c->device));
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  double tk = 0.0, tp = 0.0;
  for (size_t i = 0; i + 2 < c->prof_used; i += 3) {
    float k = 0.f, p = 0.f;
    HIPCHECK(c, hipEventElapsedTime(&k, c->prof_ev[i], c->prof_ev[i + 1]));
    HIPCHECK(c, hipEventElapsedTime(&p, c->prof_ev[i], c->prof_ev[i + 2]));
    tk += k;
    tp += p;
  }
  *kernel_ms = tk;
  *pass_ms = tp;
  *launches = (int64_t)(c->prof_used / 3);
  c->prof_used = 0;
  return FSDF_OK;
}

extern "C" int fsdf_pass_time(fsdf_ctx* c, double* total_ms, int64_t* launches) {
  double k = 0.0;
  return fsdf_pass_times(c, &k, total_ms, launches);
}


#ifndef FSDF_WAVE_TIMES
#define FSDF_WAVE_TIMES 0
#endif
// 24 counters; diagnostic builds with -DFSDF_WAVE_TIMES=1 append per-wave clocks
static constexpr int kStatCount = FSDF_WAVE_TIMES ? 32 + 32 * fsdf::kMaxBlocks : 24;

extern "C" int fsdf_kernel_stats(fsdf_ctx* c, int32_t enable, uint64_t* counters) {
  if (!c) return FSDF_ERR_ARG;
  HIPCHECK(c, hipSetDevice(c->device));
  if (!c->d_stats) HIPCHECK(c, hipMalloc(&c->d_stats, kStatCount * sizeof(unsigned long long)));
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  if (enable) {
    HIPCHECK(c, hipMemset(c->d_stats, 0, kStatCount * sizeof(unsigned long long)));
    c->stats_on = true;
    return FSDF_OK;
  }
  c->stats_on = false;
  if (counters) HIPCHECK(c, hipMemcpy(counters, c->d_stats, kStatCount * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return FSDF_OK;
}

extern "C" int fsdf_raycast(fsdf_ctx* c, const double* poses, const double* origin, const double* rays, int64_t n,
                            double* depth_out) {
  if (!c) return FSDF_ERR_ARG;
  if (c->lm.S == 0) return fail(c, FSDF_ERR_STATE, "raycast: no model (call fsdf_set_surfaces first)");
  if (!poses || !origin || n < 0 || (n > 0 && (!rays || !depth_out))) return fail(c, FSDF_ERR_ARG, "raycast: bad arguments");
  if (c->lm.R > 0 && !c->rbf_ready)
    return fail(c, FSDF_ERR_STATE, "raycast: the scene has RBF surfaces: call fsdf_set_rbf_params first");
  for (int j = 0; j < 3; ++j)
    if (!std::isfinite(origin[j])) return fail(c, FSDF_ERR_ARG, "raycast: origin not finite");
  HIPCHECK(c, hipSetDevice(c->device));
  if (n == 0) return FSDF_OK;
  int rc = ensure_outputs(c, n);
  if (rc) return rc;
  if (c->q64_cap < n) {
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    dfree(c->d_q64);
    c->q64_cap = 0;
    HIPCHECK(c, hipMalloc(&c->d_q64, (size_t)n * 3 * sizeof(double)));
    c->q64_cap = n;
  }
  HIPCHECK(c, hipMemcpyAsync(c->d_q64, rays, (size_t)n * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
  fsdf::PosedModel* P = nullptr;
  int pbuf = 0;
  rc = pose_model(c, poses, &P, &pbuf);
  if (rc) return rc;
  HIPCHECK(c, fsdf::launch_raycast(c->precision, c->cull != 0, c->lm, *P, origin, c->d_q64, n, c->d_d, c->stream));
  rc = release_posed(c, pbuf);
  if (rc) return rc;
  HIPCHECK(c, hipMemcpyAsync(depth_out, c->d_d, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  return FSDF_OK;
}
