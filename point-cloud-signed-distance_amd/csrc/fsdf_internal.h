// Internal declarations shared by the kernel translation unit and the C-ABI.
// Device layouts (all per-evaluation "world" arrays are produced on the device
// by the pose kernel from the resident local model and the K poses):
//
//   local model (uploaded once by fsdf_set_model)
//     verts_l   [V][3]  f64     hull vertices, body frame
//     faces     [F][3]  i32     global vertex indices (CCW from outside)
//     planes_l  [F][4]  f64     (n, d), n·x <= d inside
//     face_hull [F]     i32     owning hull of each face
//     sphere_l  [K][4]  f64     vertex centroid (inside the hull) + radius
//     box_l     [K][8]  f64     body-frame bounding box: centre xyz, 0, half extents xyz
//                               (rounded up to f32), 0
//     face_off  [K+1]   i32     faces of hull k are [face_off[k], face_off[k+1])
//     vert_hull [V]     i32     owning hull of each vertex
//     vert_off  [K+1]   i32     vertices of hull k are [vert_off[k], vert_off[k+1])
//     face_rows [F][4]  i32     packed hull-local (v0|v1<<16, v2|n0<<16, n1|n2<<16, dup):
//                               vertex indices, the face across edge i (v_i -> v_{i+1}),
//                               dup = 1 if an earlier face of the hull has the same plane
//
//   posed model (rewritten by every evaluation; T = double or float)
//     planes_w  [F][4]  T       world plane
//     spheres_w [K][20] f32     culling bounds: world centroid + radius, then the world
//                               oriented box: (centre, 0), 3 x (body axis i, half extent i)
//     verts_w   [V][4]  T       world vertices (support/optimality certificate)
//     hscale_w  [K]     T       max_v |v|_1 over the hull's world vertices
//     screen_w  [F+K][4] f32    fp32 screening planes, hull-centred, in face pairs:
//                               hull k's pair j at slots face_off[k]+k+2j (32 B):
//                               (nx_a nx_b ny_a ny_b nz_a nz_b -d'_a -d'_b), a = 2j,
//                               b = 2j+1 (= a when nf is odd and j is the last pair),
//                               d' = d - n·c with c the hull's f32 sphere centre
//
//   per-block partial sums  partials [len/8][nblocks][8] f64 line tiles, len = 1+6S+Σ(4n+4)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fsdf {

// fp32-screened plane max in f64 contexts (sdf_kernels.hip screen_plane_max);
// it also fixes the f64 LDS stage layout (screening pairs instead of planes),
// so fsdf_set_surfaces sizes the stage from the same switch.
#ifndef FSDF_SCREEN32
#define FSDF_SCREEN32 1
#endif
// f64 contexts stage the fp64 planes too (fix-up, max face, certificates read
// LDS instead of L1/L2); sizes the stage in fsdf_set_surfaces
// Wrench rows in the wave's stage for one-chunk-per-wave passes (pass_kernel
// ALIAS); the stage is then at least the rows + the gradient transpose.
#ifndef FSDF_RED_IN_STAGE
#define FSDF_RED_IN_STAGE 1
#endif
constexpr int kRedInStageMinBytes = (64 * 6 + 2) * 8 + 64 * 3 * 8;
#ifndef FSDF_STAGE_PLANES64
#define FSDF_STAGE_PLANES64 1
#endif

constexpr int kBlock = 256;
#ifndef FSDF_PASS_BLOCK
#define FSDF_PASS_BLOCK 256
#endif
constexpr int kPassBlock = FSDF_PASS_BLOCK;  // pass-kernel workgroup (64 or a multiple)
constexpr int kBoundFloats = 20;   // spheres_w row (sphere + oriented box)        // 4 waves of 64
constexpr int kLdsPerCu = 163840;  // gfx950 LDS per CU
constexpr int kMaxLds = 163840;    // LDS a workgroup may declare (gfx950)
constexpr int kMaxHulls = 256;     // 4 accumulator slots per lane
#ifndef FSDF_MAX_BLOCKS
#define FSDF_MAX_BLOCKS 16384
#endif
constexpr int kMaxBlocks = FSDF_MAX_BLOCKS;  // pass grid cap (grid-stride beyond)
constexpr int kMaxRbfAccum = 512;  // Σ (4n+4) over RBF skins (= kMaxRbfAcc in the kernel)

struct LocalModel {
  int K = 0, F = 0, V = 0;   // K = convex hulls
  int S = 0, R = 0;          // surfaces (k* index space), RBF skins
  int rbf_rows = 0;          // Σ (n_centres + 1)
  int rbf_acc = 0;           // Σ (4 n_centres + 4)
  const int32_t* hull_surface = nullptr;  // [K]
  const int32_t* surface_kind = nullptr;  // [S]
  const int32_t* rbf_surface = nullptr;   // [R]
  const int32_t* rbf_row_off = nullptr;   // [R+1]
  const int32_t* rbf_acc_off = nullptr;   // [R+1]
  const double* verts_l = nullptr;
  const int32_t* faces = nullptr;
  const double* planes_l = nullptr;
  const int32_t* face_hull = nullptr;
  const double* sphere_l = nullptr;
  const double* box_l = nullptr;       // [K][8]
  const int32_t* face_off = nullptr;
  const int32_t* vert_hull = nullptr;
  const int32_t* vert_off = nullptr;
  const int32_t* face_rows = nullptr;  // [F][4]
  // per pose item (faces, then vertices) [F+V][4]: surface | nf << 16, hull,
  // face_off[hull], vert_off[hull] — one 16-B load instead of a chain of them
  const int32_t* item_meta = nullptr;
  int stage_bytes = 0;                 // per-wave LDS stage, context precision (multiple of 16)
  int planes64 = 0;                    // f64: stage the fp64 planes too (FSDF_STAGE_PLANES64, if they fit)
  // hull-partitioned pass tiers (pass_kernel HPART, hpart_parts): clouds of
  // up to hpart4_points run 4 waves per chunk, up to hpart2_points 2; -1 =
  // the model's default (hpart_default_limits), 0 = tier off (fsdf_set_partition)
  int64_t hpart4_points = -1, hpart2_points = -1;
};

// the model-dependent defaults of the two tiers (sdf_kernels.hip)
void hpart_default_limits(const LocalModel& lm, int64_t* four, int64_t* two);
// waves per chunk a pass over n points runs (4, 2; 0 = one wave per chunk)
int hpart_parts(const LocalModel& lm, int64_t n);
// the pass-kernel variant the last launch_pass on this thread dispatched
// ("pass_kernel<T, SLOTS, CULL, RBF, ALIAS, HPART, NB, NPART>", as rocprofv3
// prints it without the namespace); "" before any
const char* last_pass_kernel();

struct PosedModel {
  void* planes_w = nullptr;   // T
  float* spheres_w = nullptr;
  void* verts_w = nullptr;    // T
  void* hscale_w = nullptr;   // T
  float* screen_w = nullptr;  // [F+K][4] (f64 contexts; see the layout above)
  // f64 planes64 contexts: every hull's LDS stage image, [4F + K + 2V] 16-B
  // chunks; hull k at chunk 4·face_off[k] + k + 2·vert_off[k]: its screening
  // pairs (nf + 1 chunks, as in screen_w), fp64 planes (2 per face), fp64
  // vertex rows (2 per vertex), face rows (1 per face; static, written at
  // set_model). One contiguous copy stages a hull.
  void* image_w = nullptr;
  void* rbf_rows = nullptr;   // T [rbf_rows][4], per pass (fsdf_set_rbf_params)
};

struct PassOutputs {
  double* partials = nullptr;  // line tiles (sdf_kernels.hip pidx)
  int32_t* kstar = nullptr;    // optional, caller order
  double* d = nullptr;         // optional
  double* grad = nullptr;      // optional [n][3]
  const int32_t* perm = nullptr;  // optional: resident index -> caller index
  unsigned long long* stats = nullptr;  // optional kernel counters (fsdf_debug_stats)
  // optional cost-ordered schedule (resident-cloud passes): launch slot b runs
  // logical block order[b] (a permutation of [0, nblocks)); every logical block
  // writes its duration (100 MHz ticks) to cost[block]. Partial sums stay in
  // logical-block columns, so results do not depend on the order.
  const int32_t* order = nullptr;
  uint32_t* cost = nullptr;
  // optional [n64/64][4] f32 bounding sphere of each 64-point chunk of the
  // resident cloud (launch_chunk_spheres at set_points; pose-independent)
  const float* chunk_ws = nullptr;
  // optional [n] nearest surface of each resident point in the previous pass
  // over this cloud (hull-only scenes of <= 64 surfaces): read as the point's
  // best-first seed (a heuristic — any seed gives the same bits), rewritten by
  // this pass. prior_in is null on a cloud's first pass.
  const uint8_t* prior_in = nullptr;
  uint8_t* prior_out = nullptr;
  // optional device flag: set, the launch returns at once (the passes a
  // converged device solver loop still has queued, solver.hip)
  const int* skip = nullptr;
};

// Planned pass (sdf_kernels.hip planned_pass_kernel): per-chunk partial rows
// of a resident cloud (nc = ceil(n/64) chunks) and the workgroup plan.
struct ChunkOutputs {
  int32_t* hdr = nullptr;      // [nc][4] surfaces of entries 0..3 (-1: none); [c][0] == -2: dense row
  double* ent = nullptr;       // [nc][4][6] (F, M) of each entry
  double* csum = nullptr;      // [nc] Σ d² over the chunk's points
  double* dense = nullptr;     // [nc][S][6] (F, M) per surface (chunks with > 4 surfaces)
  uint32_t* dur = nullptr;     // [nc] serial-equivalent chunk durations (100 MHz ticks)
  const int32_t* plan = nullptr;  // [grid][4] workgroup plan (chunk | parts << 24, chunk, chunk, chunk), or null
  int dparts = 1;              // waves per chunk without a plan (4, 2 or 1)
  // a split chunk's wall time x (num / den) is its serial-equivalent duration
  // (the speed-up of the 4- / 2-wave split; set per model by the context:
  // capi.hip run_planned, tools/split_speedup.py)
  int r4n = 5, r4d = 2, r2n = 8, r2d = 5;
  int64_t cap = 0;             // chunks allocated: csum = ent + 24 cap, dense = ent + 25 cap (one allocation
                               // of (25 + 6 S) doubles per chunk: 1.6 KB per chunk at S = 64, i.e. 13 MB at
                               // the default 524,288-point planned window, 105 MB at kMaxPlanChunks)
};
constexpr int kPlanPartsShift = 24;
constexpr int64_t kMaxPlanChunks = 1 << 16;  // planned passes: clouds of <= 4,194,304 points per device

// a resident pass over n points of this model can run planned
bool planned_pass(const LocalModel& lm, int64_t n);
// the cloud sizes the planned pass runs by default (fsdf_set_plan max_points
// -1): min < n <= max
int64_t planned_default_max_points(const LocalModel& lm);
int64_t planned_default_min_points();
hipError_t launch_planned_pass(int precision, bool cull, const LocalModel& lm, const PosedModel& pm, const void* d_pts,
                               int64_t n, int grid, const PassOutputs& out, const ChunkOutputs& co, hipStream_t s,
                               hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);
// the accumulator d_accum [1 + 6S] from the chunk rows, in chunk order: 16-chunk
// group rows into `partials` (reduce_chunk_groups(nc) rows, line-tiled), then
// the unplanned pass's tile reduce over them
int64_t reduce_chunk_groups(int64_t nc);
hipError_t launch_reduce_chunks(const ChunkOutputs& co, int64_t nc, int S, double* partials, double* d_accum,
                                hipStream_t s, hipEvent_t ev_stop = nullptr, const int* skip = nullptr);
// the plan of the next passes from the chunk durations of this one
hipError_t launch_plan(const uint32_t* dur, int64_t nc, int n4, int n2, int32_t* order, int32_t* plan, hipStream_t s);

// Surfaces whose poses ride in the pose kernel's arguments (12·64 doubles =
// 6 KiB of kernarg; larger scenes upload them with a copy).
constexpr int kPoseArgMax = 64;
struct PoseArgs {
  double v[12 * kPoseArgMax];
};

// precision: 64 or 32. Points are AoS of the matching precision. h_poses (host,
// S <= kPoseArgMax) are passed by value in the launch; otherwise d_poses is read.
hipError_t launch_pose(int precision, const LocalModel& lm, const double* d_poses,
                       const PosedModel& pm, hipStream_t s, const double* h_poses = nullptr,
                       const int* skip = nullptr);

// ev_start / ev_stop (optional): timing events stamped by the pass kernel's
// dispatch itself (hipExtLaunchKernel), not by packets of their own
hipError_t launch_pass(int precision, bool cull, const LocalModel& lm, const PosedModel& pm,
                       const void* d_pts, int64_t n, int nblocks, const PassOutputs& out,
                       hipStream_t s, hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);

// origin: 3 host doubles (passed by value); d_rays [n][3] f64 unit directions.
hipError_t launch_raycast(int precision, bool cull, const LocalModel& lm, const PosedModel& pm, const double* origin,
                          const double* d_rays, int64_t n, double* d_depth, hipStream_t s);

// With cost/order: one extra workgroup also rebuilds order[] (heaviest logical
// blocks first) from this pass's costs, for the next pass of the same grid.
hipError_t launch_reduce(const double* partials, int nblocks, int len, double* d_accum,
                         hipStream_t s, const uint32_t* cost = nullptr, int32_t* order = nullptr,
                         hipEvent_t ev_stop = nullptr, const int* skip = nullptr);

hipError_t launch_to_f32(const double* src, float* dst, int64_t count, hipStream_t s);

// per-chunk (64 points) bounding spheres of a resident cloud of the context
// precision -> d_out [ceil(n/64)][4] f32 (the pass kernel's wave culling input)
hipError_t launch_chunk_spheres(int precision, const void* d_pts, int64_t n, int64_t nchunks, float* d_out,
                                hipStream_t s);

int pass_blocks(int64_t n, const LocalModel& lm);
bool hpart_pass(const LocalModel& lm, int64_t n);

// dynamic LDS of one pass (raycast=false) / raycast workgroup for this model
size_t pass_lds_bytes(const LocalModel& lm, bool raycast, bool alias = false);

// Scratch of the per-frame spatial sort, owned by the context and grown only
// (a frame makes no allocation).
struct SortScratch {
  double* part = nullptr;  // bbox partials [256][6] + the final box [6]
  uint32_t* k0 = nullptr;  // keys, double-buffered
  uint32_t* k1 = nullptr;
  int32_t* i1 = nullptr;   // alternate index buffer
  void* tmp = nullptr;     // rocPRIM temporary storage
  void* pts = nullptr;     // (regroup_points) the cloud buffer the regrouped points go to
  uint64_t* q0 = nullptr;  // (sort_points_keyed) composite keys, double-buffered
  uint64_t* q1 = nullptr;
  size_t part_cap = 0, k_cap0 = 0, k_cap1 = 0, i_cap1 = 0, tmp_cap = 0, pts_cap = 0, q_cap0 = 0, q_cap1 = 0;
};
void free_sort_scratch(SortScratch& s);

// Hilbert-order (sort.hip) the f64 AoS cloud d_src into d_dst (context
// precision) and write the permutation d_perm[resident i] = caller index
// (n < 2^31). Asynchronous on `st`.
hipError_t sort_points_spatial(const double* d_src, int64_t n, int precision, void* d_dst, int32_t* d_perm,
                              SortScratch& s, hipStream_t st);
// Regroup a resident cloud by each point's nearest surface in the last pass
// (prior[i] < 64), keeping the current (Hilbert) order within each group: a
// stable counting sort (sort.hip regroup_*_kernel, three launches). The
// regrouped points replace *d_pts (the old buffer becomes the scratch's:
// *d_pts / *pts_cap are updated); d_perm and prior are permuted in place.
// Asynchronous on `st`.
hipError_t regroup_points(void** d_pts, int64_t* pts_cap, int64_t n, int precision, int32_t* d_perm, uint8_t* prior,
                          SortScratch& s, hipStream_t st);
// ---- device solver iteration (solver.hip) ------------------------------------
// The mechanism of a rigid scene as two device buffers built by the context
// from fsdf_set_mechanism (capi.hip build_solver_tree) — integers and doubles,
// each array at an offset — with the level schedules of the parallel FK and
// chain rule. The solver kernels copy both buffers into LDS first, so every
// later access in their level loops is an LDS access.
struct SolverTree {
  int nb = 0, nx = 0, S = 0;
  int D = 0;  // depth of the deepest body
  int H = 0;  // height levels of bodies with children: height_order[height_off[h] .. ) at height h+1
  int narrow = 0;  // every height level has <= 10 parents: the subtree sums run in one wave
  int chains = 0;  // every non-root body has <= 1 child: subtree sums along chain lists, no levels
  // one blob: the doubles [nd], then the ints [ni], padded to 16 B — copied into
  // LDS with one batch of 16-B loads per thread (one memory latency)
  const void* blob = nullptr;
  int ni = 0, nd = 0, chunks16 = 0;
  // offsets into the ints
  // path_list[path_off[b] .. path_off[b+1]): body b's ancestors from depth 1 down to b
  int parent = 0, kind = 0, qoff = 0, path_list = 0, path_off = 0, height_order = 0, height_off = 0;
  int child_off = 0, child_list = 0;  // [nb+1], children in descending index
  int surf_off = 0, surf_list = 0;    // [nb+1], surfaces in ascending index
  int surface_body = 0;               // [S]
  int chain_list = 0, chain_off = 0;  // (chains) [nb+1]: body b, its child, grandchild, ...
  // offsets into the doubles
  int axis = 0, AR = 0, At = 0, BR = 0, Bt = 0, frame_R = 0, frame_t = 0;  // frames: [S][9], [S][3]
};
// One frame's solver state (device), two slots by iteration parity (a step
// launch's workgroups read slot (k & 1) while its workgroup 0 writes slot
// (k+1 & 1)): x [2][nx], the joint frames of the last FK Rb|tb [2][12 nb]
// (Rb [nb][9] then tb [nb][3] per slot); optional divisors [nx]; f = the last
// evaluation's cost / n_points; flags [3] = (done — the skip flag of the
// frame's launches —, iterations (x of the last one in slot iterations & 1),
// error: 1 FK / chain rule, 2 a non-finite pose). (The next pass's posed
// model is written by the step itself: pose_impl.h.)
struct SolverState {
  double* x = nullptr;
  const double* div = nullptr;
  double *Rb = nullptr, *f = nullptr;
  int* flags = nullptr;
  double rate = 0.0, max_step = 0.0, tol = 0.0, n_points = 1.0, weight = 0.0;
  int limit = 0;
};
// the step's LDS (the tree, the accumulator and the work arrays) fits one workgroup
bool solver_fits(int nb, int nx, int S, int ni);
// diagnostic builds (-DFSDF_SOLVER_TIMES=1): the last step's phase clocks (16, 100 MHz)
void solver_times(unsigned long long* out);
// FK of st.x -> Rb, tb and the first pass's posed model pm (flags zeroed by the
// caller; set on an error)
hipError_t launch_solver_init(const SolverTree& T, const SolverState& st, const LocalModel& lm,
                              const PosedModel& pm, int precision, hipStream_t s);
// one NaiveSolver iteration from the pass's accumulator, ending with the next
// pass's posed model pm (skips once flags[0] is set)
hipError_t launch_solver_step(const SolverTree& T, const SolverState& st, const double* d_accum,
                              const LocalModel& lm, const PosedModel& pm, int precision, int it_before,
                              hipStream_t s);

// Exchanged spatial shards (fsdf_set_points_keyed_device): the bounding box
// (lo xyz, hi xyz; a device pointer into the scratch) of a device f64 cloud,
// the 30-bit curve keys of a cloud in a given device box (the keys
// sort_points_spatial orders by), and a resident cloud ordered by (key,
// whole-cloud index) with perm = those indices (< 2^31) — the order a shard of
// the whole cloud's sort_points_spatial order has. Asynchronous on `st`.
hipError_t cloud_box(const double* d_src, int64_t n, SortScratch& s, hipStream_t st, double** d_box);
// Seeds carried from one cloud to the next (sort.hip): a kVoxDim^3 grid of
// uint8 k* over a box fixed per context (lo, cells per unit length inv)
constexpr int kVoxDim = 64;
struct VoxBox {
  double lo[3] = {0, 0, 0}, inv[3] = {0, 0, 0};
};
// every point of a resident cloud (context precision) writes its prior k* (< 64) into its voxel
hipError_t vox_scatter(int precision, const void* d_pts, int64_t n, const uint8_t* d_prior, const VoxBox& b,
                       uint8_t* d_grid, hipStream_t st);
// every point's prior from its voxel (0xFF outside the box or in an empty voxel)
hipError_t vox_gather(int precision, const void* d_pts, int64_t n, const VoxBox& b, const uint8_t* d_grid,
                      uint8_t* d_prior, hipStream_t st);
hipError_t curve_keys(const double* d_src, int64_t n, const double* d_box, uint32_t* d_keys, hipStream_t st);
hipError_t sort_points_keyed(const double* d_src, const uint32_t* d_keys, const int64_t* d_index, int64_t n,
                             int precision, void* d_dst, int32_t* d_perm, SortScratch& s, hipStream_t st);

// d_out[i] = d_perm[i] as int64 (fsdf_get_permutation's layout)
hipError_t widen_permutation(const int32_t* d_perm, int64_t n, int64_t* d_out, hipStream_t st);

}  // namespace fsdf
