/*
 * flashsdf.h — C-ABI of the MI355X-native signed-distance residual pass.
 *
 * This is the drop-in boundary for the hot path of Flash.jl
 * (JuliaTagBot/point-cloud-signed-distance). In the reference the path is pure
 * Julia; no FFI exists. The entry points below are exactly what a Julia
 * `ccall` shim under src/tracking.jl would bind:
 *
 *   reference                                     replaced by
 *   ---------------------------------------------------------------------------
 *   Flash.skin(state)          src/Flash.jl:265-268   fsdf_eval / fsdf_skin
 *     (min over surfaces, one closure per point)      (all points in one launch)
 *   skin(state, ::ConvexGeometry) src/Flash.jl:245-250 fsdf_set_model + poses
 *     + ConvexSurface functor  src/Flash.jl:233-243    (exact polytope SDF)
 *   GradientDescent.cost       src/gradientdescent.jl:28-39
 *     c = Σ_p skin(p)^2                               accum[0]
 *     ∂c/∂x via ForwardDiff (Dual{9} chunk passes)    accum[1..6K] wrenches,
 *                                                     chained to ∂c/∂q on host
 *   CostFunctor(manip, pts)    src/gradientdescent.jl:41-57
 *     sensed_points held by reference             fsdf_set_points (once/frame)
 *   EnhancedGJK.NeighborMesh / conv(vertices)   src/models.jl:152
 *                                                     fsdf_convex_hull
 *   transform_to_root(state, frame) src/Flash.jl:248  fsdf_tree_transforms
 *     (RigidBodyDynamics forward kinematics)          (host, per pass; on the
 *                                                     device inside fsdf_descend)
 *
 * Conventions
 *   - All host buffers are caller-owned. Nothing is retained past a call
 *     except what set_model / set_points copy to the device.
 *   - Points are AoS xyz float64, exactly Julia's Vector{SVector{3,Float64}}.
 *   - A pose is 12 float64: R (3x3, row-major) then t (3); x_world = R x_local + t.
 *   - Every function returns 0 (FSDF_OK) or a nonzero status; the message of the
 *     last failure on a context is fsdf_last_error(ctx).
 *   - Accumulator layout (length 1 + 6K + Σ_rbf (4 n_r + 4), K = surfaces):
 *       accum[0]            = Σ_p d*(p)^2                     (cost, no regularizer)
 *       accum[1+6k+0..2]    = Σ_{p: k*(p)=k} 2 d*(p) ∇d*(p)   (force-like, world)
 *       accum[1+6k+3..5]    = Σ_{p: k*(p)=k} 2 d*(p) p × ∇d*(p) (moment about origin)
 *     so that for a world twist (ω, v) of hull k:  δc = -(ω·M_k + v·F_k)
 *     (zero for RBF surfaces); then per RBF surface r with n_r centres, over
 *     the points with k* = r:
 *       λ_w[n_r], λ_a, λ_b[3]  = Σ 2 s ∂s/∂(w, a, b)
 *       E[n_r][3]              = Σ 2 s ∂s/∂c_i (coefficients held fixed)
 *     from which the host forms dc/dc_i = E_i − μᵀ(∂M/∂c_i)u, μ = M⁻ᵀλ.
 *   - Nearest-primitive index k*(p) is the FIRST k attaining the minimum,
 *     matching Julia's left-fold `minimum` (src/Flash.jl:267).
 *   - The library never falls back to a CPU path: without a usable gfx950
 *     device every compute call fails with FSDF_ERR_HIP.
 */
#ifndef FLASHSDF_H
#define FLASHSDF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FSDF_OK 0
#define FSDF_ERR_ARG 1        /* bad argument (null pointer, size, index)      */
#define FSDF_ERR_HIP 2        /* HIP runtime failure / no device                */
#define FSDF_ERR_STATE 3      /* call order violated (no model / no points)     */
#define FSDF_ERR_NOMEM 4      /* allocation failure                             */
#define FSDF_ERR_DEGENERATE 5 /* geometry degenerate (coplanar hull input, ...) */

#define FSDF_PRECISION_F64 64
#define FSDF_PRECISION_F32 32

typedef struct fsdf_ctx fsdf_ctx;

typedef struct fsdf_opts {
  int32_t device;      /* HIP device ordinal (process-local)                      */
  int32_t precision;   /* FSDF_PRECISION_F64 (default) or FSDF_PRECISION_F32       */
  int32_t sort_points; /* 1: reorder the resident cloud spatially at set_points
                          (outputs are still returned in caller order)            */
  int32_t cull;        /* 1 (default): exact-safe bounding-sphere culling;
                          0: brute force over every hull (reference loop order)    */
} fsdf_opts;

/* One convex primitive in its body (local) frame.
 * Replaces ConvexGeometry(NeighborMesh(mesh), frame) (src/models.jl:152,159). */
typedef struct fsdf_hull {
  int32_t n_vertices;
  int32_t n_faces;
  const double* vertices; /* [n_vertices][3]                                     */
  const int32_t* faces;   /* [n_faces][3], counter-clockwise seen from outside    */
  const double* planes;   /* [n_faces][4] = (n, d), |n| = 1, n·x <= d inside      */
} fsdf_hull;

/* A scene surface, in the reference's surface order (Manipulator.surfaces,
 * src/Flash.jl:62-65): k* indexes this list.
 *   FSDF_SURFACE_HULL: a convex primitive (`hull`), posed by poses[k].
 *   FSDF_SURFACE_RBF:  an interpolating skin (src/Flash.jl:207-213) over
 *                      `n_centers` centres; its world centres and RBF
 *                      coefficients are supplied per pass (fsdf_set_rbf_params),
 *                      its pose is ignored. Value: s = f/|∇f| with
 *                      f(x) = Σ w_i |x-c_i|^3 + a + b·x (XCubed + affine).
 *                      Matches the reference KAT (test/runtests.jl:17) but NOT
 *                      the costs printed by examples/manipulator.ipynb:5512,
 *                      :14179 (ours 4.44x / 2.0x; no candidate formulation fits
 *                      all three): a documented divergence, DESIGN.md §2. */
#define FSDF_SURFACE_HULL 0
#define FSDF_SURFACE_RBF 1
typedef struct fsdf_surface {
  int32_t kind;      /* FSDF_SURFACE_HULL or FSDF_SURFACE_RBF */
  int32_t n_centers; /* RBF only */
  fsdf_hull hull;    /* HULL only */
} fsdf_surface;

/* ---- geometry ingest (host only, no device needed) --------------------------
 * Convex hull of a point set (the shape GJK's support function sees,
 * EnhancedGJK.NeighborMesh over the mesh vertices, src/models.jl:152).
 * Capacities: vertices_out >= 3n doubles, faces_out >= 3(2n-4) ints,
 * planes_out >= 4(2n-4) doubles. Output faces are triangles, outward, CCW. */
int fsdf_convex_hull(const double* points, int32_t n, int32_t* n_vertices_out,
                     double* vertices_out, int32_t* n_faces_out, int32_t* faces_out,
                     double* planes_out);

/* Forward kinematics of a mechanism tree (host only, no device): the body
 * poses transform_to_root(state, body) that the per-pass surface poses are
 * built from (src/Flash.jl:248; RigidBodyDynamics in the reference). Bodies in
 * topological order (parent[b] < b, body 0 = root). Per body b >= 1:
 * kind 0 fixed, 1 revolute about unit axis[b] by q[qoff[b]], 2 quaternion
 * floating q[qoff[b] .. +7] = (w, x, y, z, tx, ty, tz) (normalized here);
 * joint_to_parent (AR[b] row-major 3x3, At[b]) and body_to_joint (BR[b], Bt[b]).
 * Out: R[b], t[b] = transform_to_root(body b); Rb[b], tb[b] = the parent's
 * transform composed with joint_to_parent (the joint frame before its motion,
 * where the chain rule's motion subspaces live). All arrays [nb][9] / [nb][3]. */
int fsdf_tree_transforms(int32_t nb, const int32_t* parent, const int32_t* kind, const int32_t* qoff,
                         const double* axis, const double* AR, const double* At, const double* BR,
                         const double* Bt, const double* q, double* R, double* t, double* Rb, double* tb);

/* Host chain rule (no device): ∂c/∂q of the mechanism from the accumulator's
 * per-surface wrenches (surface_wrench[k] = accum[1+6k .. 7+6k]: F, M about the
 * world origin) on surface_body[k] (-1: none), plus optional per-body wrenches
 * body_wrench [nb][6] (the RBF chain's); tree arrays as fsdf_tree_transforms,
 * Rb/tb = its joint frames before the motion; work = nb*6 doubles of scratch;
 * gq [num_positions]. Replaces ForwardDiff's ⌈n/9⌉ Dual passes through
 * RigidBodyDynamics (src/gradientdescent.jl:28-39, src/tracking.jl:16-21) for
 * fixed, revolute and quaternion-floating joints (with normalize!'s projection,
 * src/gradientdescent.jl:30); flash/mechanism.py config_gradient is the numpy
 * twin the tests compare it with. */
int fsdf_config_gradient(int32_t nb, const int32_t* parent, const int32_t* kind, const int32_t* qoff,
                         const double* axis, const double* Rb, const double* tb, const double* q, int32_t nsurf,
                         const int32_t* surface_body, const double* surface_wrench, const double* body_wrench,
                         double* work, double* gq);

/* RBF weight solve and its adjoint (host only, no device; the host side of
 * the interpolating skins, src/Flash.jl:143-213, around fsdf_set_rbf_params and
 * the pass). fsdf_rbf_solve: centres [n][3] (world), values [n] (0 surface
 * points, -1 skeleton points) -> u [n+4] = (w, a, b) of
 * [A P; Pᵀ 0] u = [v; 0], A_ij = |c_i - c_j|^3, P_i = (1, c_iᵀ); lu
 * [(n+4)^2] and piv [n+4] receive the factorization for the adjoint.
 * fsdf_rbf_adjoint: this surface's accumulator block [4n+4] (λ [n+4], then E
 * [n][3]) -> G [n][3] = ∂cost/∂c_j (world); work [n+4]. flash/rbf.py solve /
 * chain are the numpy twins. FSDF_ERR_DEGENERATE: singular system. */
int fsdf_rbf_solve(int32_t n, const double* centres, const double* values, double* u, double* lu, int32_t* piv);
int fsdf_rbf_adjoint(int32_t n, const double* centres, const double* u, const double* lu, const int32_t* piv,
                     const double* block, double* G, double* work);

/* The whole CostFunctor iteration of a rigid (hull-only) scene in one call:
 * fsdf_set_mechanism registers the mechanism tree (the arrays of
 * fsdf_tree_transforms, nq = num_positions) and, per surface of
 * fsdf_set_surfaces, its body (-1: none) and body-to-geometry frame (R
 * row-major [S][9], t [S][3]); fsdf_value_and_gradient(x) then runs host FK,
 * the surface poses, one residual pass over the resident cloud, and the chain
 * rule: cost_out = Σ_p d*(p)^2 and grad_out [nq] = ∂cost/∂x at the caller's x
 * (quaternion blocks normalized for the evaluation, the projection in the
 * gradient) — CostFunctor(x) with its ForwardDiff gradient
 * (src/gradientdescent.jl:28-57). Scenes with RBF skins also declare their
 * centres (fsdf_set_rbf_centres, below; FSDF_ERR_STATE until every RBF
 * surface has them). */
int fsdf_set_mechanism(fsdf_ctx* ctx, int32_t nb, const int32_t* parent, const int32_t* kind, const int32_t* qoff,
                       const double* axis, const double* AR, const double* At, const double* BR, const double* Bt,
                       int32_t nq, const int32_t* surface_body, const double* frame_R, const double* frame_t);
int fsdf_value_and_gradient(fsdf_ctx* ctx, const double* x, double* cost_out, double* grad_out);
/* RBF scenes in fsdf_value_and_gradient: after fsdf_set_mechanism (which
 * clears earlier declarations) every RBF surface's centres are declared once —
 * n_sp surface points (body, body-frame xyz, deformation row or -1; value 0)
 * then n_sk skeleton points (value -1), n_sp + n_sk = its n_centers
 * (src/Flash.jl:143-213) — and fsdf_set_deformations gives the deformation
 * count (x = [q; δ], 3 per deformable point, src/gradientdescent.jl:9-17) and
 * the regularizer weight (default_deformation_cost_weight = 10, :7). value_and_gradient then also
 * places the centres (c = R_b (p + δ) + t_b), solves the weights, uploads the
 * rows, and chains the pass's RBF block through the solve: cost_out = Σ d*^2 +
 * weight Σ|δ|^2, grad_out [nq + 3 n_deform] (CostFunctor(x) with its gradient,
 * src/gradientdescent.jl:28-57). */
int fsdf_set_rbf_centres(fsdf_ctx* ctx, int32_t surface, int32_t n_sp, const int32_t* body_sp,
                         const double* local_sp, const int32_t* deform_row_sp, int32_t n_sk, const int32_t* body_sk,
                         const double* local_sk);
int fsdf_set_deformations(fsdf_ctx* ctx, int32_t n_deform, double weight);
/* The same iteration split around a multi-GPU all-reduce (one context per
 * rank, each over its shard): fsdf_eval_state_device(x) runs FK, the RBF solve,
 * the poses and the pass into the DEVICE accumulator d_accum (asynchronous on
 * the context's stream); after the caller's all-reduce (RCCL) and read-back,
 * fsdf_state_gradient(x, accum) returns cost and gradient as
 * fsdf_value_and_gradient does, on the FK / weight solve of that pass. x may
 * be the x of either of this context's last two fsdf_eval_state_device passes
 * (pipelined passes: the next pass is enqueued before the previous all-reduce
 * completes): the host FK and weight solve are then redone for x — the same
 * arithmetic, the same bits. Any other x (not the configuration of an
 * accumulator this context produced) is refused with FSDF_ERR_STATE. */
int fsdf_eval_state_device(fsdf_ctx* ctx, const double* x, double* d_accum);
int fsdf_state_gradient(fsdf_ctx* ctx, const double* x, const double* accum, double* cost_out, double* grad_out);

/* estimate_state's solver loop (src/tracking.jl:16-26: wrapped_cost c/N, warm
 * start x) around fsdf_value_and_gradient, with no host-language round trip per
 * iteration. Up to iteration_limit times: f = cost/n_points, g = (grad/n_points)
 * ./ divisors (NULL = ones); stop when |g|_2 < tolerance; else x += clamp(-rate g,
 * ±max_step) component-wise (NaiveSolver's rule as restated in
 * flash/tracking.py — the solver itself is the un-vendored
 * SimpleGradientDescent.jl; the rule is pinned by examples/manipulator.ipynb's
 * own per-trial traces, tests/test_manipulator_traces.py). n_points = 1
 * reproduces the notebook's session, whose objective was the undivided c.
 * x [nq + 3 n_deform] is updated in place;
 * value_out = f of the last evaluation, iterations_out = evaluations made. */
int fsdf_descend(fsdf_ctx* ctx, double* x, int32_t iteration_limit, double rate, double max_step, double tolerance,
                 const double* divisors, double n_points, double* value_out, int32_t* iterations_out);
/* Where fsdf_descend iterates. device_loop = 1 (default): rigid scenes (no RBF
 * skin, no deformation) iterate on the device where the mechanism fits the
 * solver step's 64 KB of LDS, others on the host; 0: always the host loop
 * around fsdf_value_and_gradient, one synchronization per iteration; 2: the
 * device loop is required (FSDF_ERR_STATE otherwise). The device loop enqueues
 * the frame's passes and solver steps up front and reads x, value and count
 * back once (csrc/solver.hip: FK, chain rule, the clipped NaiveSolver step and
 * the next pass's pose after each pass, the host loop's arithmetic in the same
 * order — x, value and iterations bit-identical to it; after convergence the
 * remaining launches return at once). Measured: on
 * resident clouds 7-8 % faster per iteration than the host loop (C2, C4, M64),
 * per fresh 2^20 frame 1.5 % (M64) or level (IRB140). */
int fsdf_set_solver(fsdf_ctx* ctx, int32_t device_loop);

/* ---- context ---------------------------------------------------------------- */
int fsdf_create(fsdf_ctx** out, const fsdf_opts* opts);
int fsdf_destroy(fsdf_ctx* ctx);
const char* fsdf_last_error(const fsdf_ctx* ctx);
/* Launch on a caller-owned hipStream_t (NULL = the context's own stream;
 * FSDF_HIP_NULL_STREAM = HIP's null/default stream, the handle 0 that e.g.
 * torch's default stream reports). */
#define FSDF_HIP_NULL_STREAM ((void*)(intptr_t)-1)
int fsdf_set_stream(fsdf_ctx* ctx, void* hip_stream);
int fsdf_num_hulls(const fsdf_ctx* ctx, int32_t* k_out);
int fsdf_accum_len(const fsdf_ctx* ctx, int32_t* len_out); /* 1 + 6K + Σ(4n+4) */

/* Upload the model once (per model). Replaces the per-evaluation
 * CollisionCache construction of src/Flash.jl:246. fsdf_set_model is the
 * hull-only form of fsdf_set_surfaces. */
int fsdf_set_model(fsdf_ctx* ctx, const fsdf_hull* hulls, int32_t n_hulls);
int fsdf_set_surfaces(fsdf_ctx* ctx, const fsdf_surface* surfaces, int32_t n_surfaces);

/* Per-pass RBF parameters (before fsdf_eval / fsdf_skin when the scene has RBF
 * surfaces): for every RBF surface in surface order, n_centers rows
 * (c_x, c_y, c_z, w) in the world frame, then one row (a, b_x, b_y, b_z).
 * n_doubles must equal 4·Σ(n_centers + 1). The host solves the (n+4)² system
 * [A P; Pᵀ 0][w; a; b] = [v; 0] (surface points v = 0, skeleton v = -1). */
int fsdf_set_rbf_params(fsdf_ctx* ctx, const double* params, int64_t n_doubles);

/* Upload the sensed cloud once per frame (src/gradientdescent.jl:43 holds it
 * by reference across every cost evaluation). A sorting hull-only context
 * seeds the new cloud's first pass from the previous cloud's last nearest
 * surfaces (a voxel grid over the first cloud's box, grown by half its extent;
 * seeds order the search only — results do not depend on them). */
int fsdf_set_points(fsdf_ctx* ctx, const double* xyz, int64_t n);
/* Same, from a device-resident AoS buffer (copied device-to-device). */
int fsdf_set_points_device(fsdf_ctx* ctx, const double* d_xyz, int64_t n);
/* The next frame's cloud ahead of time (a frame loop over recorded or queued
 * clouds, src/gradientdescent.jl:43 once per frame): fsdf_prefetch_points
 * queues its host-to-device copy on a stream of the context's own and returns
 * at once; the copy is issued right after the context's next pass is launched
 * (or by fsdf_set_points_prefetched when no pass comes between), so it runs
 * during the current frame's passes (overlapped from page-locked memory; the
 * caller keeps xyz unchanged until the next call below returns; a second
 * prefetch replaces a pending one);
 * fsdf_set_points_prefetched then makes it resident as fsdf_set_points would
 * (FSDF_ERR_STATE when nothing is pending). A sorting context also Hilbert-
 * sorts the prefetched cloud on that stream, into a second resident buffer set,
 * so fsdf_set_points_prefetched only swaps buffers. fsdf_set_points meanwhile
 * leaves a pending prefetch pending. */
int fsdf_prefetch_points(fsdf_ctx* ctx, const double* xyz, int64_t n);
int fsdf_set_points_prefetched(fsdf_ctx* ctx);
/* One rank's shard of a cloud split over several devices (the
 * cost is a plain sum over points, src/gradientdescent.jl:32): the whole
 * n-point cloud is uploaded and ordered (the Hilbert order with sort_points,
 * else the caller's), and positions [begin, end) of that order stay resident —
 * a contiguous region of space, so the shard keeps the whole cloud's point
 * density per 64-point chunk (a slice of an arbitrary order would scatter each
 * rank's points over the whole scene). Every rank of a job passes the same
 * cloud and its own range; the ranges partition [0, n). Per-point outputs of a
 * ranged cloud are always in its resident order, and fsdf_get_permutation names
 * each resident point's index in the whole cloud. fsdf_chunk_costs then reports
 * the range's chunks — the chunks of the whole cloud's order when begin is a
 * multiple of 64 — which is what flash.distributed balances the ranges by; once
 * the range has been regrouped (fsdf_regroup_points) its chunks are no longer
 * the whole cloud's and fsdf_chunk_costs refuses (FSDF_ERR_STATE) until the
 * next set_points. */
int fsdf_set_points_range(fsdf_ctx* ctx, const double* xyz, int64_t n, int64_t begin, int64_t end);
int fsdf_set_points_range_device(fsdf_ctx* ctx, const double* d_xyz, int64_t n, int64_t begin, int64_t end);
int fsdf_num_points(const fsdf_ctx* ctx, int64_t* n_out);
/* Spatial shards with O(N/W) ingest per rank (flash.distributed.exchange_points):
 * each rank uploads only its 1/W slice of the sensed cloud; the ranks agree on
 * the whole cloud's bounding box (fsdf_cloud_box_device of each slice, then a
 * 6-double all-reduce), compute each point's 30-bit Hilbert key in it
 * (fsdf_curve_keys_device: the keys fsdf_set_points orders by), split the key
 * range into W contiguous ranges from an all-reduced key histogram, move every
 * point to the rank owning its key over one all-to-all, and each rank makes its
 * received points resident (fsdf_set_points_keyed_device): ordered by (key,
 * whole-cloud index) — exactly the whole cloud's sorted order restricted to its
 * key range — with the whole-cloud indices as the permutation (FSDF_ORDER_RESIDENT
 * outputs, like fsdf_set_points_range; indices < 2^31). Per-point results are
 * those of a single context over the whole cloud, bit for bit. box: host
 * [6] = (lo xyz, hi xyz); all calls synchronous. */
int fsdf_cloud_box_device(fsdf_ctx* ctx, const double* d_xyz, int64_t n, double* box_out);
int fsdf_curve_keys_device(fsdf_ctx* ctx, const double* d_xyz, int64_t n, const double* box, uint32_t* d_keys);
int fsdf_set_points_keyed_device(fsdf_ctx* ctx, const double* d_xyz, const uint32_t* d_keys, const int64_t* d_index,
                                 int64_t n);
/* Regroup the resident cloud by each point's nearest surface in the last pass
 * over it, keeping the current (Hilbert) order within each surface's group: a
 * stable device sort, once per frame after its first pass. The reference has no
 * counterpart — its track! loop (src/tracking.jl:8-27) evaluates the cost of
 * one frame's cloud over and over (src/gradientdescent.jl:43), which is what
 * this exploits: the passes seed each point from its last nearest surface, and
 * a 64-point chunk whose points share one evaluates fewer hulls. Per-point
 * results are unchanged; the cost and wrench sums change in rounding only (the
 * chunks group other points). It pays where the pass is bound by its summed
 * work — the one-wave grid of clouds above the planned window — and costs where
 * the planned pass is bound by its heaviest chunk, which grouping makes heavier
 * (DESIGN.md §7 round 5). The resident order changes: re-read
 * fsdf_get_permutation for FSDF_ORDER_RESIDENT outputs. Requires a sorted
 * (sort_points) or ranged cloud and a pass over it (hull-only scenes of <= 64
 * surfaces); asynchronous on the context stream. */
int fsdf_regroup_points(fsdf_ctx* ctx);
/* The regroup where it pays, decided by the library: only after a pass that
 * ran one wave per chunk (the grid above the planned window, bound by its
 * summed work), on a sorted or ranged cloud not yet regrouped since its
 * set_points. *applied_out = 1 when it regrouped (NULL allowed).
 * fsdf_set_regroup: FSDF_REGROUP_AUTO (default) — the iteration entry points
 * that return no per-point outputs (fsdf_value_and_gradient,
 * fsdf_eval_state_device, fsdf_descend) apply this rule after a new cloud's
 * first pass, so track! frames regroup by themselves; FSDF_REGROUP_OFF — only
 * explicit calls regroup. fsdf_eval / fsdf_eval_device never regroup on their
 * own (their resident-order outputs index the permutation of the pass). */
#define FSDF_REGROUP_OFF 0
#define FSDF_REGROUP_AUTO 1
int fsdf_regroup_auto(fsdf_ctx* ctx, int32_t* applied_out);
int fsdf_set_regroup(fsdf_ctx* ctx, int32_t mode);

/* One residual pass over the resident cloud (synchronous, host buffers).
 * poses: [K][12] host. Outputs may be NULL when not wanted:
 *   cost_out   1 double         accum_out  1+6K doubles
 *   kstar_out  n int32          d_out      n doubles      grad_out [n][3] doubles */
int fsdf_eval(fsdf_ctx* ctx, const double* poses, double* cost_out, double* accum_out,
              int32_t* kstar_out, double* d_out, double* grad_out);

/* Same pass, asynchronous on the context stream, outputs in DEVICE memory
 * (used by the multi-GPU path: the caller all-reduces d_accum over RCCL).
 * d_accum: 1+6K doubles (required); per-point outputs may be NULL. */
int fsdf_eval_device(fsdf_ctx* ctx, const double* poses, double* d_accum,
                     int32_t* d_kstar, double* d_d, double* d_grad);

/* Scene signed distance at arbitrary query points (the closure returned by
 * Flash.skin(state), src/Flash.jl:265-268), not touching the resident cloud.
 * xyz: [n][3] host; outputs host, any may be NULL. Synchronous. */
int fsdf_skin(fsdf_ctx* ctx, const double* poses, const double* xyz, int64_t n,
              double* d_out, int32_t* kstar_out, double* grad_out);

/* Depth-sensor raycast on the scene SDF (src/depthsensors.jl:56-97, doRaycast;
 * the field is Flash.skin(state), src/depthsensors.jl:116): per ray a secant
 * march from `origin` — step = -SDF/est_grad (est_grad starts at -1, then the
 * secant slope), |step| <= 0.4, stop at |SDF| <= 1e-5 or after 60 steps;
 * depth = NaN when the final |SDF| > 1e-2. origin: 3 doubles (world);
 * rays: [n][3] unit directions (world); depth_out: n doubles. Synchronous.
 * Uses the current RBF parameters when the scene has skins. */
int fsdf_raycast(fsdf_ctx* ctx, const double* poses, const double* origin, const double* rays, int64_t n,
                 double* depth_out);

/* Order of the per-point outputs of fsdf_eval / fsdf_eval_device:
 *   FSDF_ORDER_CALLER (default): output i belongs to input point i;
 *   FSDF_ORDER_RESIDENT: output i belongs to resident point i — the device
 *     order after fsdf_opts.sort_points (Hilbert order), written with
 *     coalesced stores instead of a scatter through the permutation. Caller
 *     point perm[i] (fsdf_get_permutation) is resident point i. Without
 *     sort_points the two orders coincide. fsdf_skin always uses caller order. */
#define FSDF_ORDER_CALLER 0
#define FSDF_ORDER_RESIDENT 1
int fsdf_set_output_order(fsdf_ctx* ctx, int32_t order);
/* perm[i] = caller index of resident point i (n = fsdf_num_points int64s;
 * identity without sort_points). Host / device destination. */
int fsdf_get_permutation(fsdf_ctx* ctx, int64_t* perm_out);
int fsdf_get_permutation_device(fsdf_ctx* ctx, int64_t* d_perm_out);

/* Block until all work queued on the context stream has finished. */
int fsdf_synchronize(fsdf_ctx* ctx);

/* ---- measurement ------------------------------------------------------------
 * With profiling enabled, every residual pass stamps HIP events at the start
 * and end of the pass kernel (the dominant launch) and at the end of the
 * reduction that follows it, through the kernel dispatches themselves
 * (hipExtLaunchKernel: no event packets between the kernels, so profiling
 * leaves the step's timing alone). fsdf_pass_times synchronizes, returns the
 * summed pass-kernel time, the summed pass + reduction time of the passes
 * recorded since the last query and their count, and resets the record;
 * fsdf_pass_time returns the pass + reduction sum only. */
int fsdf_profile_pass(fsdf_ctx* ctx, int32_t enable);
int fsdf_pass_times(fsdf_ctx* ctx, double* kernel_ms_out, double* pass_ms_out, int64_t* launches_out);
int fsdf_pass_time(fsdf_ctx* ctx, double* total_ms_out, int64_t* launches_out);

/* The pass-kernel variant the context's last residual pass dispatched, as
 * rocprofv3 names it without the namespace, e.g.
 * "pass_kernel<double, 1, true, false, true, false, 256, 4>"; "" before any
 * pass. (bench.py attaches PMC counters to its roofline only when the
 * profiled kernel is this one.) */
const char* fsdf_pass_kernel_name(const fsdf_ctx* ctx);

/* ---- hull-partitioned pass tiers ---------------------------------------------
 * Small clouds leave wave slots idle while a chunk's serial hull evaluations
 * set the pass time; up to a tier's point count the pass instead runs 4 (or
 * 2) waves per 64-point chunk, each evaluating every 4th (2nd) hull, merged by
 * the first-index (d, k) minimum — bit-identical per point. The tiers apply to
 * f64 hull-only scenes of <= 64 surfaces. Defaults depend on the model (hull
 * count); fsdf_set_partition overrides them for this context:
 * -1 = the model's default, 0 = tier off, else the largest cloud (points per
 * device) the tier runs. fsdf_get_partition reports the limits in effect and
 * the waves per chunk (4, 2, 0 = one) a pass over n points would run.
 * Replaces the reference's nothing: a scheduling knob of this build. */
int fsdf_set_partition(fsdf_ctx* ctx, int64_t four_way_max_points, int64_t two_way_max_points);
int fsdf_get_partition(fsdf_ctx* ctx, int64_t n, int64_t* four_way_max_out, int64_t* two_way_max_out,
                       int32_t* parts_out);

/* ---- planned pass --------------------------------------------------------------
 * Resident-cloud passes of f64 hull-only scenes with <= 64 surfaces (the
 * metric's M64, IRB140) run a planned grid: every 64-point chunk writes its
 * own partial row (so the accumulator sums chunks in index order, bit-identical
 * whatever the plan), records its duration, and from the cloud's first pass on
 * (rebuilt every 16 passes) the heaviest chunks — `four_way_share` of them —
 * are split over 4 waves (hull-partitioned), the next `two_way_share` over 2,
 * the rest run one wave each grouped by similar cost, heaviest workgroups
 * first. enable = 0 runs the unplanned one-block-per-4-chunks grid instead
 * (A/B). Shares < 0 select the default: the heaviest 96 chunks over 4 waves
 * and the next 192 over 2; at least as many chunks go 4 ways as the device has
 * idle wave slots for (a strong-scaling shard smaller than the machine splits
 * its heaviest third). A new cloud's first pass runs the tier shape of
 * fsdf_set_partition. max_points: the largest cloud (points per device) the
 * planned pass runs, -1 = the model's default window: more than 98,304 and
 * at most 524,288 points for models of >= 32 hulls, 393,216 for smaller ones
 * (outside it the unplanned grid measured faster); a value >= 0
 * runs it for every cloud of 1 .. max_points points. Memory: the per-chunk
 * rows take (25 + 6 S) doubles per 64-point chunk per context (1.6 KB at
 * S = 64: 13 MB for the default window's 524,288 points, 105 MB at the
 * 4,194,304-point limit); a second context in flight holds its own. */
int fsdf_set_plan(fsdf_ctx* ctx, int32_t enable, double four_way_share, double two_way_share, int64_t max_points);

/* Diagnostics: the serial-equivalent durations (100 MHz ticks) the last
 * planned pass measured per 64-point chunk of the resident cloud (resident
 * order), as the plan is built from them. *count_out = the chunk count (0
 * before a planned pass); costs_out may be NULL to query it. FSDF_ERR_STATE
 * for a ranged cloud that has been regrouped (see fsdf_set_points_range). */
int fsdf_chunk_costs(fsdf_ctx* ctx, uint32_t* costs_out, int64_t* count_out);

/* Kernel work counters (diagnostics). enable=1 zeroes and starts counting in
 * every following pass; enable=0 stops and writes the counters:
 *   [0] wave-iterations (64 points each)  [1] hull evaluations (per wave)
 *   [2] slow-path entries (per wave)      [3] lane-needs summed over evaluations
 *   [4] lanes on the slow path            [5] best-first seed evaluations
 *   [6] waves reaching the exhaustive scan [7] lanes in the exhaustive scan
 *   [8] candidate hulls after wave culling [9] faces of the evaluated hulls
 *   [10..18] reserved (0; the per-phase clocks live in the -DFSDF_WAVE_TIMES=1
 *   timeline build, tools/wave_times.py)
 *   [19] screened plane maxima that fell back to the full fp64 scan (per
 *   wave) [20] evaluations rejected early by the screen [21] descent-walk
 *   steps (per wave) [22..23] reserved (0). 24 counters. */
int fsdf_kernel_stats(fsdf_ctx* ctx, int32_t enable, uint64_t* counters_out);

#ifdef __cplusplus
}
#endif

#endif /* FLASHSDF_H */
