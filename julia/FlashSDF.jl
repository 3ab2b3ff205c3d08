# FlashSDF.jl — the Julia drop-in for Flash.jl's residual path over libflashsdf
# (include/flashsdf.h). To be `include`d from src/Flash.jl after
# gradientdescent.jl; src/tracking.jl:16 then builds
#     cost = FlashSDF.GPUCost(manipulator, sensed_points)
# instead of CostFunctor(manipulator, sensed_points) — the same callable with
# Float64 or ForwardDiff.Dual input (src/gradientdescent.jl:49-57).
#
# Julia 0.5 syntax, like the reference (REQUIRE.dev:1). Julia is not installed
# in this image, so this file is not executed here; its ccall signatures and C
# struct layouts are checked against include/flashsdf.h by
# tests/test_julia_shim.py, and its arithmetic mirrors the tested Python host
# (flash/gradientdescent.py, flash/rbf.py).
#
# How the gradient is formed. The reference differentiates the whole cost with
# ForwardDiff chunk passes: ⌈n/9⌉ Dual evaluations of every (point, surface)
# pair (examples/irb_and_squishable.ipynb:482-485). Here the per-point work runs
# ONCE per distinct value(x) on the GPU, which returns the cost and its
# first-order sensitivities to the scene geometry:
#   * per convex surface k: F_k = Σ 2d∇d, M_k = Σ 2d p×∇d (accum[1+6k..]), so
#     that a world twist (ω, v) of the surface changes the cost by
#     δc = −(ω·M_k + v·F_k);
#   * per RBF skin: λ = Σ 2s ∂s/∂(w, a, b) and E_i = Σ 2s ∂s/∂c_i.
# Everything upstream of the GPU — forward kinematics (RigidBodyDynamics,
# src/Flash.jl:248), normalize! (src/gradientdescent.jl:30), the deformed
# surface points (src/Flash.jl:143-201) and the RBF weight solve
# (src/Flash.jl:212) — is evaluated by the reference's own code in the Dual
# number type, and the chunk's partials are contracted with those
# sensitivities. The result is the first-order Dual the reference would
# produce, from one residual pass instead of ⌈n/9⌉.

module FlashSDF

import Flash
import Flash: Manipulator, ManipulatorState, ConvexGeometry, InterpolatingGeometry
import Flash.GradientDescent: unflatten!, default_deformation_cost_weight
import Base: normalize!   # extended for MechanismState in src/gradientdescent.jl:19-26
using RigidBodyDynamics
using CoordinateTransformations
import StaticArrays: SVector
import GeometryTypes
import ForwardDiff
import ForwardDiff: Dual, value, partials

const lib = get(ENV, "FLASHSDF_LIB", "libflashsdf")

const FSDF_SURFACE_HULL = Int32(0)
const FSDF_SURFACE_RBF = Int32(1)

# C structs of include/flashsdf.h (field order and types as declared there)
immutable Opts          # fsdf_opts
    device::Int32
    precision::Int32
    sort_points::Int32
    cull::Int32
end

immutable Hull          # fsdf_hull
    n_vertices::Int32
    n_faces::Int32
    vertices::Ptr{Float64}
    faces::Ptr{Int32}
    planes::Ptr{Float64}
end

immutable Surface       # fsdf_surface
    kind::Int32
    n_centers::Int32
    hull::Hull
end

last_error(ptr::Ptr{Void}) = unsafe_string(ccall((:fsdf_last_error, lib), Cstring, (Ptr{Void},), ptr))
check(ptr::Ptr{Void}, st::Cint, what) = st == 0 || error("flashsdf $what (status $st): ", last_error(ptr))

"conv(points) for a 3×n vertex matrix → (3×m vertices, 3×f zero-based faces, 4×f
planes): the shape EnhancedGJK's NeighborMesh support function sees (src/models.jl:152)."
function convex_hull(points::Matrix{Float64})
    n = size(points, 2)
    cap = max(2n - 4, 4)
    v = zeros(3, max(n, 4)); f = zeros(Int32, 3, cap); p = zeros(4, cap)
    nv = Ref{Int32}(0); nf = Ref{Int32}(0)
    st = ccall((:fsdf_convex_hull, lib), Cint,
               (Ptr{Float64}, Int32, Ref{Int32}, Ptr{Float64}, Ref{Int32}, Ptr{Int32}, Ptr{Float64}),
               points, n, nv, v, nf, f, p)
    st == 0 || error("fsdf_convex_hull: status $st")
    v[:, 1:nv[]], f[:, 1:nf[]], p[:, 1:nf[]]
end

"One device context holding the manipulator's surfaces (uploaded once)."
type Context
    ptr::Ptr{Void}
    manipulator::Manipulator
    S::Int
    accum_len::Int
    prefetched::Any   # the cloud fsdf_prefetch_points is copying (rooted until consumed)
end
Context(ptr, manip, S, accum_len) = Context(ptr, manip, S, accum_len, nothing)

function Context(manip::Manipulator; device::Integer=0, precision::Integer=64, sort_points::Bool=true)
    ref = Ref{Ptr{Void}}(C_NULL)
    st = ccall((:fsdf_create, lib), Cint, (Ref{Ptr{Void}}, Ref{Opts}),
               ref, Opts(device, precision, sort_points ? 1 : 0, 1))
    st == 0 || error("fsdf_create: no usable HIP device (status $st; libflashsdf has no CPU fallback)")
    keep = Any[]          # the hull arrays must outlive fsdf_set_surfaces (it copies them)
    descs = Surface[]
    for s in manip.surfaces
        if isa(s, ConvexGeometry)
            # the vertex set Flash.surface_points(::ConvexGeometry) uses (src/Flash.jl:143-148)
            verts = GeometryTypes.vertices(s.geometry)
            V = Float64[v[i] for i in 1:3, v in verts]
            hv, hf, hp = convex_hull(V)
            push!(keep, hv, hf, hp)
            push!(descs, Surface(FSDF_SURFACE_HULL, 0,
                                 Hull(size(hv, 2), size(hf, 2), pointer(hv), pointer(hf), pointer(hp))))
        else
            n = length(s.surface_points) + length(s.skeleton_points)
            push!(descs, Surface(FSDF_SURFACE_RBF, n, Hull(0, 0, C_NULL, C_NULL, C_NULL)))
        end
    end
    check(ref[], ccall((:fsdf_set_surfaces, lib), Cint, (Ptr{Void}, Ptr{Surface}, Int32),
                       ref[], descs, length(descs)), "set_surfaces")
    len = Ref{Int32}(0)
    check(ref[], ccall((:fsdf_accum_len, lib), Cint, (Ptr{Void}, Ref{Int32}), ref[], len), "accum_len")
    ctx = Context(ref[], manip, length(descs), len[])
    finalizer(ctx, c -> ccall((:fsdf_destroy, lib), Cint, (Ptr{Void},), c.ptr))
    ctx
end

"Upload the sensed cloud once per frame (CostFunctor keeps it by reference,
src/gradientdescent.jl:41-47). Vector{SVector{3,Float64}} is a contiguous AoS
buffer of 3n doubles: passed zero-copy."
function set_points!{T}(ctx::Context, pts::AbstractVector{SVector{3, T}})
    P = convert(Vector{SVector{3, Float64}}, pts)
    check(ctx.ptr, ccall((:fsdf_set_points, lib), Cint, (Ptr{Void}, Ptr{Float64}, Int64),
                         ctx.ptr, reinterpret(Float64, P), length(P)), "set_points")
end

"Start the NEXT frame's upload now (fsdf_prefetch_points: a copy on the context's
own stream, under the current frame's iterations — overlapped when the buffer is
page-locked); set_points_prefetched! makes it resident. The buffer is rooted in the
context until then and must not change."
function prefetch_points!{T}(ctx::Context, pts::AbstractVector{SVector{3, T}})
    P = convert(Vector{SVector{3, Float64}}, pts)
    check(ctx.ptr, ccall((:fsdf_prefetch_points, lib), Cint, (Ptr{Void}, Ptr{Float64}, Int64),
                         ctx.ptr, reinterpret(Float64, P), length(P)), "prefetch_points")
    ctx.prefetched = P
end

function set_points_prefetched!(ctx::Context)
    check(ctx.ptr, ccall((:fsdf_set_points_prefetched, lib), Cint, (Ptr{Void},), ctx.ptr), "set_points_prefetched")
    ctx.prefetched = nothing
end

"One GPU's shard of the frame's cloud (the cost is a sum over points,
src/gradientdescent.jl:32): the whole cloud is Hilbert-sorted on the device and
this context keeps the contiguous range [first, last] (1-based, inclusive) of
that order — the partition of DESIGN.md §6, balanced by fsdf_chunk_costs."
function set_points_range!{T}(ctx::Context, pts::AbstractVector{SVector{3, T}}, first::Integer, last::Integer)
    P = convert(Vector{SVector{3, Float64}}, pts)
    check(ctx.ptr, ccall((:fsdf_set_points_range, lib), Cint, (Ptr{Void}, Ptr{Float64}, Int64, Int64, Int64),
                         ctx.ptr, reinterpret(Float64, P), length(P), first - 1, last), "set_points_range")
end

"Once per frame, after its first cost evaluation: regroup the resident cloud by
each point's nearest surface in that pass (fsdf_regroup_points). The frame's
later evaluations (the rest of track!'s iterations, src/tracking.jl:8-27) give
the same per-point results and evaluate fewer hulls per 64-point chunk."
regroup_points!(ctx::Context) = check(ctx.ptr, ccall((:fsdf_regroup_points, lib), Cint, (Ptr{Void},), ctx.ptr),
                                      "regroup_points")

"The same where the library's rule says it pays (fsdf_regroup_auto: the last pass
ran one wave per 64-point chunk — clouds above the planned window); true when it
regrouped. GPUCost applies it after a new cloud's first evaluation."
function regroup_auto!(ctx::Context)
    applied = Ref{Int32}(0)
    check(ctx.ptr, ccall((:fsdf_regroup_auto, lib), Cint, (Ptr{Void}, Ref{Int32}), ctx.ptr, applied), "regroup_auto")
    applied[] != 0
end

"The posed scene in the state's number type (Float64 or Dual): per surface the
world pose (R, t) (identity for RBF skins) and, per RBF skin, its world centres
and solved coefficients u = (w; a; b)."
immutable SceneGeometry{T}
    R::Vector{Matrix{T}}
    t::Vector{Vector{T}}
    centres::Vector{Vector{SVector{3, T}}}
    u::Vector{Vector{T}}
end

function scene_geometry{P, T}(state::ManipulatorState{P, T, T})
    R = Matrix{T}[]; t = Vector{T}[]; C = Vector{SVector{3, T}}[]; U = Vector{T}[]
    o = SVector{3, Float64}(0, 0, 0)
    for s in state.manipulator.surfaces
        if isa(s, ConvexGeometry)
            A = convert(AffineMap, transform_to_root(state.mechanism_state, s.frame))   # src/Flash.jl:248
            push!(R, Matrix{T}(transform_deriv(A, o)))
            push!(t, Vector{T}(A(o)))
        else
            push!(R, eye(T, 3)); push!(t, zeros(T, 3))
            # src/Flash.jl:207-212: surface points (value 0, deformed) and skeleton points (value −1)
            sp = Flash.surface_points(state, s)
            kp = Flash.skeleton_points(state, s)
            c = vcat(sp, kp)
            n = length(c)
            M = zeros(T, n + 4, n + 4)   # [A P; Pᵀ 0], A_ij = |c_i − c_j|³ (XCubed), P_i = [1 c_iᵀ]
            for i in 1:n, j in 1:n
                M[i, j] = i == j ? zero(T) : norm(c[i] - c[j])^3
            end
            for i in 1:n
                M[i, n + 1] = M[n + 1, i] = one(T)
                for d in 1:3
                    M[i, n + 1 + d] = M[n + 1 + d, i] = c[i][d]
                end
            end
            rhs = vcat(zeros(T, length(sp)), -ones(T, length(kp)), zeros(T, 4))
            push!(C, c)
            push!(U, M \ rhs)
        end
    end
    SceneGeometry{T}(R, t, C, U)
end

"(poses [12 × S] row-major R then t; RBF rows [4 × Σ(n+1)]: (c_i, w_i) then (a, b))."
function device_inputs(geo::SceneGeometry)
    S = length(geo.R)
    poses = zeros(12, S)
    for k in 1:S
        R = map(value, geo.R[k])
        poses[1:9, k] = vec(R')
        poses[10:12, k] = map(value, geo.t[k])
    end
    rows = Float64[]
    for (c, u) in zip(geo.centres, geo.u)
        n = length(c)
        for i in 1:n
            append!(rows, [value(c[i][1]), value(c[i][2]), value(c[i][3]), value(u[i])])
        end
        append!(rows, map(value, u[n + 1:n + 4]))
    end
    poses, rows
end

"Drop-in for CostFunctor(manipulator, sensed_points) (src/gradientdescent.jl:41-57)."
type GPUCost{P} <: Function
    manipulator::Manipulator{P}
    ctx::Context
    states::Dict{DataType, ManipulatorState}   # one per number type, as CostFunctor caches it (:50-53)
    memo_x::Vector{Float64}
    memo_accum::Vector{Float64}
    weight::Float64
    fresh::Bool   # the resident cloud has not been evaluated yet (the regroup follows its first pass)
end

function GPUCost(manipulator::Manipulator, sensed_points::AbstractVector;
                 device::Integer=0, deformation_cost_weight=default_deformation_cost_weight)
    ctx = Context(manipulator; device=device)
    set_points!(ctx, sensed_points)
    GPUCost(manipulator, ctx, Dict{DataType, ManipulatorState}(), Float64[], Float64[],
            Float64(deformation_cost_weight), true)
end

function state_for{T}(f::GPUCost, ::Type{T})
    get!(f.states, T) do
        ManipulatorState(f.manipulator, T, T)
    end
end

"One residual pass per distinct value(x): cost Σ d² and the accumulator."
function residual_pass!(f::GPUCost, geo::SceneGeometry, xv::Vector{Float64})
    if xv != f.memo_x
        poses, rows = device_inputs(geo)
        if !isempty(rows)
            check(f.ctx.ptr, ccall((:fsdf_set_rbf_params, lib), Cint, (Ptr{Void}, Ptr{Float64}, Int64),
                                   f.ctx.ptr, rows, length(rows)), "set_rbf_params")
        end
        accum = zeros(f.ctx.accum_len)   # 1 + 6S + Σ(4n+4) (fsdf_accum_len)
        c = Ref{Float64}(0)
        check(f.ctx.ptr, ccall((:fsdf_eval, lib), Cint,
                               (Ptr{Void}, Ptr{Float64}, Ref{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64},
                                Ptr{Float64}),
                               f.ctx.ptr, poses, c, accum, C_NULL, C_NULL, C_NULL), "eval")
        if f.fresh   # once per frame, after its first pass (per-point results unchanged, sums to rounding)
            regroup_auto!(f.ctx)
            f.fresh = false
        end
        f.memo_x = copy(xv)
        f.memo_accum = accum
    end
    f.memo_accum
end

# Σ_p d*(p)² as a number of the state's type: the value from the pass; for a
# Dual chunk, the first-order change of the cost through every surface pose
# (δc = −(ω·(M − t×F) + δt·F) with ω = vee(δR Rᵀ)) and every RBF skin's
# centres and coefficients (δc = Σ E_i·δc_i + λ·δu).
assemble(geo::SceneGeometry{Float64}, accum::Vector{Float64}) = accum[1]

function assemble{N, V}(geo::SceneGeometry{Dual{N, V}}, accum::Vector{Float64})
    g = zeros(N)
    S = length(geo.R)
    for k in 1:S
        F = accum[2 + 6(k - 1):4 + 6(k - 1)]
        M = accum[5 + 6(k - 1):7 + 6(k - 1)]
        Rk = geo.R[k]; tk = geo.t[k]
        Rv = map(value, Rk); tv = map(value, tk)
        Mo = M - cross(tv, F)
        for p in 1:N
            dR = Float64[partials(Rk[i, j], p) for i in 1:3, j in 1:3]
            W = dR * Rv'
            ω = 0.5 * [W[3, 2] - W[2, 3], W[1, 3] - W[3, 1], W[2, 1] - W[1, 2]]
            dt = Float64[partials(tk[i], p) for i in 1:3]
            g[p] -= dot(ω, Mo) + dot(dt, F)
        end
    end
    off = 2 + 6S
    for (c, u) in zip(geo.centres, geo.u)
        n = length(c)
        lam = accum[off:off + n + 3]             # λ_w (n), λ_a, λ_b (3)
        E = accum[off + n + 4:off + 4n + 3]      # E_i (3 each)
        off += 4n + 4
        for p in 1:N
            s = 0.0
            for i in 1:n, d in 1:3
                s += E[3(i - 1) + d] * partials(c[i][d], p)
            end
            for i in 1:n + 4
                s += lam[i] * partials(u[i], p)
            end
            g[p] += s
        end
    end
    Dual(accum[1], ForwardDiff.Partials(tuple(g...)))
end

function (f::GPUCost){T}(x::AbstractVector{T})
    state = state_for(f, T)
    unflatten!(state, x)
    normalize!(state.mechanism_state)   # src/gradientdescent.jl:30 — in T, so its projection reaches the partials
    geo = scene_geometry(state)
    accum = residual_pass!(f, geo, Float64[value(xi) for xi in x])
    c = assemble(geo, accum)
    for deformation_set in values(state.deformations)   # src/gradientdescent.jl:33-37
        for deformation in deformation_set
            c += f.weight * sum(deformation .^ 2)
        end
    end
    c
end

"Flash.skin(state) (src/Flash.jl:265-268) on the device: x -> minimum over surfaces."
function skin(ctx::Context, state::ManipulatorState)
    poses, rows = device_inputs(scene_geometry(state))
    if !isempty(rows)
        check(ctx.ptr, ccall((:fsdf_set_rbf_params, lib), Cint, (Ptr{Void}, Ptr{Float64}, Int64),
                             ctx.ptr, rows, length(rows)), "set_rbf_params")
    end
    function (x)
        d = Ref{Float64}(0); k = Ref{Int32}(0); g = zeros(3)
        xyz = Float64[x[1], x[2], x[3]]
        check(ctx.ptr, ccall((:fsdf_skin, lib), Cint,
                             (Ptr{Void}, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}),
                             ctx.ptr, poses, xyz, 1, d, k, g), "skin")
        d[]
    end
end

end # module
