# KinematicsHIP.jl -- Julia-side drop-in for Kinematics.jl's hot path on MI355X.
#
# Binds libkinhip.so (include/kinhip.h) with `ccall`.  Keeps the reference's
# Mechanism / parse_urdf / find_link / set_joint_angles API untouched (they stay
# in Kinematics.jl) and adds batched methods of the hot-path functions:
#
#   get_transform(m, link)                 src/algorithm.jl:1-4     -> get_transform(hm, links, joints, Q)
#   get_jacobian!(m, link, joints, ...)    src/algorithm.jl:83-106  -> get_jacobian!(hm, link, joints, with_rot, J, Q; rpy_jac)
#   inverse_kinematics!(m, link, ...)      src/inverse_kinematics.jl:23-30 -> inverse_kinematics!(hm, link, joints, targets, Q)
#   point_inverse_kinematics_nakamura      src/algorithm.jl:116-131 -> point_inverse_kinematics_nakamura!(hm, link, joints, points, Q)
#
# and the reference's own single-target signatures, unchanged but for `hm` in place of `m`:
#   inverse_kinematics!(hm, link, joints, target::Transform; ftol, with_rot) -> (q, :FTOL_REACHED | ...)
#   inverse_kinematics!(hm, link, joints, target::Transform, sscc, sdf; use_bistage, ftol, with_rot) -> (q, status)
#   compute_coll_dists(hm, sscc, joints, sdf), compute_coll_dists_and_grads(hm, sscc, joints, sdf; truncation_dist)
#
# Device arrays are AMDGPU.jl `ROCArray`s in Julia's column-major layout:
#   Q :: ROCMatrix{T}(N, n_joints [+3 base])      (configuration index fastest)
#   poses :: ROCArray{T,3}(N, 12, n_links)        (3x4 column-major per link)
#   J :: ROCArray{T,3}(N, rows, n_cols)           (get_jacobian!'s mat_out per configuration)
# which is exactly the SoA layout of the C-ABI, so `pointer(A)` is passed
# zero-copy.  T is Float32 or Float64.
#
# NOTE: this file is not executed in the build container (no Julia toolchain);
# the same C-ABI is exercised by tests/ through Python ctypes.
module KinematicsHIP

using Kinematics
using Kinematics: Joint  # (not in Kinematics.jl's export list, src/Kinematics.jl:45-73)
using AMDGPU

const libkinhip = joinpath(@__DIR__, "..", "lib", "libkinhip.so")
const KINHIP_ABI_VERSION = 2  # include/kinhip.h: the layout of KinIkParams below

function __init__()
    v = ccall((:kin_abi_version, libkinhip), Cint, ())
    v == KINHIP_ABI_VERSION || error("$libkinhip: C-ABI version $v, KinematicsHIP needs $KINHIP_ABI_VERSION (rebuild)")
end

const KIN_F32 = Int32(0)
const KIN_F64 = Int32(1)
const KIN_WITH_ROT = UInt32(1)
const KIN_RPY_JAC = UInt32(2)
const KIN_ZERO_FILL = UInt32(4)

struct KinTreeDesc
    n_links::Int32
    n_joints::Int32
    joint_type::Ptr{Int32}
    joint_plink::Ptr{Int32}
    joint_clink::Ptr{Int32}
    joint_pose::Ptr{Float64}
    joint_axis::Ptr{Float64}
    joint_lower::Ptr{Float64}
    joint_upper::Ptr{Float64}
    with_base::Int32
end

struct KinPlanDesc
    dtype::Int32
    n_q::Int32
    q_joint_ids::Ptr{Int32}
    n_out::Int32
    out_link_ids::Ptr{Int32}
    jac_link_id::Int32
    n_jac::Int32
    jac_joint_ids::Ptr{Int32}
    jac_flags::UInt32
end

struct KinIkParams
    max_iters::Int32
    lambda::Float64
    tol_pos::Float64
    tol_rot::Float64
    max_step::Float64
    with_rot::Int32
    restarts::Int32
    seed::UInt64
    lanes::Int32
    index_base::Int64
    damp_err::Float64
end

function check(rc::Cint)
    if rc != 0
        msg = unsafe_string(ccall((:kin_last_error, libkinhip), Cstring, ()))
        rc == -2 && throw(KeyError(msg))                   # reference: Dict KeyError
        rc == -3 && throw(MethodError(joint_jacobian_stub, (msg,)))  # no joint_jacobian! method (fixed joint)
        error("kinhip error $rc: $msg")
    end
    nothing
end
joint_jacobian_stub(x) = nothing

joint_type_code(::Kinematics.Joint{Kinematics.Fixed}) = Int32(0)
joint_type_code(::Kinematics.Joint{Kinematics.Revolute}) = Int32(1)
joint_type_code(::Kinematics.Joint{Kinematics.Prismatic}) = Int32(2)
joint_axis(j::Kinematics.Joint{Kinematics.Fixed}) = (1.0, 0.0, 0.0)
joint_axis(j::Kinematics.Joint) = Tuple(j.jt.axis)

"""HIP-side model of a Mechanism.  Follows the Mechanism's state the way the reference's methods do
(they read `m.angles` and the tree on every call, src/mechanism.jl:223-231, src/algorithm.jl:1-37):
every batched call goes through `sync!`, which
  * rebuilds the C model when `add_new_link` grew the tree (length(m.links) / length(m.joints)),
  * pushes `m.angles` to kin_model_set_angles when they changed since the last push,
and `plan!` / `coll_plan!` re-stage a cached plan whose baked angles (the joints it does NOT take as
batch columns, `baked_angles`) differ from the current ones.  So `set_joint_angles(m, [head_pan], ...)`
or `add_new_link` followed by a batched call sees the new state, as in the reference."""
mutable struct HIPModel
    handle::Ptr{Cvoid}
    m::Mechanism
    plans::Dict{Any,Tuple{Ptr{Cvoid},Vector{Float64}}}  # request => (kin_plan, angles it baked in)
    specialize::Bool  # compile every new plan into constant-folded kernels (kin_plan_specialize)
    angles::Vector{Float64}  # m.angles as last passed to kin_model_set_angles
    n_links::Int             # length(m.links) the C model was built with
end

function model_handle(m::Mechanism)
    J = length(m.joints)
    jt = Int32[joint_type_code(j) for j in m.joints]
    jp = Int32[j.plink_id for j in m.joints]
    jc = Int32[j.clink_id for j in m.joints]
    pose = Float64[]
    axis = Float64[]
    for j in m.joints
        append!(pose, vec(Matrix(j.pose.mat)))          # column-major 4x4
        append!(axis, collect(joint_axis(j)))
    end
    lo = Float64[Kinematics.lower_limit(j) for j in m.joints]
    hi = Float64[Kinematics.upper_limit(j) for j in m.joints]
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve jt jp jc pose axis lo hi begin
        d = KinTreeDesc(length(m.links), J, pointer(jt), pointer(jp), pointer(jc), pointer(pose), pointer(axis),
                        pointer(lo), pointer(hi), Int32(m.with_base))
        check(ccall((:kin_model_create, libkinhip), Cint, (Ref{KinTreeDesc}, Ref{Ptr{Cvoid}}), d, h))
    end
    check(ccall((:kin_model_set_angles, libkinhip), Cint, (Ptr{Cvoid}, Ptr{Float64}), h[], m.angles))
    h[]
end

function free_plans!(hm::HIPModel)
    for (p, _) in values(hm.plans)
        ccall((:kin_plan_destroy, libkinhip), Cint, (Ptr{Cvoid},), p)
    end
    empty!(hm.plans)
end

function HIPModel(m::Mechanism; specialize::Bool=true)
    hm = HIPModel(model_handle(m), m, Dict{Any,Tuple{Ptr{Cvoid},Vector{Float64}}}(), specialize, copy(m.angles),
                  length(m.links))
    finalizer(hm) do x
        free_plans!(x)
        ccall((:kin_model_destroy, libkinhip), Cint, (Ptr{Cvoid},), x.handle)
    end
    hm
end

"""Bring the C model up to the Mechanism's current tree and angles (see HIPModel)."""
function sync!(hm::HIPModel)
    m = hm.m
    if length(m.links) != hm.n_links || length(m.angles) != length(hm.angles)  # add_new_link
        free_plans!(hm)
        ccall((:kin_model_destroy, libkinhip), Cint, (Ptr{Cvoid},), hm.handle)
        hm.handle = model_handle(m)
        hm.n_links = length(m.links)
        hm.angles = copy(m.angles)
    elseif m.angles != hm.angles  # set_joint_angle(s) since the last call
        check(ccall((:kin_model_set_angles, libkinhip), Cint, (Ptr{Cvoid}, Ptr{Float64}), hm.handle, m.angles))
        hm.angles = copy(m.angles)
    end
    hm
end

"""The angles a plan over batch joints `qj` bakes in: m.angles with the batch joints zeroed."""
function baked_angles(m::Mechanism, qj::Vector{Int32})
    a = copy(m.angles)
    a[qj] .= 0.0
    a
end

dtype_code(::Type{Float32}) = KIN_F32
dtype_code(::Type{Float64}) = KIN_F64

"""Cached plan for a request, re-staged when the angles it baked in changed (after sync!)."""
function cached_plan!(make, hm::HIPModel, key, qj::Vector{Int32})
    sync!(hm)
    baked = baked_angles(hm.m, qj)
    hit = get(hm.plans, key, nothing)
    if hit !== nothing
        hit[2] == baked && return hit[1]
        ccall((:kin_plan_destroy, libkinhip), Cint, (Ptr{Cvoid},), hit[1])
        delete!(hm.plans, key)
    end
    p = make()
    hm.plans[key] = (p, baked)
    p
end

function plan!(hm::HIPModel, ::Type{T}, qj, outs, jl, jj, flags) where {T}
    key = (T, qj, outs, jl, jj, flags)
    cached_plan!(hm, key, qj) do
        h = Ref{Ptr{Cvoid}}(C_NULL)
        GC.@preserve qj outs jj begin
            d = KinPlanDesc(dtype_code(T), length(qj), pointer(qj), length(outs), pointer(outs), jl, length(jj),
                            pointer(jj), flags)
            check(ccall((:kin_plan_create, libkinhip), Cint, (Ptr{Cvoid}, Ref{KinPlanDesc}, Ref{Ptr{Cvoid}}),
                        hm.handle, d, h))
        end
        # every kernel kind that applies (0); a failed compilation leaves the generic kernels
        hm.specialize && ccall((:kin_plan_specialize, libkinhip), Cint, (Ptr{Cvoid}, UInt32), h[], UInt32(0))
        h[]
    end
end

stream_ptr() = AMDGPU.stream().stream

# Device batches: a ROCArray, or a view of one whose first dimension is contiguous (a padded batch from
# batch_array); pointer() and stride(A, 2) give the C-ABI's base pointer and leading dimension.
const DevMat{T} = Union{ROCMatrix{T},SubArray{T,2,<:ROCArray{T}}}
const DevArr3{T} = Union{ROCArray{T,3},SubArray{T,3,<:ROCArray{T}}}

"""`batch_array(T, N, dims...)`: an (N, dims...) device batch in the C-ABI's SoA layout (configuration index
fastest) whose leading dimension is padded to N + 256.  Use it for Q, J and poses at batch sizes that are
powers of two: rows exactly 2^k elements apart fall on the same Infinity-Cache sets and lose the cache's
reuse between launches (2^20 FK + J: 47.5 us with ld = N against 41 us padded, DESIGN.md section 3).  A
view of the first N rows; passed zero-copy."""
function batch_array(::Type{T}, N::Integer, dims::Integer...; pad::Integer=256) where {T}
    A = ROCArray{T}(undef, N + pad, dims...)
    view(A, 1:N, ntuple(_ -> Colon(), length(dims))...)
end

"""Batched `get_transform`: poses[:, :, k] = world pose (3x4, column-major) of links[k] for every row of Q."""
function Kinematics.get_transform(hm::HIPModel, links::Vector{<:Link}, joints::Vector{<:Joint},
                                  Q::DevMat{T}) where {T<:Union{Float32,Float64}}
    N = size(Q, 1)
    poses = batch_array(T, N, 12, length(links))  # (padded rows, see batch_array)
    p = plan!(hm, T, Int32[j.id for j in joints], Int32[l.id for l in links], Int32(0), Int32[], UInt32(0))
    check(ccall((:kin_plan_run, libkinhip), Cint,
                (Ptr{Cvoid}, Ptr{T}, Int64, Int64, Ptr{T}, Int64, Ptr{T}, Int64, Ptr{Cvoid}),
                p, pointer(Q), stride(Q, 2), N, pointer(poses), stride(poses, 2), C_NULL, 0, stream_ptr()))
    poses
end

"""Batched `get_jacobian!`: J[i, :, :] is mat_out of configuration i; untouched entries keep their values."""
function Kinematics.get_jacobian!(hm::HIPModel, link::Link, joints::Vector{<:Joint}, with_rot::Bool,
                                  J::DevArr3{T}, Q::DevMat{T}; rpy_jac=false,
                                  pose::Union{Nothing,DevArr3{T}}=nothing) where {T<:Union{Float32,Float64}}
    N = size(Q, 1)
    flags = (with_rot ? KIN_WITH_ROT : UInt32(0)) | (rpy_jac ? KIN_RPY_JAC : UInt32(0))
    ids = Int32[j.id for j in joints]
    outs = pose === nothing ? Int32[] : Int32[link.id]
    p = plan!(hm, T, ids, outs, Int32(link.id), ids, flags)
    check(ccall((:kin_plan_run, libkinhip), Cint,
                (Ptr{Cvoid}, Ptr{T}, Int64, Int64, Ptr{T}, Int64, Ptr{T}, Int64, Ptr{Cvoid}),
                p, pointer(Q), stride(Q, 2), N, pose === nothing ? C_NULL : pointer(pose),
                pose === nothing ? N : stride(pose, 2), pointer(J), stride(J, 2), stream_ptr()))
    J
end

"""Batched `get_jacobian!` on the tiled layout (kin_plan_run_tiled, DESIGN.md section 3):
Q is (tile, dof, ntiles), J (tile, rows, cols, ntiles), pose (tile, 12, ntiles) or nothing; N <= tile * ntiles
configurations, configuration i at [i % tile + 1, ..., i ÷ tile + 1]."""
function get_jacobian_tiled!(hm::HIPModel, link::Link, joints::Vector{<:Joint}, with_rot::Bool, J::ROCArray{T,4},
                             Q::ROCArray{T,3}, N::Integer; rpy_jac=false,
                             pose::Union{Nothing,ROCArray{T,3}}=nothing) where {T<:Union{Float32,Float64}}
    tile = size(Q, 1)
    flags = (with_rot ? KIN_WITH_ROT : UInt32(0)) | (rpy_jac ? KIN_RPY_JAC : UInt32(0))
    ids = Int32[j.id for j in joints]
    outs = pose === nothing ? Int32[] : Int32[link.id]
    p = plan!(hm, T, ids, outs, Int32(link.id), ids, flags)
    check(ccall((:kin_plan_run_tiled, libkinhip), Cint,
                (Ptr{Cvoid}, Int64, Ptr{T}, Int64, Int64, Int64, Ptr{T}, Int64, Int64, Ptr{T}, Int64, Int64, Ptr{Cvoid}),
                p, tile, pointer(Q), stride(Q, 2), stride(Q, 3), N,
                pose === nothing ? C_NULL : pointer(pose), tile, pose === nothing ? 0 : stride(pose, 3),
                pointer(J), tile, stride(J, 4), stream_ptr()))
    J
end

function Kinematics.get_jacobian(hm::HIPModel, link::Link, joints::Vector{<:Joint}, with_rot::Bool,
                                 Q::DevMat{T}; rpy_jac=false) where {T}
    rows = with_rot ? 6 : 3
    cols = length(joints) + (hm.m.with_base ? 3 : 0)
    J = batch_array(T, size(Q, 1), rows, cols)  # (padded rows, see batch_array)
    fill!(J, zero(T))
    Kinematics.get_jacobian!(hm, link, joints, with_rot, J, Q; rpy_jac=rpy_jac)
end

"""Batched IK (damped least squares on the GPU): targets (N, 12) 3x4 poses, Q (N, dof) seeds, solved in place.
Returns (Q, iters, err); converged where iters <= max_iters (max_iters + 1: no attempt converged).
`rpy_objective=true` solves the reference's own objective (f_objective, src/inverse_kinematics.jl:38-50:
[p* - p; rpy* - rpy] with the rpy_jac Jacobian; tol_rot then bounds |d rpy|)."""
function Kinematics.inverse_kinematics!(hm::HIPModel, link::Link, joints::Vector{<:Joint}, targets::ROCMatrix{T},
                                        Q::ROCMatrix{T}; max_iters=64, lambda=1e-2, tol_pos=1e-3, tol_rot=1e-3,
                                        max_step=0.5, with_rot=true, rpy_objective=false, restarts=0, seed=0, lanes=0,
                                        index_base=0, damp_err=0.0) where {T}
    N = size(Q, 1)
    ids = Int32[j.id for j in joints]
    p = plan!(hm, T, ids, Int32[link.id], Int32(link.id), ids, KIN_WITH_ROT)
    iters = ROCVector{Int32}(undef, N)
    err = ROCMatrix{T}(undef, N, 2)
    mode = with_rot ? (rpy_objective ? 2 : 1) : 0
    prm = KinIkParams(max_iters, lambda, tol_pos, tol_rot, max_step, mode, restarts, seed, lanes, index_base, damp_err)
    check(ccall((:kin_ik_dls_batch, libkinhip), Cint,
                (Ptr{Cvoid}, Ref{KinIkParams}, Ptr{T}, Int64, Ptr{T}, Int64, Int64, Ptr{Int32}, Ptr{T}, Int64,
                 Ptr{Cvoid}),
                p, prm, pointer(targets), stride(targets, 2), pointer(Q), stride(Q, 2), N, pointer(iters),
                pointer(err), N, stream_ptr()))
    Q, iters, err
end

"""Batched IK from the seeds Q0 (N, dof; not modified) into Q (written, not read): the same results as
copyto!(Q, Q0) followed by inverse_kinematics!, without the copy (kin_ik_dls_batch_from)."""
function inverse_kinematics_from!(hm::HIPModel, link::Link, joints::Vector{<:Joint}, targets::ROCMatrix{T},
                                  Q0::ROCMatrix{T}, Q::ROCMatrix{T}; max_iters=64, lambda=1e-2, tol_pos=1e-3,
                                  tol_rot=1e-3, max_step=0.5, with_rot=true, restarts=0, seed=0, lanes=0,
                                  index_base=0, damp_err=0.0) where {T}
    N = size(Q, 1)
    size(Q0) == size(Q) && stride(Q0, 2) == stride(Q, 2) || throw(DimensionMismatch("Q0 and Q differ in shape"))
    ids = Int32[j.id for j in joints]
    p = plan!(hm, T, ids, Int32[link.id], Int32(link.id), ids, KIN_WITH_ROT)
    iters = ROCVector{Int32}(undef, N)
    err = ROCMatrix{T}(undef, N, 2)
    prm = KinIkParams(max_iters, lambda, tol_pos, tol_rot, max_step, with_rot, restarts, seed, lanes, index_base,
                      damp_err)
    check(ccall((:kin_ik_dls_batch_from, libkinhip), Cint,
                (Ptr{Cvoid}, Ref{KinIkParams}, Ptr{T}, Int64, Ptr{T}, Ptr{T}, Int64, Int64, Ptr{Int32}, Ptr{T},
                 Int64, Ptr{Cvoid}),
                p, prm, pointer(targets), stride(targets, 2), pointer(Q0), pointer(Q), stride(Q, 2), N,
                pointer(iters), pointer(err), N, stream_ptr()))
    Q, iters, err
end

function point_inverse_kinematics_nakamura!(hm::HIPModel, link::Link, joints::Vector{<:Joint},
                                            points::ROCMatrix{T}, Q::ROCMatrix{T}) where {T}
    N = size(Q, 1)
    ids = Int32[j.id for j in joints]
    p = plan!(hm, T, ids, Int32[], Int32(link.id), ids, UInt32(0))
    check(ccall((:kin_point_ik_nakamura_batch, libkinhip), Cint,
                (Ptr{Cvoid}, Ptr{T}, Int64, Ptr{T}, Int64, Int64, Ptr{Cvoid}),
                p, pointer(points), stride(points, 2), pointer(Q), stride(Q, 2), N, stream_ptr()))
    Q
end

# --- collision (src/sdf.jl, src/collision.jl) and planning constraints (src/planning.jl) ---

struct KinCollDesc
    dtype::Int32
    n_q::Int32
    q_joint_ids::Ptr{Int32}
    n_spheres::Int32
    sphere_link_ids::Ptr{Int32}
    centers::Ptr{Float64}
    radii::Ptr{Float64}
end

struct KinIkCollParams
    margin::Float64
    band::Float64
    weight::Float64
    feas::Float64
end

"""Device copy of a UnionSDF of BoxSDFs (or a single BoxSDF); `n_scene_cols` > 0 (or `attached`):
the boxes ride on a scene mechanism's links (kin_sdf_create_attached) and every batched call takes
the scene columns."""
mutable struct HIPSDF
    handle::Ptr{Cvoid}
    attached::Bool
    n_scene_cols::Int
    scene::Union{Nothing,HIPModel}  # keeps the scene model alive
end
HIPSDF(h::Ptr{Cvoid}) = HIPSDF(h, false, 0, nothing)

function HIPSDF(sdf::Kinematics.AbstractSDF)
    boxes = sdf isa Kinematics.UnionSDF ? sdf.sdfs : [sdf]
    poses = Float64[]
    widths = Float64[]
    for b in boxes
        # a box of UnionSDF(mechanism) (src/sdf.jl:82-97) is attached to a link of the scene: its world pose is
        # written into b.pose by the SdfLinkType get_transform override (:14-20), which inv_pose runs when
        # the link is not cached (:24-32) -- so the snapshot is the box at the scene's current angles
        Kinematics.inv_pose(b)
        append!(poses, vec(Matrix(b.pose.mat)))
        append!(widths, collect(b.width))
    end
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:kin_sdf_create_boxes, libkinhip), Cint, (Int32, Ptr{Float64}, Ptr{Float64}, Ref{Ptr{Cvoid}}),
                length(boxes), poses, widths, h))
    s = HIPSDF(h[])
    finalizer(x -> ccall((:kin_sdf_destroy, libkinhip), Cint, (Ptr{Cvoid},), x.handle), s)
    s
end

"""UnionSDF(scene) (src/sdf.jl:82-97) that keeps following the scene: one box per link with box collision
geometry, attached to that link (attach_to_link, :43-46); `joints` (+ the scene's base) are the scene
columns of compute_coll_dists_and_grads!(...; scene_q) -- one value per column for the batch, or one
column per configuration (e.g. a door-angle sweep)."""
function HIPSDF(scene::Mechanism, joints::Vector{<:Joint})
    links = [l for l in scene.links if l.geometric_meta_data isa Kinematics.BoxMetaData]
    org = Float64[]
    wid = Float64[]
    for l in links
        append!(org, vec(Matrix(l.geometric_meta_data.origin.mat)))
        append!(wid, collect(l.geometric_meta_data.extents))
    end
    hm = HIPModel(scene; specialize=false)  # the scene's other joints at their current angles
    jids = Int32[j.id for j in joints]
    lids = Int32[l.id for l in links]
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:kin_sdf_create_attached, libkinhip), Cint,
                (Ptr{Cvoid}, Int32, Ptr{Int32}, Int32, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Ref{Ptr{Cvoid}}),
                hm.handle, length(jids), jids, length(lids), lids, org, wid, h))
    s = HIPSDF(h[], true, length(joints) + (scene.with_base ? 3 : 0), hm)
    finalizer(x -> ccall((:kin_sdf_destroy, libkinhip), Cint, (Ptr{Cvoid},), x.handle), s)
    s
end

function coll_plan!(hm::HIPModel, ::Type{T}, sscc::Kinematics.SweptSphereCollisionChecker,
                    joints::Vector{<:Joint}) where {T}
    ids = Int32[j.id for j in joints]
    sph = Int32[l.id for l in sscc.sphere_links]
    key = (:coll, T, ids, sph)
    cached_plan!(hm, key, ids) do
        h = Ref{Ptr{Cvoid}}(C_NULL)
        r = Float64.(sscc.sphere_radii)
        GC.@preserve ids sph r begin
            d = KinCollDesc(dtype_code(T), length(ids), pointer(ids), length(sph), pointer(sph), C_NULL, pointer(r))
            check(ccall((:kin_coll_plan_create, libkinhip), Cint, (Ptr{Cvoid}, Ref{KinCollDesc}, Ref{Ptr{Cvoid}}),
                        hm.handle, d, h))
        end
        hm.specialize && ccall((:kin_plan_specialize, libkinhip), Cint, (Ptr{Cvoid}, UInt32), h[], UInt32(0))
        h[]
    end
end

"""Batched `compute_coll_dists_and_grads!`: vals (N, n_spheres), grads (N, n_dof, n_spheres) for every row of Q.
`hm` must be built after the spheres were added (`add_coll_links`)."""
function compute_coll_dists_and_grads!(hm::HIPModel, sscc::Kinematics.SweptSphereCollisionChecker,
                                       joints::Vector{<:Joint}, sdf::HIPSDF, Q::ROCMatrix{T},
                                       vals::ROCMatrix{T}, grads::Union{Nothing,ROCArray{T,3}};
                                       truncation_dist=Inf, scene_q=nothing) where {T}
    N = size(Q, 1)
    p = coll_plan!(hm, T, sscc, joints)
    if sdf.attached
        scene_q === nothing && throw(ArgumentError("an attached HIPSDF needs scene_q"))
        lds = scene_q isa ROCMatrix ? stride(scene_q, 2) : 0  # (N, cols) per configuration, or one vector
        check(ccall((:kin_coll_batch_scene, libkinhip), Cint,
                    (Ptr{Cvoid}, Ptr{Cvoid}, Float64, Ptr{T}, Int64, Ptr{T}, Int64, Int64, Ptr{T}, Int64, Ptr{T}, Int64,
                     Ptr{T}, Ptr{Cvoid}),
                    p, sdf.handle, truncation_dist, pointer(Q), stride(Q, 2), pointer(scene_q), lds, N, pointer(vals),
                    N, grads === nothing ? C_NULL : pointer(grads), N, C_NULL, stream_ptr()))
        return vals, grads
    end
    check(ccall((:kin_coll_batch, libkinhip), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Float64, Ptr{T}, Int64, Int64, Ptr{T}, Int64, Ptr{T}, Int64, Ptr{T},
                 Ptr{Cvoid}),
                p, sdf.handle, truncation_dist, pointer(Q), stride(Q, 2), N, pointer(vals), N,
                grads === nothing ? C_NULL : pointer(grads), N, C_NULL, stream_ptr()))
    vals, grads
end

"""Cached kin_coll_ik_plan_create plan: the IK plan of `link` over `joints` with the checker's spheres."""
function collik_plan!(hm::HIPModel, ::Type{T}, sscc::Kinematics.SweptSphereCollisionChecker, link::Link,
                      joints::Vector{<:Joint}) where {T}
    ids = Int32[j.id for j in joints]
    sph = Int32[l.id for l in sscc.sphere_links]
    key = (:collik, T, ids, sph, link.id)
    cached_plan!(hm, key, ids) do
        h = Ref{Ptr{Cvoid}}(C_NULL)
        r = Float64.(sscc.sphere_radii)
        GC.@preserve ids sph r begin
            d = KinCollDesc(dtype_code(T), length(ids), pointer(ids), length(sph), isempty(sph) ? C_NULL : pointer(sph),
                            C_NULL, isempty(r) ? C_NULL : pointer(r))
            check(ccall((:kin_coll_ik_plan_create, libkinhip), Cint,
                        (Ptr{Cvoid}, Ref{KinCollDesc}, Int32, Ref{Ptr{Cvoid}}), hm.handle, d, Int32(link.id), h))
        end
        hm.specialize && ccall((:kin_plan_specialize, libkinhip), Cint, (Ptr{Cvoid}, UInt32), h[], UInt32(0))
        h[]
    end
end

"""Batched collision-aware IK, inverse_kinematics!(m, link, joints, target, sscc, sdf; use_bistage)
(src/inverse_kinematics.jl:1-21) for every row of `targets` (N, 12): stage 1 the collision-free DLS
(kin_ik_dls_batch_from, seeds Q0), stage 2 the IneqConst(sscc, joints, sdf, 1, margin) sphere rows, both on
one plan of kin_coll_ik_plan_create, stage 2's restart attempt 1 from Q0 (kin_ik_coll_batch_alt).  A static
`HIPSDF(UnionSDF)` runs kin_ik_coll_batch's kernel; an attached one
(`HIPSDF(fridge, [door_joint])`, the reference's `UnionSDF(fridge)` of test/test_inverse_kinematics.jl:55
and fridge_demo.jl) runs kin_ik_coll_batch_scene's kernel with `scene_q`: the scene columns per target, an
(N, n_scene_cols) ROCMatrix (e.g. a door angle per target), or one ROCVector for the whole batch.
Returns (Q, iters, err (N, 3))."""
function Kinematics.inverse_kinematics!(hm::HIPModel, link::Link, joints::Vector{<:Joint}, targets::ROCMatrix{T},
                                        Q0::ROCMatrix{T}, sscc::Kinematics.SweptSphereCollisionChecker, sdf::HIPSDF;
                                        use_bistage=true, margin=0.02, band=0.0, weight=1.0, feas=1e-6,
                                        max_iters=64, lambda=1e-2, tol_pos=1e-3, tol_rot=1e-3, max_step=0.5,
                                        rpy_objective=true, restarts=3, seed=0, index_base=0,
                                        scene_q=nothing) where {T}
    sdf.attached && scene_q === nothing && throw(ArgumentError("an attached HIPSDF needs scene_q"))
    N = size(Q0, 1)
    p = collik_plan!(hm, T, sscc, link, joints)
    Q1 = similar(Q0)
    Q = similar(Q0)
    iters = ROCVector{Int32}(undef, N)
    err = ROCMatrix{T}(undef, N, 3)
    prm = KinIkParams(max_iters, lambda, tol_pos, tol_rot, max_step, rpy_objective ? 2 : 1, restarts, seed, 0,
                      index_base, 0.0)
    if use_bistage
        check(ccall((:kin_ik_dls_batch_from, libkinhip), Cint,
                    (Ptr{Cvoid}, Ref{KinIkParams}, Ptr{T}, Int64, Ptr{T}, Ptr{T}, Int64, Int64, Ptr{Int32}, Ptr{T},
                     Int64, Ptr{Cvoid}),
                    p, prm, pointer(targets), stride(targets, 2), pointer(Q0), pointer(Q1), stride(Q1, 2), N,
                    pointer(iters), pointer(err), N, stream_ptr()))
    else
        copyto!(Q1, Q0)
    end
    cprm = KinIkCollParams(margin, band, weight, feas)
    # stage 2 from stage 1's answers; its restart attempt 1 from Q0, the pose stage 1 started from
    # (kin_ik_coll_batch_alt; static or attached union alike)
    sq = sdf.attached ? pointer(scene_q) : Ptr{T}(C_NULL)
    lds = scene_q isa ROCMatrix ? stride(scene_q, 2) : 0  # (N, cols) per target, or one vector
    check(ccall((:kin_ik_coll_batch_alt, libkinhip), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ref{KinIkParams}, Ref{KinIkCollParams}, Ptr{T}, Int64, Ptr{T}, Int64,
                 Ptr{T}, Ptr{T}, Ptr{T}, Int64, Int64, Ptr{Int32}, Ptr{T}, Int64, Ptr{Cvoid}),
                p, sdf.handle, prm, cprm, pointer(targets), stride(targets, 2), sq, lds, pointer(Q1),
                use_bistage ? pointer(Q0) : Ptr{T}(C_NULL), pointer(Q), stride(Q, 2), N, pointer(iters),
                pointer(err), N, stream_ptr()))
    Q, iters, err
end

# --- the reference's own single-target calls (src/inverse_kinematics.jl:1-30, src/collision.jl:51-103) ---
# Same signatures and return values as Kinematics.jl, so call sites and tests stay as they are (with `hm`,
# the HIPModel of the Mechanism, in place of `m`): (q, status) with the reference's NLopt status symbols, the
# mechanism's angles left at the answer.  fp64 throughout (the reference's precision).

"""The 3x4 column-major 12-vector of a Transform (the C-ABI's target layout), as a (1, 12) device batch."""
target_batch(T::Transform) = ROCMatrix{Float64}(reshape(Float64[T.mat[r, c] for c in 1:4 for r in 1:3], 1, 12))

"""The mechanism's current angles of `joints` (+ base) as a (1, dof) device batch (get_joint_angles,
src/mechanism.jl:203-221)."""
angles_batch(m::Mechanism, joints::Vector{<:Joint}) = ROCMatrix{Float64}(reshape(get_joint_angles(m, joints), 1, :))

"""inverse_kinematics!(m, link, joints, target; ftol, with_rot) (src/inverse_kinematics.jl:23-30) on the GPU ->
(q, status).  The reference's objective (f_objective, :38-50: |[p* - p; rpy* - rpy]|^2 with the rpy_jac
Jacobian; position only when !with_rot) minimised by damped least squares from the mechanism's current
angles, stopped by the reference's ftol_abs rule -- NLopt stops when one step changes the objective by less
than ftol (:62) -- checked on every iterate: one launch of max_iters steps records every iterate's residual
(kin_ik_dls_batch_trace), the stopping iterate k is one launch of k steps from the same angles
(kin_ik_dls_batch_from).  :FTOL_REACHED when the rule stopped it, :MAXEVAL_REACHED after max_iters steps.
Sets the mechanism's angles to the answer.  Python mirror: kinhip.inverse_kinematics_ (mechanism.py)."""
function Kinematics.inverse_kinematics!(hm::HIPModel, link::Link, joints::Vector{<:Joint}, target_pose::Transform;
                                        ftol=1e-5, with_rot=true, max_iters=200, lambda=1e-2, max_step=0.5)
    m = hm.m
    ids = Int32[j.id for j in joints]
    p = plan!(hm, Float64, ids, Int32[link.id], Int32(link.id), ids, KIN_WITH_ROT)
    tgt = target_batch(target_pose)
    q0 = angles_batch(m, joints)
    q = similar(q0)
    iters = ROCVector{Int32}(undef, 1)
    M = Int(max_iters)
    mode = with_rot ? Int32(2) : Int32(0)
    trace = fill!(ROCMatrix{Float64}(undef, 1, 2 * (M + 1)), NaN)  # [|dp|, |d rpy|] of iterates 0..M
    prm = KinIkParams(M, lambda, 0.0, 0.0, max_step, mode, 0, 0, 1, 0, 0.0)
    check(ccall((:kin_ik_dls_batch_trace, libkinhip), Cint,
                (Ptr{Cvoid}, Ref{KinIkParams}, Ptr{Float64}, Int64, Ptr{Float64}, Ptr{Float64}, Int64, Int64,
                 Ptr{Int32}, Ptr{Float64}, Int64, Ptr{Cvoid}),
                p, prm, pointer(tgt), 1, pointer(q0), pointer(q), 1, 1, pointer(iters), pointer(trace), 1, stream_ptr()))
    tr = Array(trace)
    f = tr[1, 1:2:end] .^ 2 .+ tr[1, 2:2:end] .^ 2  # the objective sum(pose_diff.^2) of iterates 0..M
    status, k = :MAXEVAL_REACHED, M
    for kk in 1:M
        if abs(f[kk] - f[kk+1]) < ftol
            status, k = :FTOL_REACHED, kk
            break
        end
    end
    prm_k = KinIkParams(k, lambda, 0.0, 0.0, max_step, mode, 0, 0, 1, 0, 0.0)
    check(ccall((:kin_ik_dls_batch_from, libkinhip), Cint,
                (Ptr{Cvoid}, Ref{KinIkParams}, Ptr{Float64}, Int64, Ptr{Float64}, Ptr{Float64}, Int64, Int64,
                 Ptr{Int32}, Ptr{Float64}, Int64, Ptr{Cvoid}),
                p, prm_k, pointer(tgt), 1, pointer(q0), pointer(q), 1, 1, pointer(iters), C_NULL, 1, stream_ptr()))
    qv = vec(Array(q))
    set_joint_angles(m, joints, qv)
    qv, status
end

"""inverse_kinematics!(m, link, joints, target, sscc, sdf; use_bistage, ftol, with_rot)
(src/inverse_kinematics.jl:1-21) on the GPU -> (q, status).  Stage 1 (use_bistage) is the collision-free
call above (it moves the mechanism to its answer, as the reference's NLopt stage 1 does through
f_objective's set_joint_angles); stage 2 solves the same objective subject to IneqConst(sscc, joints, sdf, 1,
margin)'s sphere distances (:16-17) and the joint limits from the mechanism's current angles: the batched
kin_ik_coll_batch kernel on a batch of one, 3 restarts (with use_bistage the first from the angles stage 1
started from, kin_ik_coll_batch_alt; the others seeded draws), converged when |dp|, |d rpy| < 1e-6 with every
sphere at >= margin - 1e-6 (:FTOL_REACHED); otherwise the attempt of lowest merit, :MAXEVAL_REACHED.  `sdf`
is the reference's UnionSDF / BoxSDF (a snapshot at the scene's current angles, HIPSDF(sdf)) or a HIPSDF; an
attached HIPSDF(scene, joints) takes `scene_q`, its scene column values (a ROCVector).  A checker without
spheres (the reference's own PR2 test adds none: test/test_inverse_kinematics.jl:63 is an un-iterated
generator) leaves stage 2 an unconstrained solve.  Python mirror: kinhip.planning.collision_aware_ik."""
function Kinematics.inverse_kinematics!(hm::HIPModel, link::Link, joints::Vector{<:Joint}, target_pose::Transform,
                                        sscc::Kinematics.SweptSphereCollisionChecker,
                                        sdf::Union{HIPSDF,Kinematics.AbstractSDF}; use_bistage=true, ftol=1e-5,
                                        with_rot=true, max_iters=200, lambda=1e-2, max_step=0.5, margin=0.02,
                                        scene_q=nothing)
    m = hm.m
    m === sscc.mech || throw(ArgumentError("the HIPModel must be the checker's mechanism (sscc.mech)"))
    q_start = angles_batch(m, joints)  # stage 2's restart attempt 1 starts here (kin_ik_coll_batch_alt)
    if use_bistage  # stage 1 seeds stage 2 (src/inverse_kinematics.jl:8-13)
        Kinematics.inverse_kinematics!(hm, link, joints, target_pose; ftol=ftol, with_rot=with_rot,
                                       max_iters=max_iters, lambda=lambda, max_step=max_step)
    end
    hs = sdf isa HIPSDF ? sdf : HIPSDF(sdf)
    hs.attached && scene_q === nothing && throw(ArgumentError("an attached HIPSDF needs scene_q"))
    p = collik_plan!(hm, Float64, sscc, link, joints)
    tgt = target_batch(target_pose)
    q0 = angles_batch(m, joints)
    q = similar(q0)
    iters = ROCVector{Int32}(undef, 1)
    err = ROCMatrix{Float64}(undef, 1, 3)
    prm = KinIkParams(max_iters, lambda, 1e-6, 1e-6, max_step, with_rot ? Int32(2) : Int32(0), 3, 0, 0, 0, 0.0)
    cprm = KinIkCollParams(margin, 0.0, 1.0, 1e-6)
    check(ccall((:kin_ik_coll_batch_alt, libkinhip), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ref{KinIkParams}, Ref{KinIkCollParams}, Ptr{Float64}, Int64, Ptr{Float64},
                 Int64, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Int64, Ptr{Int32}, Ptr{Float64}, Int64,
                 Ptr{Cvoid}),
                p, hs.handle, prm, cprm, pointer(tgt), 1, hs.attached ? pointer(scene_q) : Ptr{Float64}(C_NULL), 0,
                pointer(q0), use_bistage ? pointer(q_start) : Ptr{Float64}(C_NULL), pointer(q), 1, 1,
                pointer(iters), pointer(err), 1, stream_ptr()))
    qv = vec(Array(q))
    set_joint_angles(m, joints, qv)
    qv, (Array(iters)[1] <= max_iters ? :FTOL_REACHED : :MAXEVAL_REACHED)
end

"""compute_coll_dists_and_grads(sscc, joints, sdf; truncation_dist) (src/collision.jl:96-103) at the mechanism's
current angles -> (vals (n_spheres), grads (n_dof, n_spheres)), the GPU batch of one.  `sdf`: the reference's
UnionSDF / BoxSDF or a HIPSDF (attached: `scene_q`)."""
function Kinematics.compute_coll_dists_and_grads(hm::HIPModel, sscc::Kinematics.SweptSphereCollisionChecker,
                                                 joints::Vector{<:Joint}, sdf::Union{HIPSDF,Kinematics.AbstractSDF};
                                                 truncation_dist=Inf, scene_q=nothing, with_grad=true)
    n = length(sscc.sphere_links)
    n_dof = length(joints) + (hm.m.with_base ? 3 : 0)
    n == 0 && return Float64[], zeros(n_dof, 0)
    hs = sdf isa HIPSDF ? sdf : HIPSDF(sdf)
    Q = angles_batch(hm.m, joints)
    vals = ROCMatrix{Float64}(undef, 1, n)
    grads = with_grad ? ROCArray{Float64}(undef, 1, n_dof, n) : nothing
    compute_coll_dists_and_grads!(hm, sscc, joints, hs, Q, vals, grads; truncation_dist=truncation_dist, scene_q=scene_q)
    vec(Array(vals)), (with_grad ? Array(grads)[1, :, :] : nothing)
end

"""compute_coll_dists(sscc, joints, sdf) (src/collision.jl:60-65) at the mechanism's current angles."""
Kinematics.compute_coll_dists(hm::HIPModel, sscc::Kinematics.SweptSphereCollisionChecker, joints::Vector{<:Joint},
                              sdf::Union{HIPSDF,Kinematics.AbstractSDF}; scene_q=nothing) =
    Kinematics.compute_coll_dists_and_grads(hm, sscc, joints, sdf; scene_q=scene_q, with_grad=false)[1]

"""IneqConst over every waypoint column of Xi (N = waypoints of one or many trajectories, rows = dof):
vals (N, n_coll) = min(dist, margin + 0.05) - margin, jac (N, n_dof, n_coll)."""
function ineq_const!(hm::HIPModel, sscc::Kinematics.SweptSphereCollisionChecker, joints::Vector{<:Joint},
                     sdf::HIPSDF, margin::Real, Xi::ROCMatrix{T}, vals::ROCMatrix{T}, jac::ROCArray{T,3}) where {T}
    N = size(Xi, 1)
    p = coll_plan!(hm, T, sscc, joints)
    check(ccall((:kin_ineq_const_batch, libkinhip), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Float64, Ptr{T}, Int64, Int64, Ptr{T}, Int64, Ptr{T}, Int64, Ptr{Cvoid}),
                p, sdf.handle, Float64(margin), pointer(Xi), stride(Xi, 2), N, pointer(vals), N, pointer(jac), N,
                stream_ptr()))
    vals, jac
end

"""PoseConstraint of one link for N configurations: targets (N, 12), vals (N, 6 or 3), jac (N, dim, dof)."""
function pose_const!(hm::HIPModel, link::Link, joints::Vector{<:Joint}, with_rot::Bool, targets::ROCMatrix{T},
                     Q::ROCMatrix{T}, vals::ROCMatrix{T}, jac::ROCArray{T,3}) where {T}
    N = size(Q, 1)
    ids = Int32[j.id for j in joints]
    flags = with_rot ? (KIN_WITH_ROT | KIN_RPY_JAC) : UInt32(0)
    p = plan!(hm, T, ids, Int32[link.id], Int32(link.id), ids, flags | KIN_ZERO_FILL)
    poses = ROCArray{T}(undef, N, 12)
    check(ccall((:kin_pose_const_batch, libkinhip), Cint,
                (Ptr{Cvoid}, Ptr{T}, Int64, Ptr{T}, Int64, Int64, Ptr{T}, Int64, Ptr{T}, Int64, Ptr{T}, Int64,
                 Ptr{Cvoid}),
                p, pointer(targets), stride(targets, 2), pointer(Q), stride(Q, 2), N, pointer(poses), N,
                pointer(vals), N, pointer(jac), N, stream_ptr()))
    vals, jac
end

# --- the reference's plan_trajectory with the collision queries on the GPU (src/planning.jl:32-68, 332-401) ---

const HIP_MODELS = WeakKeyDict{Mechanism,HIPModel}()

"""The HIPModel of a Mechanism, made on first use and kept while the Mechanism lives: the reference's calls
that reach the robot only through `sscc.mech` (IneqConst, compute_coll_dists) use it."""
hip_model(m::Mechanism) = get!(() -> HIPModel(m), HIP_MODELS, m)

"""`GPUSDF(sdf)`: a reference SDF (UnionSDF / BoxSDF, e.g. UnionSDF(fridge)) with its device snapshot
HIPSDF(sdf).  It is an AbstractSDF, so the reference's own entry points take it unchanged --
`plan_trajectory(sscc, joints, GPUSDF(sdf), q_start, q_goal, n_wp; margin, partial_consts, ftol_abs,
solver)` -- and their collision queries run on the GPU:
  * compute_coll_dists / compute_coll_dists_and_grads(sscc, joints, sdf; truncation_dist) and their `!`
    forms (src/collision.jl:51-103) at the mechanism's current angles (kin_coll_batch, a batch of one);
  * IneqConst (src/planning.jl:55-68) called with the dense Vector / Matrix buffers NLopt's and SciPy's
    adapters pass (nloptize / scipynize, :225-247): all n_wp waypoints in one kin_ineq_const_batch launch.
    Other buffers (Ipopt's views) take the reference's per-waypoint loop, whose queries are the GPU ones
    above.  The mechanism is left at the last waypoint, as the reference's loop leaves it.
Point queries (`sdf(p)`, gradient!) forward to the wrapped SDF; the snapshot is the scene at its angles
when GPUSDF was made.  Distances use the analytic box gradient (the reference differentiates forward with
eps 1e-7)."""
struct GPUSDF <: Kinematics.AbstractSDF{Kinematics.IsStandAlone}
    sdf::Kinematics.AbstractSDF
    hip::HIPSDF
end
GPUSDF(sdf::Kinematics.AbstractSDF) = GPUSDF(sdf, HIPSDF(sdf))
HIPSDF(s::GPUSDF) = s.hip
(s::GPUSDF)(p; kw...) = s.sdf(p; kw...)
Kinematics.gradient!(s::GPUSDF, p, out_grad::AbstractVector) = Kinematics.gradient!(s.sdf, p, out_grad)

Kinematics.compute_coll_dists_and_grads(sscc::Kinematics.SweptSphereCollisionChecker, joints::Vector{<:Joint},
                                        sdf::GPUSDF; truncation_dist=Inf) =
    Kinematics.compute_coll_dists_and_grads(hip_model(sscc.mech), sscc, joints, sdf.hip;
                                            truncation_dist=truncation_dist)

Kinematics.compute_coll_dists(sscc::Kinematics.SweptSphereCollisionChecker, joints::Vector{<:Joint}, sdf::GPUSDF) =
    Kinematics.compute_coll_dists(hip_model(sscc.mech), sscc, joints, sdf.hip)

function Kinematics.compute_coll_dists_and_grads!(sscc::Kinematics.SweptSphereCollisionChecker,
                                                  joints::Vector{<:Joint}, sdf::GPUSDF,
                                                  out_vals::AbstractArray{Float64,1},
                                                  out_grads::AbstractArray{Float64,2}; truncation_dist=Inf)
    v, g = Kinematics.compute_coll_dists_and_grads(sscc, joints, sdf; truncation_dist=truncation_dist)
    out_vals .= v
    out_grads .= g
    nothing
end

function Kinematics.compute_coll_dists!(sscc::Kinematics.SweptSphereCollisionChecker, joints::Vector{<:Joint},
                                        sdf::GPUSDF, out_vals::AbstractArray{Float64,1})
    out_vals .= Kinematics.compute_coll_dists(sscc, joints, sdf)
    nothing
end

"""IneqConst over all waypoints at once when its sdf is a GPUSDF (see GPUSDF); any other IneqConst runs the
reference's method unchanged (`invoke`)."""
function (this::Kinematics.IneqConst)(xi::Vector{Float64}, val_vec::Vector{Float64}, jac_mat::Matrix{Float64})
    this.sdf isa GPUSDF ||
        return invoke(this, Tuple{AbstractVector,AbstractVector,AbstractMatrix}, xi, val_vec, jac_mat)
    n_dof, n_wp, n_coll = this.n_dof, this.n_wp, this.n_coll
    n_coll == 0 && return nothing
    X = reshape(xi, n_dof, n_wp)
    Xi = ROCMatrix{Float64}(permutedims(X))  # (n_wp, n_dof): waypoint index fastest, the C-ABI's batch
    vals = ROCMatrix{Float64}(undef, n_wp, n_coll)
    jac = ROCArray{Float64}(undef, n_wp, n_dof, n_coll)
    ineq_const!(hip_model(this.sscc.mech), this.sscc, this.joints, this.sdf.hip, this.margin, Xi, vals, jac)
    v = Array(vals)
    J = Array(jac)
    for i in 1:n_wp  # the reference's block-diagonal layout (:63-66)
        val_vec[1+n_coll*(i-1):n_coll*i] = v[i, :]
        jac_mat[1+n_dof*(i-1):n_dof*i, 1+n_coll*(i-1):n_coll*i] = J[i, :, :]
    end
    set_joint_angles(this.sscc.mech, this.joints, X[:, n_wp])
    nothing
end

export HIPModel, sync!, batch_array, get_jacobian_tiled!, point_inverse_kinematics_nakamura!, HIPSDF, compute_coll_dists_and_grads!, ineq_const!, pose_const!, GPUSDF, hip_model

end # module
