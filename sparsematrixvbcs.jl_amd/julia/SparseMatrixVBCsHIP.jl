# SparseMatrixVBCsHIP.jl -- the `ccall` layer a SparseMatrixVBCs.jl maintainer would add so that
# `mul!` on the reference's own types runs on an MI355X through libvbc (include/vbc.h).
#
# NOT EXECUTED IN THIS REPOSITORY: there is no Julia toolchain in the build image, so this file is
# syntax-reviewed only.  Every ccall signature mirrors include/vbc.h one to one; the Python mirror
# (sparsematrixvbcs.jl_amd/*.py), which IS tested on the GPU, binds the same symbols the same way.
#
# Usage (after `using SparseMatrixVBCs`; ROCArray methods load with `using AMDGPU`, see
# ext/SparseMatrixVBCsHIPAMDGPUExt.jl):
#     B  = SparseMatrix1DVBC{8}(A)                 # reference constructor, unchanged
#     Bd = HIPSparseMatrix1DVBC(B)                 # uploads once per compute eltype (vbc1d_create_ex)
#     mul!(y, Bd', x)                              # host StridedVectors: staged through HBM
#     mul!(y_dev, Bd', x_dev)                      # ROCVectors: enqueued on the task-local stream
#     Bs = HIPShardedSparseMatrix(B; devices=0:7)        # one session, 8 GPUs, RCCL over xGMI (1D or 2D B)
#     mul!(y, Bs', x)
module SparseMatrixVBCsHIP

using LinearAlgebra
using SparseArrays
using SparseMatrixVBCs: SparseMatrix1DVBC, SparseMatrixVBC

const libvbc = get(ENV, "VBC_LIBRARY", joinpath(@__DIR__, "..", "libvbc.so"))

const VBC_OK, VBC_DIM_MISMATCH, VBC_INVALID_ARG, VBC_HIP_ERROR, VBC_RCCL_ERROR,
      VBC_UNSUPPORTED_DTYPE, VBC_ASSERTION = 0, 1, 2, 3, 4, 5, 6
const VBC_F64, VBC_F32, VBC_I64, VBC_I32, VBC_BOOL = Cint(0), Cint(1), Cint(2), Cint(3), Cint(4)
const VBC_MEM_DEVICE, VBC_MEM_HOST = Cint(0), Cint(1)
const VBC_CREATE_TRANSPOSED, VBC_CREATE_FORWARD = Cuint(1), Cuint(2)
const VBC_CREATE_MULTI, VBC_CREATE_MULTI_FORWARD = Cuint(4), Cuint(16)  # matrix-core panels of B and of Bᵀ
const VBC_MUL_REFERENCE_QUIRKS = Cuint(1)
const VBC_SPLIT_STRIPES, VBC_SPLIT_ROWS, VBC_SPLIT_AUTO = Cint(0), Cint(1), Cint(2)

# the eltypes the reference's tests use (runtests.jl:15-16) and their vbc_dtype codes
vbc_dtype(::Type{Float64}) = VBC_F64
vbc_dtype(::Type{Float32}) = VBC_F32
vbc_dtype(::Type{Int64}) = VBC_I64
vbc_dtype(::Type{Int32}) = VBC_I32
vbc_dtype(::Type{Bool}) = VBC_BOOL
vbc_dtype(::Type{T}) where {T} = throw(MethodError(vbc_dtype, (T,)))

# The product computes in eltype(y) (multiply_1DVBC.jl:27,34,102): floats in themselves, integer y in
# exact wrapping Int64 (Int32 y is stored back truncated, Julia's wraparound).
compute_dtype(::Type{Float64}) = VBC_F64
compute_dtype(::Type{Float32}) = VBC_F32
compute_dtype(::Type{<:Union{Int64, Int32}}) = VBC_I64
compute_dtype(::Type{T}) where {T} = throw(MethodError(compute_dtype, (T,)))

# include/vbc.h vbc_types
struct VbcTypes
    val_dtype::Cint
    index_bits::Cint
    compute_dtype::Cint
    reserved::Cint
end
vbc_types(::Type{Tv}, ::Type{Ti}, cdt::Cint) where {Tv, Ti <: Union{Int64, Int32}} =
    VbcTypes(vbc_dtype(Tv), 8 * sizeof(Ti), cdt, 0)

# include/vbc.h VBC_VERSION: the structs below (VbcTypes; vbc_info, VBC_INFO_SIZE = 152 bytes) are those
# of ABI major version 3
function __init__()
    v = ccall((:vbc_version, libvbc), Cint, ())
    v ÷ 10000 == 3 || error("libvbc ABI version $v does not match SparseMatrixVBCsHIP (3.x); rebuild libvbc")
end

function last_error()
    buf = Vector{UInt8}(undef, 1024)
    ccall((:vbc_last_error, libvbc), Cint, (Ptr{UInt8}, Csize_t), buf, length(buf))
    return unsafe_string(pointer(buf))
end

# status -> the reference's exceptions (multiply_1DVBC.jl:44-45, SparseMatrixVBCs.jl:45-50,
# constructors_1DVBC.jl:46)
function check(st::Cint)
    st == VBC_OK && return nothing
    st == VBC_DIM_MISMATCH && throw(DimensionMismatch(last_error()))
    st == VBC_INVALID_ARG && throw(ArgumentError(last_error()))
    st == VBC_ASSERTION && throw(AssertionError(last_error()))
    st == VBC_UNSUPPORTED_DTYPE && throw(MethodError(mul!, (last_error(),)))
    throw(ErrorException(last_error()))
end

"""
    HIPSparseMatrix1DVBC(B::SparseMatrix1DVBC; device=0, forward=true, transposed=true)

Device-resident copies of `B`, one libvbc handle per compute eltype met (created on first use by
`mul!`), freed by a finalizer (`vbc_destroy`).  Immutable.
"""
mutable struct HIPSparseMatrix1DVBC{W, Tv, Ti}
    host::SparseMatrix1DVBC{W, Tv, Ti}
    device::Int
    flags::Cuint
    handles::Dict{Cint, Ptr{Cvoid}}
end

function HIPSparseMatrix1DVBC(B::SparseMatrix1DVBC{W, Tv, Ti}; device::Integer=0, forward::Bool=true,
                              transposed::Bool=true, multi::Bool=false) where {W, Tv, Ti}
    flags = (transposed ? VBC_CREATE_TRANSPOSED : Cuint(0)) | (forward ? VBC_CREATE_FORWARD : Cuint(0)) |
            (multi ? (VBC_CREATE_MULTI | VBC_CREATE_MULTI_FORWARD) : Cuint(0))
    M = HIPSparseMatrix1DVBC{W, Tv, Ti}(B, device, flags, Dict{Cint, Ptr{Cvoid}}())
    finalizer(destroy_handles, M)
    return M
end

function _create(B::SparseMatrix1DVBC{W, Tv, Ti}, device, flags, cdt::Cint) where {W, Tv, Ti}
    h = Ref{Ptr{Cvoid}}(C_NULL)
    t = Ref(vbc_types(Tv, Ti, cdt))
    GC.@preserve B t check(ccall((:vbc1d_create_ex, libvbc), Cint,
        (Ptr{Ptr{Cvoid}}, Int64, Int64, Int64, Int64, Ptr{Ti}, Ptr{Ti}, Ptr{Ti}, Ptr{Ti}, Ptr{Cvoid}, Int64,
         Ptr{VbcTypes}, Cint, Cuint),
        h, B.m, B.n, W, length(B.Φ), B.Φ.spl, B.pos, B.idx, B.ofs, B.val, length(B.val), t, device, flags))
    return h[]
end

mutable struct HIPSparseMatrixVBC{U, W, Tv, Ti}
    host::SparseMatrixVBC{U, W, Tv, Ti}
    device::Int
    flags::Cuint
    handles::Dict{Cint, Ptr{Cvoid}}
end

function HIPSparseMatrixVBC(B::SparseMatrixVBC{U, W, Tv, Ti}; device::Integer=0, forward::Bool=true,
                            transposed::Bool=true, multi::Bool=false) where {U, W, Tv, Ti}
    flags = (transposed ? VBC_CREATE_TRANSPOSED : Cuint(0)) | (forward ? VBC_CREATE_FORWARD : Cuint(0)) |
            (multi ? (VBC_CREATE_MULTI | VBC_CREATE_MULTI_FORWARD) : Cuint(0))
    M = HIPSparseMatrixVBC{U, W, Tv, Ti}(B, device, flags, Dict{Cint, Ptr{Cvoid}}())
    finalizer(destroy_handles, M)
    return M
end

function _create(B::SparseMatrixVBC{U, W, Tv, Ti}, device, flags, cdt::Cint) where {U, W, Tv, Ti}
    h = Ref{Ptr{Cvoid}}(C_NULL)
    t = Ref(vbc_types(Tv, Ti, cdt))
    GC.@preserve B t check(ccall((:vbc2d_create_ex, libvbc), Cint,
        (Ptr{Ptr{Cvoid}}, Int64, Int64, Int64, Int64, Int64, Ptr{Ti}, Int64, Ptr{Ti}, Ptr{Ti}, Ptr{Ti},
         Ptr{Ti}, Ptr{Cvoid}, Int64, Ptr{VbcTypes}, Cint, Cuint),
        h, B.m, B.n, U, W, length(B.Π), B.Π.spl, length(B.Φ), B.Φ.spl, B.pos, B.idx, B.ofs, B.val,
        length(B.val), t, device, flags))
    return h[]
end

# TrSpMV!(y, A::SparseMatrixCSC, x) (TrSpMV.jl:1-20) through a CSC handle (unit-width stripes).
mutable struct HIPSparseMatrixCSC{Tv, Ti}
    host::SparseMatrixCSC{Tv, Ti}
    device::Int
    flags::Cuint
    handles::Dict{Cint, Ptr{Cvoid}}
end

function HIPSparseMatrixCSC(A::SparseMatrixCSC{Tv, Ti}; device::Integer=0) where {Tv, Ti}
    M = HIPSparseMatrixCSC{Tv, Ti}(A, device, VBC_CREATE_TRANSPOSED, Dict{Cint, Ptr{Cvoid}}())
    finalizer(destroy_handles, M)
    return M
end

function _create(A::SparseMatrixCSC{Tv, Ti}, device, flags, cdt::Cint) where {Tv, Ti}
    h = Ref{Ptr{Cvoid}}(C_NULL)
    t = Ref(vbc_types(Tv, Ti, cdt))
    GC.@preserve A t check(ccall((:vbc_csc_create_ex, libvbc), Cint,
        (Ptr{Ptr{Cvoid}}, Int64, Int64, Ptr{Ti}, Ptr{Ti}, Ptr{Cvoid}, Ptr{VbcTypes}, Cint, Cuint),
        h, size(A, 1), size(A, 2), A.colptr, A.rowval, A.nzval, t, device, flags))
    return h[]
end

const HIPMatrix = Union{HIPSparseMatrix1DVBC, HIPSparseMatrixVBC, HIPSparseMatrixCSC}
Base.size(A::HIPMatrix) = size(A.host)
Base.size(A::HIPMatrix, d::Integer) = size(A.host, d)
Base.eltype(A::HIPMatrix) = eltype(A.host)

# the handle computing in eltype(y); a Float matrix cannot run in an integer eltype (InexactError)
function handle_for(A::HIPMatrix, ::Type{Ty}) where {Ty}
    cdt = compute_dtype(Ty)
    cdt == VBC_I64 && eltype(A) <: AbstractFloat && throw(InexactError(:convert, Ty, zero(eltype(A))))
    get!(() -> _create(A.host, A.device, A.flags, cdt), A.handles, cdt)
end

function destroy_handles(A::HIPMatrix)
    for h in values(A.handles)
        ccall((:vbc_destroy, libvbc), Cint, (Ptr{Cvoid},), h)
    end
    empty!(A.handles)
end

# Host vectors (any StridedVector, any supported eltype: x converted to eltype(y) like
# multiply_1DVBC.jl:102): vbc_mul_ex stages them through the handle's cached device buffers and
# returns when y is final.  The eltypes travel with the pointers, so a mismatch cannot overrun.
function _mul!(y::StridedVector{Ty}, A::HIPMatrix, trans::Bool, x::StridedVector{Tx}, α::Number, β::Number;
               quirks::Bool=false) where {Ty, Tx}
    h = handle_for(A, Ty)
    GC.@preserve x y check(ccall((:vbc_mul_ex, libvbc), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Tx}, Cint, Int64, Int64, Ptr{Ty}, Cint, Int64, Int64, Cdouble, Cdouble, Cint,
         Ptr{Cvoid}, Cuint),
        h, trans, pointer(x), vbc_dtype(Tx), stride(x, 1), length(x), pointer(y), vbc_dtype(Ty), stride(y, 1),
        length(y), Float64(α), Float64(β), VBC_MEM_HOST, C_NULL, quirks ? VBC_MUL_REFERENCE_QUIRKS : Cuint(0)))
    return y
end

const AdjOrTransHIP = Union{Adjoint{<:Any, <:HIPMatrix}, Transpose{<:Any, <:HIPMatrix}}

# The reference's operator surface: mul!(y, B, x, α, β) and mul!(y, B', x, α, β)
# (multiply_1DVBC.jl:9, :85; multiply_VBC.jl:3, :89) plus the 3-argument forms and Base.:*.
LinearAlgebra.mul!(y::StridedVector, A::HIPMatrix, x::StridedVector, α::Number, β::Number) =
    _mul!(y, A, false, x, α, β)
LinearAlgebra.mul!(y::StridedVector, adjA::AdjOrTransHIP, x::StridedVector, α::Number, β::Number) =
    _mul!(y, parent(adjA), true, x, α, β)
LinearAlgebra.mul!(y::StridedVector, A::HIPMatrix, x::StridedVector) = mul!(y, A, x, true, false)
LinearAlgebra.mul!(y::StridedVector, adjA::AdjOrTransHIP, x::StridedVector) = mul!(y, adjA, x, true, false)
# Base.:* (multiply_1DVBC.jl:182-185): y of promote_op(matprod, eltype(A), eltype(x))
Base.:*(A::HIPMatrix, x::StridedVector{T}) where {T} =
    mul!(similar(x, Base.promote_op(LinearAlgebra.matprod, eltype(A), T), size(A, 1)), A, x, true, false)
Base.:*(adjA::AdjOrTransHIP, x::StridedVector{T}) where {T} =
    mul!(similar(x, Base.promote_op(LinearAlgebra.matprod, eltype(parent(adjA)), T), size(adjA, 1)), adjA, x,
         true, false)

TrSpMV!(y::StridedVector, A::HIPSparseMatrixCSC, x::StridedVector) = _mul!(y, A, true, x, true, false)

"""
    HIPShardedSparseMatrix(B; devices=0:7, split=:stripes, serial=false)

`B` (a SparseMatrix1DVBC or a SparseMatrixVBC) split over several GPUs of the node by byte-balanced
stripe (`split=:stripes`, the block rows of A when B stores Aᵀ) or row (`split=:rows`; Π's block rows
for a SparseMatrixVBC) ranges, one handle per GPU, RCCL over xGMI for the exchange
(vbc1d_create_sharded / vbc2d_create_sharded).  This replaces the reference's threaded stripe loops
(multiply_1DVBC.jl:169-177, multiply_VBC.jl:182-189).  Computes in Tv (integers and Bool in exact
Int64); host StridedVectors of any supported eltype (x converted like multiply_1DVBC.jl:102) or, with
AMDGPU, ROCVectors on `devices[1]`.  `serial=true` keeps the reference's serial per-stripe summation
order in every shard (VBC_CREATE_SERIAL).
"""
mutable struct HIPShardedSparseMatrix{M}
    host::M
    handle::Ptr{Cvoid}
    compute::Cint
end
const HIPShardedSparseMatrix1DVBC = HIPShardedSparseMatrix  # round-2 name

const VBC_CREATE_SERIAL = Cuint(8)

_split_code(split) = split === :stripes ? VBC_SPLIT_STRIPES : split === :rows ? VBC_SPLIT_ROWS : VBC_SPLIT_AUTO

function _sharded_flags(split, forward, transposed, serial)
    split in (:stripes, :rows, :auto) || throw(ArgumentError("split must be :stripes, :rows or :auto"))
    return (transposed ? VBC_CREATE_TRANSPOSED : Cuint(0)) | (forward ? VBC_CREATE_FORWARD : Cuint(0)) |
           (serial ? VBC_CREATE_SERIAL : Cuint(0))
end
_default_compute(::Type{Tv}) where {Tv} = Tv <: AbstractFloat ? compute_dtype(Tv) : VBC_I64

function HIPShardedSparseMatrix(B::SparseMatrix1DVBC{W, Tv, Ti}; devices=0:7, split::Symbol=:stripes,
                                forward::Bool=true, transposed::Bool=true, serial::Bool=false) where {W, Tv, Ti}
    flags = _sharded_flags(split, forward, transposed, serial)
    devs = Cint.(collect(devices))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    cdt = _default_compute(Tv)
    t = Ref(vbc_types(Tv, Ti, cdt))
    GC.@preserve B t devs check(ccall((:vbc1d_create_sharded, libvbc), Cint,
        (Ptr{Ptr{Cvoid}}, Int64, Int64, Int64, Int64, Ptr{Ti}, Ptr{Ti}, Ptr{Ti}, Ptr{Ti}, Ptr{Cvoid}, Int64,
         Ptr{VbcTypes}, Cint, Ptr{Cint}, Cint, Cuint),
        h, B.m, B.n, W, length(B.Φ), B.Φ.spl, B.pos, B.idx, B.ofs, B.val, length(B.val), t, length(devs), devs,
        _split_code(split), flags))
    M = HIPShardedSparseMatrix(B, h[], cdt)
    finalizer(M -> ccall((:vbc_sharded_destroy, libvbc), Cint, (Ptr{Cvoid},), M.handle), M)
    return M
end

function HIPShardedSparseMatrix(B::SparseMatrixVBC{U, W, Tv, Ti}; devices=0:7, split::Symbol=:stripes,
                                forward::Bool=true, transposed::Bool=true, serial::Bool=false) where {U, W, Tv, Ti}
    flags = _sharded_flags(split, forward, transposed, serial)
    devs = Cint.(collect(devices))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    cdt = _default_compute(Tv)
    t = Ref(vbc_types(Tv, Ti, cdt))
    GC.@preserve B t devs check(ccall((:vbc2d_create_sharded, libvbc), Cint,
        (Ptr{Ptr{Cvoid}}, Int64, Int64, Int64, Int64, Int64, Ptr{Ti}, Int64, Ptr{Ti}, Ptr{Ti}, Ptr{Ti}, Ptr{Ti},
         Ptr{Cvoid}, Int64, Ptr{VbcTypes}, Cint, Ptr{Cint}, Cint, Cuint),
        h, B.m, B.n, U, W, length(B.Π), B.Π.spl, length(B.Φ), B.Φ.spl, B.pos, B.idx, B.ofs, B.val, length(B.val), t,
        length(devs), devs, _split_code(split), flags))
    M = HIPShardedSparseMatrix(B, h[], cdt)
    finalizer(M -> ccall((:vbc_sharded_destroy, libvbc), Cint, (Ptr{Cvoid},), M.handle), M)
    return M
end

Base.size(A::HIPShardedSparseMatrix) = size(A.host)

"The split a sharded matrix uses (:stripes or :rows; what split = :auto chose by the cost model, DESIGN.md §7)."
function split_kind(A::HIPShardedSparseMatrix)
    sp = Ref{Cint}(0)
    check(ccall((:vbc_sharded_split, libvbc), Cint, (Ptr{Cvoid}, Ptr{Cint}), A.handle, sp))
    return sp[] == VBC_SPLIT_STRIPES ? :stripes : :rows
end
"Shard g's x span (0-based lo:hi-1 as a Julia range lo+1:hi): the part of x its disjoint-output product reads."
function x_span(A::HIPShardedSparseMatrix, g::Integer)
    lo, hi = Ref{Int64}(0), Ref{Int64}(0)
    check(ccall((:vbc_sharded_xspan, libvbc), Cint, (Ptr{Cvoid}, Cint, Ptr{Int64}, Ptr{Int64}), A.handle, g, lo, hi))
    return (lo[] + 1):hi[]
end
Base.size(A::HIPShardedSparseMatrix, d::Integer) = size(A.host, d)
Base.eltype(A::HIPShardedSparseMatrix) = eltype(A.host)

# Host StridedVectors of any supported eltype: vbc_sharded_mul_ex carries each pointer's eltype and
# stride (x converted to the compute eltype like multiply_1DVBC.jl:102; a y of another eltype is
# refused with VBC_UNSUPPORTED_DTYPE), so a mismatch can never over-read or overwrite host memory.
function _mul!(y::StridedVector{Ty}, A::HIPShardedSparseMatrix, trans::Bool, x::StridedVector{Tx}, α::Number,
               β::Number; quirks::Bool=false) where {Ty, Tx}
    GC.@preserve x y check(ccall((:vbc_sharded_mul_ex, libvbc), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Tx}, Cint, Int64, Int64, Ptr{Ty}, Cint, Int64, Int64, Cdouble, Cdouble, Cint,
         Ptr{Cvoid}, Cuint),
        A.handle, trans, pointer(x), vbc_dtype(Tx), stride(x, 1), length(x), pointer(y), vbc_dtype(Ty), stride(y, 1),
        length(y), Float64(α), Float64(β), VBC_MEM_HOST, C_NULL, quirks ? VBC_MUL_REFERENCE_QUIRKS : Cuint(0)))
    return y
end

const AdjOrTransSharded = Union{Adjoint{<:Any, <:HIPShardedSparseMatrix}, Transpose{<:Any, <:HIPShardedSparseMatrix}}
LinearAlgebra.mul!(y::StridedVector, A::HIPShardedSparseMatrix, x::StridedVector, α::Number, β::Number) =
    _mul!(y, A, false, x, α, β)
LinearAlgebra.mul!(y::StridedVector, adjA::AdjOrTransSharded, x::StridedVector, α::Number, β::Number) =
    _mul!(y, parent(adjA), true, x, α, β)
LinearAlgebra.mul!(y::StridedVector, A::HIPShardedSparseMatrix, x::StridedVector) = mul!(y, A, x, true, false)
LinearAlgebra.mul!(y::StridedVector, adjA::AdjOrTransSharded, x::StridedVector) = mul!(y, adjA, x, true, false)

# Multi-RHS (the reference has no matrix mul!, multiply_1DVBC.jl:184-185): Y = α·op(A)·X + β·Y on
# column-major matrices of the compute eltype through vbc_mul_mat_ex (eltypes carried; B'X on
# matrix cores for a handle built with VBC_CREATE_MULTI), other eltypes column by column.
# (A handle built with multi=true runs both directions on matrix cores, the matrix read once for all
# right-hand sides; otherwise one SpMV per column.)
function _mul_mat!(Y::StridedMatrix{T}, A::HIPMatrix, trans::Bool, X::StridedMatrix{T}, α::Number,
                   β::Number) where {T <: Union{Float64, Float32}}
    h = handle_for(A, T)
    GC.@preserve X Y check(ccall((:vbc_mul_mat_ex, libvbc), Cint,
        (Ptr{Cvoid}, Cint, Int64, Ptr{T}, Cint, Int64, Int64, Ptr{T}, Cint, Int64, Int64, Cdouble, Cdouble, Cint,
         Ptr{Cvoid}, Cuint),
        h, trans, size(X, 2), X, vbc_dtype(T), stride(X, 2), size(X, 1), Y, vbc_dtype(T), stride(Y, 2), size(Y, 1),
        Float64(α), Float64(β), VBC_MEM_HOST, C_NULL, Cuint(0)))
    return Y
end
function LinearAlgebra.mul!(Y::StridedMatrix{T}, adjA::AdjOrTransHIP, X::StridedMatrix{T}, α::Number,
                            β::Number) where {T <: Union{Float64, Float32}}
    (stride(X, 1) == 1 && stride(Y, 1) == 1) || return _mul_cols!(Y, adjA, X, α, β)
    return _mul_mat!(Y, parent(adjA), true, X, α, β)
end
function LinearAlgebra.mul!(Y::StridedMatrix{T}, A::HIPMatrix, X::StridedMatrix{T}, α::Number,
                            β::Number) where {T <: Union{Float64, Float32}}
    (stride(X, 1) == 1 && stride(Y, 1) == 1) || return _mul_cols!(Y, A, X, α, β)
    return _mul_mat!(Y, A, false, X, α, β)
end
function _mul_cols!(Y::StridedMatrix, adjA, X::StridedMatrix, α::Number, β::Number)
    size(X, 2) == size(Y, 2) || throw(DimensionMismatch("X and Y have different numbers of columns"))
    for c in axes(X, 2)
        mul!(view(Y, :, c), adjA, view(X, :, c), α, β)
    end
    return Y
end
LinearAlgebra.mul!(Y::StridedMatrix, adjA::AdjOrTransHIP, X::StridedMatrix, α::Number, β::Number) =
    _mul_cols!(Y, adjA, X, α, β)
LinearAlgebra.mul!(Y::StridedMatrix, A::HIPMatrix, X::StridedMatrix, α::Number, β::Number) = _mul_cols!(Y, A, X, α, β)

export HIPShardedSparseMatrix
export HIPSparseMatrix1DVBC, HIPSparseMatrixVBC, HIPSparseMatrixCSC, HIPShardedSparseMatrix1DVBC, TrSpMV!

end # module
