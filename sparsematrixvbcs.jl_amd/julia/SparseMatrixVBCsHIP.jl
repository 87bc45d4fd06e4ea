# SparseMatrixVBCsHIP.jl -- the `ccall` layer a SparseMatrixVBCs.jl maintainer would add so that
# `mul!` on the reference's own types runs on an MI355X through libvbc (include/vbc.h).
#
# NOT EXECUTED IN THIS REPOSITORY: there is no Julia toolchain in the build image, so this file is
# syntax-reviewed only.  Every ccall signature mirrors include/vbc.h one to one; the Python mirror
# (sparsematrixvbcs.jl_amd/*.py), which IS tested on the GPU, binds the same symbols the same way.
#
# Usage (after `using SparseMatrixVBCs, AMDGPU`):
#     B  = SparseMatrix1DVBC{8}(A)                 # reference constructor, unchanged
#     Bd = HIPSparseMatrix1DVBC(B)                 # uploads once (vbc1d_create)
#     mul!(y_dev, Bd', x_dev)                      # ROCArrays: enqueued on the task-local stream
#     mul!(y_host, Bd', x_host)                    # Vectors: staged through HBM, synchronous
module SparseMatrixVBCsHIP

using LinearAlgebra
using SparseArrays
using SparseMatrixVBCs: SparseMatrix1DVBC, SparseMatrixVBC

const libvbc = get(ENV, "VBC_LIBRARY", joinpath(@__DIR__, "..", "libvbc.so"))

const VBC_OK, VBC_DIM_MISMATCH, VBC_INVALID_ARG, VBC_HIP_ERROR, VBC_RCCL_ERROR,
      VBC_UNSUPPORTED_DTYPE, VBC_ASSERTION = 0, 1, 2, 3, 4, 5, 6
const VBC_F64, VBC_F32 = Cint(0), Cint(1)
const VBC_MEM_DEVICE, VBC_MEM_HOST = Cint(0), Cint(1)
const VBC_CREATE_TRANSPOSED, VBC_CREATE_FORWARD = Cuint(1), Cuint(2)
const VBC_MUL_REFERENCE_QUIRKS = Cuint(1)

vbc_dtype(::Type{Float64}) = VBC_F64
vbc_dtype(::Type{Float32}) = VBC_F32
vbc_dtype(::Type{T}) where {T} = throw(MethodError(vbc_dtype, (T,)))

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
    throw(ErrorException(last_error()))
end

"""
    HIPSparseMatrix1DVBC(B::SparseMatrix1DVBC; device=0, forward=true, transposed=true)

Device-resident copy of `B` (the host struct is kept for `size`, printing and CPU fallbacks the
caller may want).  Immutable; freed by a finalizer (`vbc_destroy`).
"""
mutable struct HIPSparseMatrix1DVBC{W, Tv}
    host::SparseMatrix1DVBC{W, Tv, Int}
    handle::Ptr{Cvoid}
end

function HIPSparseMatrix1DVBC(B::SparseMatrix1DVBC{W, Tv, Int}; device::Integer=0,
                              forward::Bool=true, transposed::Bool=true) where {W, Tv}
    h = Ref{Ptr{Cvoid}}(C_NULL)
    flags = (transposed ? VBC_CREATE_TRANSPOSED : Cuint(0)) | (forward ? VBC_CREATE_FORWARD : Cuint(0))
    GC.@preserve B check(ccall((:vbc1d_create, libvbc), Cint,
        (Ptr{Ptr{Cvoid}}, Int64, Int64, Int64, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Int64},
         Ptr{Int64}, Ptr{Cvoid}, Int64, Cint, Cint, Cuint),
        h, B.m, B.n, W, length(B.Φ), B.Φ.spl, B.pos, B.idx, B.ofs, B.val, length(B.val),
        vbc_dtype(Tv), device, flags))
    M = HIPSparseMatrix1DVBC{W, Tv}(B, h[])
    finalizer(M) do M
        ccall((:vbc_destroy, libvbc), Cint, (Ptr{Cvoid},), M.handle)
    end
    return M
end

mutable struct HIPSparseMatrixVBC{U, W, Tv}
    host::SparseMatrixVBC{U, W, Tv, Int}
    handle::Ptr{Cvoid}
end

function HIPSparseMatrixVBC(B::SparseMatrixVBC{U, W, Tv, Int}; device::Integer=0,
                            forward::Bool=true, transposed::Bool=true) where {U, W, Tv}
    h = Ref{Ptr{Cvoid}}(C_NULL)
    flags = (transposed ? VBC_CREATE_TRANSPOSED : Cuint(0)) | (forward ? VBC_CREATE_FORWARD : Cuint(0))
    GC.@preserve B check(ccall((:vbc2d_create, libvbc), Cint,
        (Ptr{Ptr{Cvoid}}, Int64, Int64, Int64, Int64, Int64, Ptr{Int64}, Int64, Ptr{Int64},
         Ptr{Int64}, Ptr{Int64}, Ptr{Int64}, Ptr{Cvoid}, Int64, Cint, Cint, Cuint),
        h, B.m, B.n, U, W, length(B.Π), B.Π.spl, length(B.Φ), B.Φ.spl, B.pos, B.idx, B.ofs,
        B.val, length(B.val), vbc_dtype(Tv), device, flags))
    M = HIPSparseMatrixVBC{U, W, Tv}(B, h[])
    finalizer(M) do M
        ccall((:vbc_destroy, libvbc), Cint, (Ptr{Cvoid},), M.handle)
    end
    return M
end

const HIPMatrix = Union{HIPSparseMatrix1DVBC, HIPSparseMatrixVBC}
Base.size(A::HIPMatrix) = size(A.host)
Base.size(A::HIPMatrix, d::Integer) = size(A.host, d)

# Host vectors: staged by libvbc, synchronous.
function _mul!(y::StridedVector{T}, A::HIPMatrix, trans::Bool, x::StridedVector{T},
               α::Number, β::Number; quirks::Bool=false) where {T}
    (stride(x, 1) == 1 && stride(y, 1) == 1) || throw(ArgumentError("unit-stride vectors only"))
    GC.@preserve x y check(ccall((:vbc_mul, libvbc), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cdouble, Cdouble, Cint, Ptr{Cvoid}, Cuint),
        A.handle, trans, x, length(x), y, length(y), Float64(α), Float64(β), VBC_MEM_HOST, C_NULL,
        quirks ? VBC_MUL_REFERENCE_QUIRKS : Cuint(0)))
    return y
end

# The reference's operator surface: mul!(y, B, x, α, β) and mul!(y, B', x, α, β)
# (multiply_1DVBC.jl:9, :85; multiply_VBC.jl:3, :89) plus the 3-argument forms and Base.:*.
LinearAlgebra.mul!(y::StridedVector, A::HIPMatrix, x::StridedVector, α::Number, β::Number) =
    _mul!(y, A, false, x, α, β)
LinearAlgebra.mul!(y::StridedVector, adjA::Union{Adjoint{<:Any, <:HIPMatrix}, Transpose{<:Any, <:HIPMatrix}},
                   x::StridedVector, α::Number, β::Number) = _mul!(y, parent(adjA), true, x, α, β)
LinearAlgebra.mul!(y::StridedVector, A::HIPMatrix, x::StridedVector) = mul!(y, A, x, true, false)
LinearAlgebra.mul!(y::StridedVector, adjA::Union{Adjoint{<:Any, <:HIPMatrix}, Transpose{<:Any, <:HIPMatrix}},
                   x::StridedVector) = mul!(y, adjA, x, true, false)
Base.:*(A::HIPMatrix, x::StridedVector{T}) where {T} = mul!(similar(x, T, size(A, 1)), A, x, true, false)
Base.:*(adjA::Union{Adjoint{<:Any, <:HIPMatrix}, Transpose{<:Any, <:HIPMatrix}}, x::StridedVector{T}) where {T} =
    mul!(similar(x, T, size(adjA, 1)), adjA, x, true, false)

# TrSpMV!(y, A::SparseMatrixCSC, x) (TrSpMV.jl:1-20) through a CSC handle.
mutable struct HIPSparseMatrixCSC{Tv}
    host::SparseMatrixCSC{Tv, Int}
    handle::Ptr{Cvoid}
end
function HIPSparseMatrixCSC(A::SparseMatrixCSC{Tv, Int}; device::Integer=0) where {Tv}
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve A check(ccall((:vbc_csc_create, libvbc), Cint,
        (Ptr{Ptr{Cvoid}}, Int64, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Cvoid}, Cint, Cint, Cuint),
        h, size(A, 1), size(A, 2), A.colptr, A.rowval, A.nzval, vbc_dtype(Tv), device, VBC_CREATE_TRANSPOSED))
    M = HIPSparseMatrixCSC{Tv}(A, h[])
    finalizer(M) do M
        ccall((:vbc_destroy, libvbc), Cint, (Ptr{Cvoid},), M.handle)
    end
    return M
end
function TrSpMV!(y::Vector{T}, A::HIPSparseMatrixCSC{T}, x::Vector{T}) where {T}
    GC.@preserve x y check(ccall((:vbc_mul, libvbc), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cdouble, Cdouble, Cint, Ptr{Cvoid}, Cuint),
        A.handle, 1, x, length(x), y, length(y), 1.0, 0.0, VBC_MEM_HOST, C_NULL, Cuint(0)))
    return y
end

# Device arrays (AMDGPU.jl ROCArray): enqueue on the task-local HIP stream, no synchronisation.
# Kept behind a package extension so the shim has no hard AMDGPU dependency:
#
#   function LinearAlgebra.mul!(y::ROCVector{T}, adjA::Adjoint{<:Any,<:HIPMatrix}, x::ROCVector{T},
#                               α::Number, β::Number) where {T}
#       check(ccall((:vbc_mul, libvbc), Cint,
#           (Ptr{Cvoid}, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cdouble, Cdouble, Cint, Ptr{Cvoid}, Cuint),
#           parent(adjA).handle, 1, pointer(x), length(x), pointer(y), length(y), α, β,
#           VBC_MEM_DEVICE, AMDGPU.stream().stream, 0))
#       return y
#   end

export HIPSparseMatrix1DVBC, HIPSparseMatrixVBC, HIPSparseMatrixCSC, TrSpMV!

end # module
