# Package extension: ROCArray operands for SparseMatrixVBCsHIP (loaded by `using AMDGPU`).
# Syntax-reviewed only (no Julia in the build image); the device-pointer path it binds
# (VBC_MEM_DEVICE, caller's stream, no synchronisation) is the one the Python mirror runs on the GPU
# with torch tensors.
module SparseMatrixVBCsHIPAMDGPUExt

using LinearAlgebra
using AMDGPU: ROCVector, AMDGPU
using SparseMatrixVBCsHIP: SparseMatrixVBCsHIP, HIPMatrix, AdjOrTransHIP, HIPShardedSparseMatrix,
                           AdjOrTransSharded, handle_for, check, vbc_dtype, libvbc, VBC_MEM_DEVICE,
                           VBC_MUL_REFERENCE_QUIRKS

# mul!(y, op(B), x, α, β) on device vectors: enqueued on the task-local HIP stream (AMDGPU.stream()),
# returns without synchronising -- a solver's product sequence stays on the device.
function _mul_dev!(y::ROCVector{Ty}, A::HIPMatrix, trans::Bool, x::ROCVector{Tx}, α::Number, β::Number;
                   quirks::Bool=false) where {Ty, Tx}
    h = handle_for(A, Ty)
    check(ccall((:vbc_mul_ex, libvbc), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Cvoid}, Cint, Int64, Int64, Ptr{Cvoid}, Cint, Int64, Int64, Cdouble, Cdouble, Cint,
         Ptr{Cvoid}, Cuint),
        h, trans, pointer(x), vbc_dtype(Tx), 1, length(x), pointer(y), vbc_dtype(Ty), 1, length(y), Float64(α),
        Float64(β), VBC_MEM_DEVICE, AMDGPU.stream().stream, quirks ? VBC_MUL_REFERENCE_QUIRKS : Cuint(0)))
    return y
end

LinearAlgebra.mul!(y::ROCVector, A::HIPMatrix, x::ROCVector, α::Number, β::Number) = _mul_dev!(y, A, false, x, α, β)
LinearAlgebra.mul!(y::ROCVector, adjA::AdjOrTransHIP, x::ROCVector, α::Number, β::Number) =
    _mul_dev!(y, parent(adjA), true, x, α, β)
LinearAlgebra.mul!(y::ROCVector, A::HIPMatrix, x::ROCVector) = mul!(y, A, x, true, false)
LinearAlgebra.mul!(y::ROCVector, adjA::AdjOrTransHIP, x::ROCVector) = mul!(y, adjA, x, true, false)
SparseMatrixVBCsHIP.TrSpMV!(y::ROCVector, A::SparseMatrixVBCsHIP.HIPSparseMatrixCSC, x::ROCVector) =
    _mul_dev!(y, A, true, x, true, false)

# Sharded handle: x and y on devices[1]; the exchange with the other GPUs is ordered on the same
# stream.  vbc_sharded_mul_ex carries both eltypes (x converted to the compute eltype on the device,
# a y of another eltype refused), so a mismatched ROCVector can never be read as another type.
function _mul_dev!(y::ROCVector{Ty}, A::HIPShardedSparseMatrix, trans::Bool, x::ROCVector{Tx}, α::Number,
                   β::Number; quirks::Bool=false) where {Ty, Tx}
    check(ccall((:vbc_sharded_mul_ex, libvbc), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Cvoid}, Cint, Int64, Int64, Ptr{Cvoid}, Cint, Int64, Int64, Cdouble, Cdouble, Cint,
         Ptr{Cvoid}, Cuint),
        A.handle, trans, pointer(x), vbc_dtype(Tx), 1, length(x), pointer(y), vbc_dtype(Ty), 1, length(y), Float64(α),
        Float64(β), VBC_MEM_DEVICE, AMDGPU.stream().stream, quirks ? VBC_MUL_REFERENCE_QUIRKS : Cuint(0)))
    return y
end
LinearAlgebra.mul!(y::ROCVector, A::HIPShardedSparseMatrix, x::ROCVector, α::Number, β::Number) =
    _mul_dev!(y, A, false, x, α, β)
LinearAlgebra.mul!(y::ROCVector, adjA::AdjOrTransSharded, x::ROCVector, α::Number, β::Number) =
    _mul_dev!(y, parent(adjA), true, x, α, β)
LinearAlgebra.mul!(y::ROCVector, A::HIPShardedSparseMatrix, x::ROCVector) = mul!(y, A, x, true, false)
LinearAlgebra.mul!(y::ROCVector, adjA::AdjOrTransSharded, x::ROCVector) = mul!(y, adjA, x, true, false)

end # module
