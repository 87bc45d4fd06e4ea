"""sparsematrixvbcs.jl_amd -- MI355X-native variable-block SpMV behind SparseMatrixVBCs.jl's surface.

Host mirror (Python stands in for the absent Julia host) of the reference's operator API:
SparseMatrix1DVBC / SparseMatrixVBC / mul! / TrSpMV! / Base.:*, over libvbc's C ABI
(include/vbc.h), whose hand-written gfx950 kernels do every product.  Import it as
`sparsematrixvbcs_amd` (the repo-root loader) since the directory name is not an identifier.
"""
from . import _lib, costs, distributed, io, synthetic
from ._lib import ArgumentError, DimensionMismatch, HIPError, UnsupportedDtype
from .matrices import (DEFAULT_SIMD_SIZE, Adjoint, SparseMatrix1DVBC, SparseMatrixCSC, SparseMatrixVBC,
                       Transpose, adjoint, transpose)
from .multiply import TrSpMV_, matmul, mul_, mulmat_
from .costs import TimedChunker, model_SparseMatrix1DVBC_TrSpMV_time, model_SparseMatrixVBC_TrSpMV_time
from .partition import (AlternatePacker, AlternatingPacker, BlockComponentCostModel, ColumnBlockCostModel,
                        ConstrainedCost, DynamicTotalChunker, EquiChunker, Line, OverlapChunker, SplitPartition,
                        StrictChunker, VertexCount, model_SparseMatrix1DVBC_blocks, model_SparseMatrix1DVBC_memory,
                        model_SparseMatrixVBC_blocks, model_SparseMatrixVBC_memory, pack_plaid, pack_stripe,
                        permutedims, total_value_2d)

# Julia spellings
globals()["mul!"] = mul_
globals()["TrSpMV!"] = TrSpMV_

__all__ = [
    "SparseMatrix1DVBC", "SparseMatrixVBC", "SparseMatrixCSC", "Adjoint", "Transpose", "adjoint",
    "transpose", "mul_", "mulmat_", "matmul", "TrSpMV_", "SplitPartition", "EquiChunker",
    "StrictChunker", "OverlapChunker", "DynamicTotalChunker", "ConstrainedCost", "VertexCount",
    "AlternatingPacker", "AlternatePacker", "pack_stripe", "pack_plaid",
    "model_SparseMatrix1DVBC_blocks", "model_SparseMatrix1DVBC_memory", "model_SparseMatrix1DVBC_TrSpMV_time", "TimedChunker",
    "ColumnBlockCostModel", "BlockComponentCostModel", "Line", "permutedims", "total_value_2d",
    "model_SparseMatrixVBC_blocks", "model_SparseMatrixVBC_memory", "model_SparseMatrixVBC_TrSpMV_time",
    "DimensionMismatch",
    "ArgumentError", "HIPError", "UnsupportedDtype", "DEFAULT_SIMD_SIZE",
]
