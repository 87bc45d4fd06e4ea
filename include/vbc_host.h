/*
 * vbc_host.h -- host-side layout producers of libvbc (no GPU needed).
 *
 * These build the reference's own data structures (1-based Int64 fields of SparseMatrix1DVBC /
 * SparseMatrixVBC) from a SparseMatrixCSC, so that a host without Julia (the Python mirror, tests,
 * bench) can produce exactly what `SparseMatrix1DVBC{W}(A, Φ)` / `SparseMatrixVBC{U,W}(A, Π, Φ)`
 * produce, and hand them to vbc1d_create / vbc2d_create.  A Julia caller does not need them: it
 * builds the struct with the reference's constructors and passes the fields straight to vbc.h.
 *
 * Partitioners stand in for the external ChainPartitioners.jl 1.1.6 (`pack_stripe`, Manifest.toml:
 * 23-29), which is absent from the container; partition parity is UNPINNED -- all
 * parity is defined per given partition.  Layout parity (given Φ / Π) is exact and is checked
 * against the oracle restatement of constructors_1DVBC.jl / constructors_VBC.jl.
 *
 * Conventions: colptr[n+1], rowval[nnz] are 1-based Int64 (SparseMatrixCSC fields), rows sorted
 * ascending within a column.  Output spl arrays are 1-based, spl[0] = 1, spl[L] = n+1; the caller
 * provides n+1 slots.  Return: vbc_status (vbc.h).
 */
#ifndef VBC_HOST_H
#define VBC_HOST_H

#ifndef VBC_API
#define VBC_API __attribute__((visibility("default")))  /* the library builds with -fvisibility=hidden */
#endif

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* EquiChunker(w): stripes of exactly w columns (last one shorter). */
VBC_API int vbcx_partition_equi(int64_t n, int64_t w, int64_t *spl, int64_t *L);

/* StrictChunker(W): maximal runs of consecutive columns with identical row patterns, width <= W. */
VBC_API int vbcx_partition_strict(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                          int64_t W, int64_t *spl, int64_t *L);

/* OverlapChunker(ρ, W): greedy; column j joins the open stripe while
 * |S(j) ∩ S(first)| >= ρ · max(|S(j)|, |S(first)|) and width < W (S = row pattern). */
VBC_API int vbcx_partition_overlap(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                           double rho, int64_t W, int64_t *spl, int64_t *L);

/* DynamicTotalChunker(model, W): optimal (minimum total cost) contiguous partition with width <= W
 * by dynamic programming, for the affine per-stripe cost
 *     cost(stripe) = c_stripe + c_col·w + c_pin·pins + c_row·rows + c_cell·w·rows
 * where rows = distinct rows of the stripe.  model_SparseMatrix1DVBC_memory(Tv, Ti) (costs.jl:10)
 * is (3Ti, 0, 0, Ti, Tv); model_SparseMatrix1DVBC_blocks() (costs.jl:8) is (0, 0, 0, 1, 0). */
VBC_API int vbcx_partition_dynamic(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                           int64_t W, double c_stripe, double c_col, double c_pin, double c_row,
                           double c_cell, int64_t *spl, int64_t *L);

/* DynamicTotalChunker over a ColumnBlockComponentCostModel (costs.jl:12, the TrSpMV time model):
 *     cost(stripe of width w with R distinct rows) = alpha[w-1] + beta[w-1]·R,   1 <= w <= W,
 * alpha / beta hold W entries (model_SparseMatrix1DVBC_TrSpMV_time fits them, costs.py). */
VBC_API int vbcx_partition_dynamic_table(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                                         int64_t W, const double *alpha, const double *beta, int64_t *spl,
                                         int64_t *L);

/* DynamicTotalChunker over a BlockComponentCostModel (costs.jl:138-142, the SparseMatrixVBC models):
 * the columns of A are partitioned while its rows are grouped into G block rows (grp[i] = 1-based
 * block row of row i, the other dimension's partition; NULL = every row its own group, G = m):
 *     cost(stripe of width w) = alpha[w-1] + Σ_r colw[r·W + w-1] · Σ_{block rows g it touches} gw[r·G + g]
 * i.e. the stripe's own cost plus, for every u_g × w block it stores, Σ_r β_row[r](u_g)·β_col[r](w)
 * (gw = β_row[r] evaluated at each group's height, colw = β_col[r] at each width; R <= 64 components,
 * the rank of the time model's SVD).  The row partition of pack_plaid's alternation is this call on
 * Aᵀ with the permuted model (permutedims swaps the row and column terms).  Optimal by dynamic
 * programming, width <= W. */
VBC_API int vbcx_partition_block(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                                 const int64_t *grp, int64_t G, int64_t R, const double *gw, int64_t W,
                                 const double *alpha, const double *colw, int64_t *spl, int64_t *L);

/* SparseMatrix1DVBC{W}(A, Φ) (constructors_1DVBC.jl:9-92): pass 1 fills pos[L+1], ofs[L+1]. */
VBC_API int vbcx_1dvbc_count(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval, int64_t L,
                     const int64_t *spl, int64_t *pos, int64_t *ofs);
/* pass 2 fills idx[pos[L]-1] and val[ofs[L]-1 + pad] (pad trailing zeros, :35-39).
 * dtype: any vbc_dtype (nzval and val have that eltype; values are copied, never converted). */
VBC_API int vbcx_1dvbc_fill(int64_t m, int64_t n, int64_t W, const int64_t *colptr, const int64_t *rowval,
                    const void *nzval, int dtype, int64_t L, const int64_t *spl, const int64_t *pos,
                    const int64_t *ofs, int64_t *idx, void *val, int64_t pad);

/* SparseMatrixVBC{U,W}(A, Π, Φ) (constructors_VBC.jl:15-133). */
VBC_API int vbcx_vbc_count(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval, int64_t K,
                   const int64_t *pspl, int64_t L, const int64_t *spl, int64_t *pos, int64_t *ofs);
VBC_API int vbcx_vbc_fill(int64_t m, int64_t n, int64_t U, int64_t W, const int64_t *colptr,
                  const int64_t *rowval, const void *nzval, int dtype, int64_t K,
                  const int64_t *pspl, int64_t L, const int64_t *spl, const int64_t *pos,
                  const int64_t *ofs, int64_t *idx, void *val, int64_t pad);

/* Row pattern of Aᵀ (CSR of A) for row partitioning: rowptr[m+1], colval[nnz], 1-based. */
VBC_API int vbcx_transpose_pattern(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                           int64_t *rowptr, int64_t *colval);

#ifdef __cplusplus
}
#endif
#endif /* VBC_HOST_H */
