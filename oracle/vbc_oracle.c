/*
 * oracle/vbc_oracle.c -- CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the SparseMatrixVBCs.jl (reference, v0.1.12, Julia) algorithms that sit on
 * the variable-block SpMV hot path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline -- never as the
 * thing measured or shipped.  The product path (sparsematrixvbcs.jl_amd/) never links it.
 *
 * Conventions: every index array holds 1-based Int64 values exactly as the Julia struct fields do
 * (Ti = Int64), so each loop below reads like the Julia line it restates.  AT(a, i) is a[i] in Julia.
 *
 * Pinning: the reference cannot run here (no julia binary -- SURVEY.md §8c).  This restatement is
 * pinned by (1) the reference's own test protocol (test/runtests.jl:29-53,63-87: one-hot probes must
 * reproduce the CSC product exactly) on the six matrices of test/matrices.jl, committed as
 * tests/golden/ fixtures; (2) random-x products vs scipy CSC within the reference's own isapprox
 * tolerance (bin/test_table.jl:42,84,126); (3) hand-derived layout KATs (tests/test_oracle.py).
 *
 * Semantics: `ref_semantics != 0` reproduces the reference exactly, including its quirks
 * (forward: alpha is computed and dropped, multiply_1DVBC.jl:48 / multiply_VBC.jl:55-57;
 * transposed: y is overwritten, so alpha and beta are both ignored, multiply_1DVBC.jl:114-116,
 * multiply_VBC.jl:117-121).  `ref_semantics == 0` is BLAS: y = alpha*op(A)*x + beta*y.
 * At alpha=1, beta=0 the two agree; it is the only case the reference tests (runtests.jl:36-37).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef int64_t Ti;
#define AT(a, i) ((a)[(i) - 1])

enum { ORC_OK = 0, ORC_DIM_MISMATCH = 1, ORC_INVALID_ARG = 2, ORC_ASSERTION = 6 };

/* ---------------------------------------------------------------------------------------------
 * Construction: SparseMatrix1DVBC{W}(A::SparseMatrixCSC, Φ)   constructors_1DVBC.jl:9-92
 * Pass 1 (counting, :13-33): distinct rows per stripe with the last-seen histogram `hst`.
 * ------------------------------------------------------------------------------------------- */
int orc_1dvbc_count(int64_t m, int64_t n, const Ti *A_pos, const Ti *A_idx, int64_t L,
                    const Ti *spl, Ti *pos, Ti *ofs)
{
    (void)n;
    Ti *hst = (Ti *)calloc((size_t)(m + 1), sizeof(Ti)); /* zeros(Ti, m + 1)  :12 */
    if (!hst) return ORC_INVALID_ARG;
    AT(pos, 1) = 1; /* :20 */
    AT(ofs, 1) = 1; /* :21 */
    for (int64_t l = 1; l <= L; l++) {
        AT(pos, l + 1) = AT(pos, l);
        Ti j = AT(spl, l), jn = AT(spl, l + 1);
        for (Ti q = AT(A_pos, j); q <= AT(A_pos, jn) - 1; q++) { /* :26-30 */
            Ti i = AT(A_idx, q);
            AT(pos, l + 1) += (AT(hst, i) < l);
            AT(hst, i) = l;
        }
        AT(ofs, l + 1) = AT(ofs, l) + (AT(pos, l + 1) - AT(pos, l)) * (jn - j); /* :31 */
    }
    free(hst);
    return ORC_OK;
}

/* Pass 2 (fill, constructors_1DVBC.jl:34-89): allocate idx/val (val gets `pad` trailing zeros,
 * the reference's Δw*cld(W,Δw) SIMD tail pad, :35-39), then per stripe either copy (w == 1, :47-55)
 * or merge the stripe's w columns row by row, zero-filling missing entries (:56-88). */
#define DEF_1DVBC_FILL(SUF, T)                                                                     \
    int orc_1dvbc_fill_##SUF(int64_t m, int64_t n, int64_t W, const Ti *A_pos, const Ti *A_idx,    \
                             const T *A_val, int64_t L, const Ti *spl, const Ti *pos,              \
                             const Ti *ofs, Ti *idx, T *val, int64_t pad)                          \
    {                                                                                              \
        (void)n;                                                                                   \
        for (Ti q = AT(ofs, L + 1); q <= AT(ofs, L + 1) - 1 + pad; q++) AT(val, q) = (T)0;         \
        Ti A_q[W + 1]; /* ones(Int, W)  :41 -- 1-based, slot 0 unused */                           \
        for (int64_t l = 1; l <= L; l++) {                                                         \
            Ti j = AT(spl, l);                                                                     \
            Ti w = AT(spl, l + 1) - j;                                                             \
            if (!(w <= W)) return ORC_ASSERTION; /* @assert w <= W  :46 */                         \
            if (w == 1) {                                                                          \
                Ti Q = AT(pos, l), q = AT(ofs, l);                                                 \
                for (Ti A_q_1 = AT(A_pos, j); A_q_1 <= AT(A_pos, j + w) - 1; A_q_1++) {            \
                    AT(idx, Q) = AT(A_idx, A_q_1);                                                 \
                    AT(val, q) = AT(A_val, A_q_1);                                                 \
                    Q += 1;                                                                        \
                    q += 1;                                                                        \
                }                                                                                  \
            } else {                                                                               \
                Ti i = m + 1;                                                                      \
                for (Ti dj = 1; dj <= w; dj++) {                                                   \
                    A_q[dj] = AT(A_pos, j + dj - 1);                                               \
                    if (A_q[dj] < AT(A_pos, j + dj)) {                                             \
                        Ti c = AT(A_idx, A_q[dj]);                                                 \
                        i = c < i ? c : i;                                                         \
                    }                                                                              \
                }                                                                                  \
                Ti Q = AT(pos, l), q = AT(ofs, l);                                                 \
                while (i != m + 1) {                                                               \
                    Ti in = m + 1;                                                                 \
                    for (Ti dj = 1; dj <= w; dj++) {                                               \
                        if (A_q[dj] < AT(A_pos, j + dj)) {                                         \
                            if (AT(A_idx, A_q[dj]) == i) {                                         \
                                AT(val, q) = AT(A_val, A_q[dj]);                                   \
                                A_q[dj] += 1;                                                      \
                            } else {                                                               \
                                AT(val, q) = (T)0;                                                 \
                            }                                                                      \
                            if (A_q[dj] < AT(A_pos, j + dj)) {                                     \
                                Ti c = AT(A_idx, A_q[dj]);                                         \
                                in = c < in ? c : in;                                              \
                            }                                                                      \
                        } else {                                                                   \
                            AT(val, q) = (T)0;                                                     \
                        }                                                                          \
                        q += 1;                                                                    \
                    }                                                                              \
                    AT(idx, Q) = i;                                                                \
                    Q += 1;                                                                        \
                    i = in;                                                                        \
                }                                                                                  \
            }                                                                                      \
        }                                                                                          \
        return ORC_OK;                                                                             \
    }
DEF_1DVBC_FILL(f64, double)
DEF_1DVBC_FILL(f32, float)

/* ---------------------------------------------------------------------------------------------
 * StrictChunker fast path  constructors_1DVBC.jl:94-143.  Assumes every column of a stripe shares
 * the first column's pattern (the reference does not check; neither do we).
 * ------------------------------------------------------------------------------------------- */
int orc_1dvbc_strict_count(int64_t m, int64_t n, const Ti *A_pos, int64_t L, const Ti *spl,
                           Ti *pos, Ti *ofs)
{
    (void)m; (void)n;
    AT(pos, 1) = 1;
    AT(ofs, 1) = 1;
    for (int64_t l = 1; l <= L; l++) { /* :110-115 */
        Ti j = AT(spl, l), jn = AT(spl, l + 1);
        Ti jj = (j + 1 < jn) ? j + 1 : jn;
        AT(pos, l + 1) = AT(pos, l) + AT(A_pos, jj) - AT(A_pos, j);
        AT(ofs, l + 1) = AT(A_pos, jn);
    }
    return ORC_OK;
}

#define DEF_STRICT_FILL(SUF, T)                                                                    \
    int orc_1dvbc_strict_fill_##SUF(int64_t m, int64_t n, int64_t W, const Ti *A_pos,              \
                                    const Ti *A_idx, const T *A_val, int64_t L, const Ti *spl,     \
                                    const Ti *pos, const Ti *ofs, Ti *idx, T *val, int64_t pad)    \
    {                                                                                              \
        (void)m; (void)n;                                                                          \
        for (Ti q = AT(ofs, L + 1); q <= AT(ofs, L + 1) - 1 + pad; q++) AT(val, q) = (T)0;         \
        for (int64_t l = 1; l <= L; l++) { /* :126-138 */                                          \
            Ti j = AT(spl, l);                                                                     \
            Ti w = AT(spl, l + 1) - j;                                                             \
            if (!(w <= W)) return ORC_ASSERTION;                                                   \
            Ti cnt = AT(A_pos, j + 1) - AT(A_pos, j);                                              \
            for (Ti Q = 0; Q <= cnt - 1; Q++) AT(idx, AT(pos, l) + Q) = AT(A_idx, AT(A_pos, j) + Q); \
            for (Ti jc = AT(spl, l); jc <= AT(spl, l + 1) - 1; jc++)                               \
                for (Ti Q = 0; Q <= cnt - 1; Q++)                                                  \
                    AT(val, AT(ofs, l) + Q * w + jc - j) = AT(A_val, AT(A_pos, jc) + Q);           \
        }                                                                                          \
        return ORC_OK;                                                                             \
    }
DEF_STRICT_FILL(f64, double)
DEF_STRICT_FILL(f32, float)

/* ---------------------------------------------------------------------------------------------
 * Construction: SparseMatrixVBC{U,W}(A, Π, Φ)   constructors_VBC.jl:15-133
 * Π_asg is convert(MapPartition, Π).asg: the block-row id of each row (:21).
 * ------------------------------------------------------------------------------------------- */
static Ti *orc_asg(int64_t m, int64_t K, const Ti *pspl)
{
    Ti *asg = (Ti *)malloc((size_t)(m > 0 ? m : 1) * sizeof(Ti));
    if (!asg) return NULL;
    for (int64_t k = 1; k <= K; k++)
        for (Ti i = AT(pspl, k); i < AT(pspl, k + 1); i++) AT(asg, i) = k;
    return asg;
}

int orc_vbc_count(int64_t m, int64_t n, const Ti *A_pos, const Ti *A_idx, int64_t K,
                  const Ti *pspl, int64_t L, const Ti *spl, Ti *pos, Ti *ofs)
{
    (void)n;
    Ti *asg = orc_asg(m, K, pspl);
    Ti *hst = (Ti *)calloc((size_t)(K + 1), sizeof(Ti)); /* zeros(Ti, K)  :22 */
    if (!asg || !hst) { free(asg); free(hst); return ORC_INVALID_ARG; }
    AT(pos, 1) = 1;
    AT(ofs, 1) = 1;
    for (int64_t l = 1; l <= L; l++) { /* :30-46 */
        AT(ofs, l + 1) = AT(ofs, l);
        AT(pos, l + 1) = AT(pos, l);
        Ti j = AT(spl, l), jn = AT(spl, l + 1), w = jn - j;
        for (Ti q = AT(A_pos, j); q <= AT(A_pos, jn) - 1; q++) {
            Ti i = AT(A_idx, q), k = AT(asg, i);
            if (AT(hst, k) < l) {
                Ti u = AT(pspl, k + 1) - AT(pspl, k);
                AT(pos, l + 1) += 1;
                AT(ofs, l + 1) += u * w;
            }
            AT(hst, k) = l;
        }
    }
    free(asg);
    free(hst);
    return ORC_OK;
}

#define DEF_VBC_FILL(SUF, T)                                                                       \
    int orc_vbc_fill_##SUF(int64_t m, int64_t n, int64_t U, int64_t W, const Ti *A_pos,            \
                           const Ti *A_idx, const T *A_val, int64_t K, const Ti *pspl, int64_t L,  \
                           const Ti *spl, const Ti *pos, const Ti *ofs, Ti *idx, T *val,           \
                           int64_t pad)                                                            \
    {                                                                                              \
        (void)n;                                                                                   \
        for (Ti q = AT(ofs, L + 1); q <= AT(ofs, L + 1) - 1 + pad; q++) AT(val, q) = (T)0;         \
        for (int64_t k = 1; k <= K; k++) /* :57-59 */                                              \
            if (!(AT(pspl, k + 1) - AT(pspl, k) <= U)) return ORC_ASSERTION;                       \
        Ti *asg = orc_asg(m, K, pspl);                                                             \
        if (!asg) return ORC_INVALID_ARG;                                                          \
        Ti A_q[W + 1];                                                                             \
        for (int64_t l = 1; l <= L; l++) {                                                         \
            Ti j = AT(spl, l);                                                                     \
            Ti w = AT(spl, l + 1) - j;                                                             \
            if (!(w <= W)) { free(asg); return ORC_ASSERTION; } /* :65 */                          \
            if (w == 1) { /* :66-83 */                                                             \
                Ti Q = AT(pos, l), q = AT(ofs, l);                                                 \
                Ti A_q_1 = AT(A_pos, j);                                                           \
                while (A_q_1 < AT(A_pos, j + 1)) {                                                 \
                    Ti k = AT(asg, AT(A_idx, A_q_1));                                              \
                    for (Ti i = AT(pspl, k); i <= AT(pspl, k + 1) - 1; i++) {                      \
                        if (A_q_1 < AT(A_pos, j + 1) && AT(A_idx, A_q_1) == i) {                   \
                            AT(val, q) = AT(A_val, A_q_1);                                         \
                            A_q_1 += 1;                                                            \
                        } else {                                                                   \
                            AT(val, q) = (T)0;                                                     \
                        }                                                                          \
                        q += 1;                                                                    \
                    }                                                                              \
                    AT(idx, Q) = k;                                                                \
                    Q += 1;                                                                        \
                }                                                                                  \
            } else { /* :84-129 */                                                                 \
                Ti k = K + 1;                                                                      \
                for (Ti dj = 1; dj <= w; dj++) {                                                   \
                    A_q[dj] = AT(A_pos, j + dj - 1);                                               \
                    if (A_q[dj] < AT(A_pos, j + dj)) {                                             \
                        Ti c = AT(asg, AT(A_idx, A_q[dj]));                                        \
                        k = c < k ? c : k;                                                         \
                    }                                                                              \
                }                                                                                  \
                Ti Q = AT(pos, l), q = AT(ofs, l);                                                 \
                while (k != K + 1) {                                                               \
                    for (Ti i = AT(pspl, k); i <= AT(pspl, k + 1) - 2; i++) {                      \
                        for (Ti dj = 1; dj <= w; dj++) {                                           \
                            if (A_q[dj] < AT(A_pos, j + dj) && AT(A_idx, A_q[dj]) == i) {          \
                                AT(val, q) = AT(A_val, A_q[dj]);                                   \
                                A_q[dj] += 1;                                                      \
                            } else {                                                               \
                                AT(val, q) = (T)0;                                                 \
                            }                                                                      \
                            q += 1;                                                                \
                        }                                                                          \
                    }                                                                              \
                    Ti kn = K + 1;                                                                 \
                    {                                                                              \
                        Ti i = AT(pspl, k + 1) - 1;                                                \
                        for (Ti dj = 1; dj <= w; dj++) {                                           \
                            if (A_q[dj] < AT(A_pos, j + dj)) {                                     \
                                if (AT(A_idx, A_q[dj]) == i) {                                     \
                                    AT(val, q) = AT(A_val, A_q[dj]);                               \
                                    A_q[dj] += 1;                                                  \
                                } else {                                                           \
                                    AT(val, q) = (T)0;                                             \
                                }                                                                  \
                                if (A_q[dj] < AT(A_pos, j + dj)) {                                 \
                                    Ti c = AT(asg, AT(A_idx, A_q[dj]));                            \
                                    kn = c < kn ? c : kn;                                          \
                                }                                                                  \
                            } else {                                                               \
                                AT(val, q) = (T)0;                                                 \
                            }                                                                      \
                            q += 1;                                                                \
                        }                                                                          \
                    }                                                                              \
                    AT(idx, Q) = k;                                                                \
                    Q += 1;                                                                        \
                    k = kn;                                                                        \
                }                                                                                  \
            }                                                                                      \
        }                                                                                          \
        free(asg);                                                                                 \
        return ORC_OK;                                                                             \
    }
DEF_VBC_FILL(f64, double)
DEF_VBC_FILL(f32, float)

/* ---------------------------------------------------------------------------------------------
 * β pre-scaling shared by every mul!: `if β != 1; β != 0 ? rmul!(y, β) : fill!(y, 0)`
 * (multiply_1DVBC.jl:50-52, :145-147; multiply_VBC.jl:55-57, :156-158).
 * ------------------------------------------------------------------------------------------- */
#define DEF_BETA(SUF, T)                                                                           \
    static void orc_beta_##SUF(T *y, int64_t ny, double beta)                                      \
    {                                                                                              \
        if (beta != 1.0) {                                                                         \
            if (beta != 0.0)                                                                       \
                for (int64_t i = 0; i < ny; i++) y[i] = (T)(y[i] * (T)beta);                       \
            else                                                                                   \
                for (int64_t i = 0; i < ny; i++) y[i] = (T)0;                                      \
        }                                                                                          \
    }
DEF_BETA(f64, double)
DEF_BETA(f32, float)

/* ---------------------------------------------------------------------------------------------
 * Forward 1DVBC  mul!(y, B, x, α, β)   multiply_1DVBC.jl:9-83.
 * Per stripe: tmp = x[j:j+w-1] (:27); per stored row: y[idx[Q]] += sum(val[q:q+w-1] .* tmp) (:34).
 * Lanes >= w of the SIMD bucket multiply by tmp = 0 and are omitted.  The horizontal `sum` is
 * accumulated left to right with fma.  ref_semantics: α dropped (yα unused, :48).
 * ------------------------------------------------------------------------------------------- */
#define DEF_1DVBC_MUL(SUF, T, FMA)                                                                 \
    int orc_1dvbc_mul_##SUF(int64_t m, int64_t n, int64_t L, const Ti *spl, const Ti *pos,         \
                            const Ti *idx, const Ti *ofs, const T *val, const T *x, int64_t nx,    \
                            T *y, int64_t ny, double alpha, double beta, int ref_semantics)        \
    {                                                                                              \
        if (m != ny) return ORC_DIM_MISMATCH; /* :44 */                                            \
        if (n != nx) return ORC_DIM_MISMATCH; /* :45 */                                            \
        orc_beta_##SUF(y, ny, beta);                                                               \
        const T a = ref_semantics ? (T)1 : (T)alpha;                                               \
        for (int64_t l = 1; l <= L; l++) {                                                         \
            Ti j = AT(spl, l), w = AT(spl, l + 1) - j;                                             \
            Ti q = AT(ofs, l);                                                                     \
            for (Ti Q = AT(pos, l); Q <= AT(pos, l + 1) - 1; Q++) {                                \
                T s = (T)0;                                                                        \
                for (Ti c = 0; c < w; c++) s = FMA(AT(val, q + c), AT(x, j + c), s);              \
                if (ref_semantics)                                                                 \
                    AT(y, AT(idx, Q)) += s;                                                        \
                else                                                                               \
                    AT(y, AT(idx, Q)) = FMA(a, s, AT(y, AT(idx, Q)));                             \
                q += w;                                                                            \
            }                                                                                      \
        }                                                                                          \
        return ORC_OK;                                                                             \
    }
DEF_1DVBC_MUL(f64, double, fma)
DEF_1DVBC_MUL(f32, float, fmaf)

/* ---------------------------------------------------------------------------------------------
 * Transposed 1DVBC  mul!(y, B', x, α, β)   multiply_1DVBC.jl:85-180.
 * Per stripe (:99-116): tmp = 0; for Q: tmp += val[q:q+w-1] * x[idx[Q]] (per lane, row order);
 * y[j:j+w-1] = tmp (overwrite).  Stripes are independent, so the OpenMP variant uses the
 * reference's dynamic 1-stripe self-scheduling (:169-177) when nthreads > 1.
 * ------------------------------------------------------------------------------------------- */
#define DEF_1DVBC_MUL_T(SUF, T, FMA)                                                               \
    int orc_1dvbc_mul_t_##SUF(int64_t m, int64_t n, int64_t L, const Ti *spl, const Ti *pos,       \
                              const Ti *idx, const Ti *ofs, const T *val, const T *x, int64_t nx,  \
                              T *y, int64_t ny, double alpha, double beta, int ref_semantics,      \
                              int nthreads)                                                        \
    {                                                                                              \
        if (n != ny) return ORC_DIM_MISMATCH; /* :139 */                                           \
        if (m != nx) return ORC_DIM_MISMATCH; /* :140 */                                           \
        if (ref_semantics) orc_beta_##SUF(y, ny, beta);                                            \
        const T a = (T)alpha, b = (T)beta;                                                         \
        (void)nthreads;                                                                            \
        _Pragma("omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)") \
        for (int64_t l = 1; l <= L; l++) {                                                         \
            Ti j = AT(spl, l), w = AT(spl, l + 1) - j;                                             \
            T tmp[64];                                                                             \
            T *t = w <= 64 ? tmp : (T *)malloc((size_t)w * sizeof(T));                             \
            for (Ti c = 0; c < w; c++) t[c] = (T)0;                                                \
            Ti q = AT(ofs, l);                                                                     \
            for (Ti Q = AT(pos, l); Q <= AT(pos, l + 1) - 1; Q++) {                                \
                T xv = AT(x, AT(idx, Q));                                                          \
                for (Ti c = 0; c < w; c++) t[c] = FMA(AT(val, q + c), xv, t[c]);                  \
                q += w;                                                                            \
            }                                                                                      \
            for (Ti c = 0; c < w; c++) {                                                           \
                if (ref_semantics)                                                                 \
                    AT(y, j + c) = t[c];                                                           \
                else if (b != (T)0)                                                                \
                    AT(y, j + c) = FMA(a, t[c], b * AT(y, j + c));                                \
                else                                                                               \
                    AT(y, j + c) = a * t[c];                                                       \
            }                                                                                      \
            if (t != tmp) free(t);                                                                 \
        }                                                                                          \
        return ORC_OK;                                                                             \
    }
DEF_1DVBC_MUL_T(f64, double, fma)
DEF_1DVBC_MUL_T(f32, float, fmaf)

/* ---------------------------------------------------------------------------------------------
 * Forward 2D VBC  mul!(y, B, x, α, β)   multiply_VBC.jl:7-87.  Per block k of stripe l:
 * rows i = Π.spl[k] .. +u-1, y[i+Δi] += sum(val[q+wΔi : q+wΔi+w-1] .* tmp) (:38-47), q += u*w (:32).
 * ref_semantics: α is not even computed on this path.
 * ------------------------------------------------------------------------------------------- */
#define DEF_VBC_MUL(SUF, T, FMA)                                                                   \
    int orc_vbc_mul_##SUF(int64_t m, int64_t n, int64_t K, const Ti *pspl, int64_t L,              \
                          const Ti *spl, const Ti *pos, const Ti *idx, const Ti *ofs,              \
                          const T *val, const T *x, int64_t nx, T *y, int64_t ny, double alpha,    \
                          double beta, int ref_semantics)                                          \
    {                                                                                              \
        (void)K;                                                                                   \
        if (m != ny) return ORC_DIM_MISMATCH; /* :51 */                                            \
        if (n != nx) return ORC_DIM_MISMATCH; /* :52 */                                            \
        orc_beta_##SUF(y, ny, beta);                                                               \
        const T a = ref_semantics ? (T)1 : (T)alpha;                                               \
        for (int64_t l = 1; l <= L; l++) {                                                         \
            Ti j = AT(spl, l), w = AT(spl, l + 1) - j;                                             \
            Ti q = AT(ofs, l);                                                                     \
            for (Ti Q = AT(pos, l); Q <= AT(pos, l + 1) - 1; Q++) {                                \
                Ti k = AT(idx, Q), i = AT(pspl, k), u = AT(pspl, k + 1) - i;                       \
                for (Ti di = 0; di < u; di++) {                                                    \
                    T s = (T)0;                                                                    \
                    for (Ti c = 0; c < w; c++) s = FMA(AT(val, q + w * di + c), AT(x, j + c), s); \
                    if (ref_semantics)                                                             \
                        AT(y, i + di) += s;                                                        \
                    else                                                                           \
                        AT(y, i + di) = FMA(a, s, AT(y, i + di));                                 \
                }                                                                                  \
                q += u * w;                                                                        \
            }                                                                                      \
        }                                                                                          \
        return ORC_OK;                                                                             \
    }
DEF_VBC_MUL(f64, double, fma)
DEF_VBC_MUL(f32, float, fmaf)

/* Transposed 2D VBC  mul!(y, B', x, α, β)   multiply_VBC.jl:89-192 (per stripe :99-124, per block
 * :126-135: tmp += val[q+wΔi : ...] * x[i+Δi]; then overwrite y[j+Δj] = tmp[1+Δj], :117-121). */
#define DEF_VBC_MUL_T(SUF, T, FMA)                                                                 \
    int orc_vbc_mul_t_##SUF(int64_t m, int64_t n, int64_t K, const Ti *pspl, int64_t L,            \
                            const Ti *spl, const Ti *pos, const Ti *idx, const Ti *ofs,            \
                            const T *val, const T *x, int64_t nx, T *y, int64_t ny, double alpha,  \
                            double beta, int ref_semantics, int nthreads)                          \
    {                                                                                              \
        (void)K;                                                                                   \
        if (n != ny) return ORC_DIM_MISMATCH; /* :152 */                                           \
        if (m != nx) return ORC_DIM_MISMATCH; /* :153 */                                           \
        if (ref_semantics) orc_beta_##SUF(y, ny, beta);                                            \
        const T a = (T)alpha, b = (T)beta;                                                         \
        (void)nthreads;                                                                            \
        _Pragma("omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)") \
        for (int64_t l = 1; l <= L; l++) {                                                         \
            Ti j = AT(spl, l), w = AT(spl, l + 1) - j;                                             \
            T tmp[64];                                                                             \
            T *t = w <= 64 ? tmp : (T *)malloc((size_t)w * sizeof(T));                             \
            for (Ti c = 0; c < w; c++) t[c] = (T)0;                                                \
            Ti q = AT(ofs, l);                                                                     \
            for (Ti Q = AT(pos, l); Q <= AT(pos, l + 1) - 1; Q++) {                                \
                Ti k = AT(idx, Q), i = AT(pspl, k), u = AT(pspl, k + 1) - i;                       \
                for (Ti di = 0; di < u; di++) {                                                    \
                    T xv = AT(x, i + di);                                                          \
                    for (Ti c = 0; c < w; c++) t[c] = FMA(AT(val, q + w * di + c), xv, t[c]);     \
                }                                                                                  \
                q += u * w;                                                                        \
            }                                                                                      \
            for (Ti c = 0; c < w; c++) {                                                           \
                if (ref_semantics)                                                                 \
                    AT(y, j + c) = t[c];                                                           \
                else if (b != (T)0)                                                                \
                    AT(y, j + c) = FMA(a, t[c], b * AT(y, j + c));                                \
                else                                                                               \
                    AT(y, j + c) = a * t[c];                                                       \
            }                                                                                      \
            if (t != tmp) free(t);                                                                 \
        }                                                                                          \
        return ORC_OK;                                                                             \
    }
DEF_VBC_MUL_T(f64, double, fma)
DEF_VBC_MUL_T(f32, float, fmaf)

/* ---------------------------------------------------------------------------------------------
 * TrSpMV!(y, A::SparseMatrixCSC, x)   TrSpMV.jl:1-20 -- y[i] = Σ_{p∈colptr[i]:colptr[i+1]-1}
 * nzval[p] * x[rowval[p]] (CSR-style product with Aᵀ), y overwritten.
 * ------------------------------------------------------------------------------------------- */
#define DEF_TRSPMV(SUF, T, FMA)                                                                    \
    int orc_trspmv_##SUF(int64_t m, int64_t n, const Ti *A_pos, const Ti *A_idx, const T *A_val,   \
                         const T *x, int64_t nx, T *y, int64_t ny, int nthreads)                   \
    {                                                                                              \
        if (n != ny) return ORC_DIM_MISMATCH; /* :3 */                                             \
        if (m != nx) return ORC_DIM_MISMATCH; /* :4 */                                             \
        (void)nthreads;                                                                            \
        _Pragma("omp parallel for schedule(dynamic, 64) num_threads(nthreads > 0 ? nthreads : 1)") \
        for (int64_t i = 1; i <= ny; i++) {                                                        \
            T tmp = (T)0;                                                                          \
            for (Ti j = AT(A_pos, i); j <= AT(A_pos, i + 1) - 1; j++)                              \
                tmp = FMA(AT(A_val, j), AT(x, AT(A_idx, j)), tmp);                                \
            AT(y, i) = tmp;                                                                        \
        }                                                                                          \
        return ORC_OK;                                                                             \
    }
DEF_TRSPMV(f64, double, fma)
DEF_TRSPMV(f32, float, fmaf)

/* Multi-RHS reference for SpMM parity: the reference has NO matrix mul! (SURVEY §0 trap 3), so
 * the only anchor is column-by-column application of the transposed vector product above.
 * X is m×k column-major (ldx), Y is n×k column-major (ldy). */
#define DEF_1DVBC_MULMAT_T(SUF, T)                                                                 \
    int orc_1dvbc_mulmat_t_##SUF(int64_t m, int64_t n, int64_t L, const Ti *spl, const Ti *pos,    \
                                 const Ti *idx, const Ti *ofs, const T *val, int64_t k,            \
                                 const T *X, int64_t ldx, T *Y, int64_t ldy, double alpha,         \
                                 double beta, int nthreads)                                        \
    {                                                                                              \
        for (int64_t r = 0; r < k; r++) {                                                          \
            int st = orc_1dvbc_mul_t_##SUF(m, n, L, spl, pos, idx, ofs, val, X + r * ldx, m,       \
                                           Y + r * ldy, n, alpha, beta, 0, nthreads);              \
            if (st) return st;                                                                     \
        }                                                                                          \
        return ORC_OK;                                                                             \
    }
DEF_1DVBC_MULMAT_T(f64, double)
DEF_1DVBC_MULMAT_T(f32, float)

int orc_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
