/*
 * oracle/vbc_simd.c -- CPU BASELINE (a port of the reference's SIMD CPU kernels).
 * TEST / BENCHMARK INFRASTRUCTURE ONLY: only bench.py's cpu_baseline leg and tests/ load it, as the
 * CPU path timed beside the GPU.  The product path (sparsematrixvbcs.jl_amd/) never links it.
 *
 * Where vbc_oracle.c restates the reference's arithmetic in scalar C (the parity checker), this file
 * restates its *performance* shape, so that the CPU number bench.py reports is the reference's own
 * CPU path and not an understated scalar loop:
 *   - transposed 1DVBC  mul!(y, B', x)  multiply_1DVBC.jl:90-134 (per stripe) and :136-180 (driver):
 *     per stripe a Vec{$w} accumulator, $w the smallest width bucket >= w from
 *     ws = (1, Δw, 2Δw, ...) (le_nest, util.jl:28-38), Δw = DEFAULT_SIMD_SIZE / sizeof(T)
 *     (SparseMatrixVBCs.jl:17; 64 B on the AVX-512 hosts the reference targets); each stored row is
 *     one vload(Vec{$w}, val, q) -- it reads past the stripe's w values, which is what the SIMD tail
 *     pad of constructors_1DVBC.jl:35-39 is for -- times the broadcast x[idx[Q]] (:101-104), then the
 *     first w lanes are stored (:114-116); @fastmath (:129-131) -> built with -ffast-math;
 *     threads self-schedule one stripe per atomic grab (Atomic{Int} + @threads, :169-177);
 *   - forward 1DVBC  mul!(y, B, x)  multiply_1DVBC.jl:9-83: serial; per stripe the zero-padded x
 *     slice as a Vec{$w}, per row y[idx[Q]] += sum(vload(val, q) * tmp);
 *   - TrSpMV!(y, A::SparseMatrixCSC, x)  TrSpMV.jl:1-20: serial row-dot per CSC column, @fastmath.
 * Index arrays are the reference's 1-based Int64 (Ti = Int64).  Semantics at α = 1, β = 0 (the
 * benchmarked case, bin/test_table.jl:80): transposed overwrites y, forward zero-fills then
 * accumulates.
 *
 * Vector width: GCC vector extensions of 64 bytes (Δw = 8 for Float64, 16 for Float32), compiled as
 * three ISA variants (AVX-512 / AVX2+FMA / baseline) dispatched at run time, so the one binary runs
 * on whatever host the GPU box has.
 */
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef int64_t Ti;
#define AT(a, i) ((a)[(i) - 1])
#define SIMD_BYTES 64 /* DEFAULT_SIMD_SIZE = CpuId.simdbytes() on AVX-512 */

typedef double vd __attribute__((vector_size(SIMD_BYTES)));
typedef float vf __attribute__((vector_size(SIMD_BYTES)));
/* unaligned views for vload (one vmovupd / vmovups) */
typedef double vd_u __attribute__((vector_size(SIMD_BYTES), aligned(1), may_alias));
typedef float vf_u __attribute__((vector_size(SIMD_BYTES), aligned(1), may_alias));

/* Compiled three times (AVX-512 / AVX2+FMA / baseline); the exported entry points dispatch on the
 * host CPU (__builtin_cpu_supports). */
#define TGT_V4 __attribute__((target("avx512f,avx512dq,avx512vl,avx2,fma,bmi2")))
#define TGT_V3 __attribute__((target("avx2,fma,bmi2")))
#define TGT_V0

/* Vec{$w} with $w = NV * Δw lanes: NV vector registers.  NV = cld(w, Δw) (bucket (1, Δw, 2Δw, ...));
 * w == 1 takes the scalar bucket. */
#define DEFINE_T(SUF, T, V, VU, DW, TGT)                                                                      \
    TGT static inline void stripe_t_##SUF(Ti l, const Ti *spl, const Ti *pos, const Ti *idx,          \
                                      const Ti *ofs, const T *val, const T *x, T *y)              \
    {                                                                                              \
        const Ti j = AT(spl, l), w = AT(spl, l + 1) - j;                                           \
        Ti q = AT(ofs, l);                                                                         \
        if (w == 1) {                                                                              \
            T tmp = 0;                                                                             \
            for (Ti Q = AT(pos, l); Q <= AT(pos, l + 1) - 1; Q++, q++)                             \
                tmp += AT(val, q) * AT(x, AT(idx, Q));                                             \
            AT(y, j) = tmp;                                                                        \
            return;                                                                                \
        }                                                                                          \
        const int nv = (int)((w + DW - 1) / DW);                                                   \
        V acc[8];                                                                                  \
        for (int k = 0; k < nv; k++) acc[k] = (V){0};                                              \
        if (nv == 1) {                                                                             \
            V a = (V){0};                                                                          \
            for (Ti Q = AT(pos, l); Q <= AT(pos, l + 1) - 1; Q++, q += w) {                        \
                a += *(const VU *)&AT(val, q) * AT(x, AT(idx, Q));                                 \
            }                                                                                      \
            acc[0] = a;                                                                            \
        } else {                                                                                   \
            for (Ti Q = AT(pos, l); Q <= AT(pos, l + 1) - 1; Q++, q += w) {                        \
                const T xv = AT(x, AT(idx, Q));                                                    \
                for (int k = 0; k < nv; k++) {                                                     \
                    acc[k] += *(const VU *)&AT(val, q + (Ti)k * DW) * xv;                          \
                }                                                                                  \
            }                                                                                      \
        }                                                                                          \
        T lanes[8 * DW];                                                                           \
        memcpy(lanes, acc, sizeof(V) * (size_t)nv);                                                \
        for (Ti dj = 0; dj < w; dj++) AT(y, j + dj) = lanes[dj];                                   \
    }                                                                                              \
                                                                                                   \
    /* mul!(y, B', x, true, false); nthreads <= 0: all OpenMP threads; chunk = stripes per grab. */ \
    TGT static int mul_t_##SUF(int64_t m, int64_t n, int64_t L, const Ti *spl, const Ti *pos, \
                                      const Ti *idx, const Ti *ofs, const T *val, const T *x,     \
                                      T *y, int nthreads, int64_t chunk)                          \
    {                                                                                              \
        (void)m;                                                                                   \
        (void)n;                                                                                   \
        for (Ti l = 1; l <= L; l++)                                                                \
            if (AT(spl, l + 1) - AT(spl, l) > 8 * DW) return 2; /* widest bucket: 8 vectors */       \
        if (chunk < 1) chunk = 1;                                                                  \
        int64_t next = 1; /* l′ = Atomic{Int}(1)  :169 */                                          \
        _Pragma("omp parallel num_threads(nthreads > 0 ? nthreads : omp_get_max_threads())")      \
        {                                                                                          \
            for (;;) {                                                                             \
                const int64_t l0 = __atomic_fetch_add(&next, chunk, __ATOMIC_RELAXED);             \
                if (l0 > L) break;                                                                 \
                const int64_t l1 = l0 + chunk - 1 < L ? l0 + chunk - 1 : L;                        \
                for (int64_t l = l0; l <= l1; l++) stripe_t_##SUF(l, spl, pos, idx, ofs, val, x, y); \
            }                                                                                      \
        }                                                                                          \
        return 0;                                                                                  \
    }                                                                                              \
                                                                                                   \
    /* mul!(y, B, x, true, false): serial, like the reference (multiply_1DVBC.jl:62-71). */        \
    TGT static int mul_##SUF(int64_t m, int64_t n, int64_t L, const Ti *spl, const Ti *pos,  \
                                    const Ti *idx, const Ti *ofs, const T *val, const T *x, T *y)  \
    {                                                                                              \
        (void)n;                                                                                   \
        memset(y, 0, sizeof(T) * (size_t)m); /* fill!(y, zero)  :51-53 */                          \
        for (Ti l = 1; l <= L; l++) {                                                              \
            const Ti j = AT(spl, l), w = AT(spl, l + 1) - j;                                       \
            Ti q = AT(ofs, l);                                                                     \
            const int nv = (int)((w + DW - 1) / DW);                                               \
            if (nv > 8) return 2;                                                                  \
            if (w == 1) {                                                                          \
                const T t = AT(x, j);                                                              \
                for (Ti Q = AT(pos, l); Q <= AT(pos, l + 1) - 1; Q++, q++)                         \
                    AT(y, AT(idx, Q)) += AT(val, q) * t;                                           \
                continue;                                                                          \
            }                                                                                      \
            T xs[8 * DW];                                                                          \
            memset(xs, 0, sizeof(xs));                                                             \
            for (Ti dj = 0; dj < w; dj++) xs[dj] = AT(x, j + dj); /* zero-padded slice  :27 */     \
            V tmp[8];                                                                              \
            memcpy(tmp, xs, sizeof(V) * (size_t)nv);                                               \
            for (Ti Q = AT(pos, l); Q <= AT(pos, l + 1) - 1; Q++, q += w) {                        \
                V s = (V){0};                                                                      \
                for (int k = 0; k < nv; k++) {                                                     \
                    s += *(const VU *)&AT(val, q + (Ti)k * DW) * tmp[k];                           \
                }                                                                                  \
                T h = 0;                                                                           \
                for (int e = 0; e < DW; e++) h += s[e]; /* sum(Vec)  :34 */                        \
                AT(y, AT(idx, Q)) += h;                                                            \
            }                                                                                      \
        }                                                                                          \
        return 0;                                                                                  \
    }                                                                                              \
                                                                                                   \
    /* TrSpMV!(y, A, x): serial row dots over the CSC columns (TrSpMV.jl:1-20). */                  \
    TGT static int trspmv_##SUF(int64_t m, int64_t n, const Ti *colptr, const Ti *rowval,         \
                                 const T *nzval, const T *x, T *y)                                 \
    {                                                                                              \
        (void)m;                                                                                   \
        for (Ti i = 1; i <= n; i++) {                                                              \
            T tmp = 0;                                                                             \
            for (Ti p = AT(colptr, i); p <= AT(colptr, i + 1) - 1; p++)                            \
                tmp += AT(nzval, p) * AT(x, AT(rowval, p));                                        \
            AT(y, i) = tmp;                                                                        \
        }                                                                                          \
        return 0;                                                                                  \
    }

DEFINE_T(f64_v4, double, vd, vd_u, 8, TGT_V4)
DEFINE_T(f64_v3, double, vd, vd_u, 8, TGT_V3)
DEFINE_T(f64_v0, double, vd, vd_u, 8, TGT_V0)
DEFINE_T(f32_v4, float, vf, vf_u, 16, TGT_V4)
DEFINE_T(f32_v3, float, vf, vf_u, 16, TGT_V3)
DEFINE_T(f32_v0, float, vf, vf_u, 16, TGT_V0)

/* 4: AVX-512, 3: AVX2 + FMA, 0: baseline x86-64 */
int simd_isa(void)
{
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") && __builtin_cpu_supports("avx512vl"))
        return 4;
    if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return 3;
    return 0;
}

#define DISPATCH(SUF, T)                                                                             \
    int simd_1dvbc_mul_t_##SUF(int64_t m, int64_t n, int64_t L, const Ti *spl, const Ti *pos,        \
                               const Ti *idx, const Ti *ofs, const T *val, const T *x, T *y,        \
                               int nthreads, int64_t chunk)                                        \
    {                                                                                              \
        const int isa = simd_isa();                                                                \
        return isa == 4 ? mul_t_##SUF##_v4(m, n, L, spl, pos, idx, ofs, val, x, y, nthreads, chunk) \
             : isa == 3 ? mul_t_##SUF##_v3(m, n, L, spl, pos, idx, ofs, val, x, y, nthreads, chunk) \
                        : mul_t_##SUF##_v0(m, n, L, spl, pos, idx, ofs, val, x, y, nthreads, chunk); \
    }                                                                                              \
    int simd_1dvbc_mul_##SUF(int64_t m, int64_t n, int64_t L, const Ti *spl, const Ti *pos,          \
                             const Ti *idx, const Ti *ofs, const T *val, const T *x, T *y)          \
    {                                                                                              \
        const int isa = simd_isa();                                                                \
        return isa == 4 ? mul_##SUF##_v4(m, n, L, spl, pos, idx, ofs, val, x, y)                   \
             : isa == 3 ? mul_##SUF##_v3(m, n, L, spl, pos, idx, ofs, val, x, y)                   \
                        : mul_##SUF##_v0(m, n, L, spl, pos, idx, ofs, val, x, y);                  \
    }                                                                                              \
    int simd_trspmv_##SUF(int64_t m, int64_t n, const Ti *colptr, const Ti *rowval, const T *nzval, \
                          const T *x, T *y)                                                        \
    {                                                                                              \
        const int isa = simd_isa();                                                                \
        return isa == 4 ? trspmv_##SUF##_v4(m, n, colptr, rowval, nzval, x, y)                     \
             : isa == 3 ? trspmv_##SUF##_v3(m, n, colptr, rowval, nzval, x, y)                     \
                        : trspmv_##SUF##_v0(m, n, colptr, rowval, nzval, x, y);                    \
    }

DISPATCH(f64, double)
DISPATCH(f32, float)

int simd_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
