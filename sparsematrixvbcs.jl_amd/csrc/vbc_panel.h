// gfx950 multi-RHS transposed product on matrix cores (device code, included by vbc_device.hip).
//
// Y = alpha * B' X + beta * Y for k right-hand sides (multiply_1DVBC.jl:90-134 and
// multiply_VBC.jl:93-147 applied column by column; the reference itself has no matrix mul!,
// multiply_1DVBC.jl:184-185).  For a stripe l of width w with stored rows r (2D tiles expanded into
// their u rows), Y[cols of l, :] = V_l' X[rows of l, :] is a (w x R_l) * (R_l x k) dense product,
// so the stripe's rows are fed to v_mfma_{f32,f64}_16x16x4 four at a time:
//     A (16 x 4)  = val of 4 stored rows, output column c on the M axis,
//     B (4 x 16)  = the 4 gathered X rows, 16 right-hand sides on the N axis,
//     C (16 x 16) += A B.
// A *panel* packs S = 16/w consecutive stripes of one width bucket onto the 16 M rows (stripe s of
// the panel owns rows s*w .. s*w+w-1), so narrow stripes still fill the accumulator: a row only
// contributes to the M rows of its own stripe (the A operand is masked by the row's stripe index,
// which the wave derives from the HEAD bits of the keys with one ballot per 64 rows).  Each panel's
// rows are padded to a multiple of 4 (sentinel key, zero val), so a 4-row group never straddles two
// panels; at a panel boundary the accumulator is written out (w*S output columns x 16 RHS, 64-B
// rows of Y) and cleared.  A wave owns a contiguous run of whole panels: no carries, no fix-up, and
// a fixed summation order (rows in stored order, one fma per row, MFMA k-order) -- deterministic.
// IEEE: a non-finite X value times a masked-out zero would put NaN into the other stripes of the
// panel, so a batch whose gathered X holds an Inf / NaN is multiplied on the VALU instead (the same
// k-ordered fma chain, so finite results are unchanged) with each row confined to its own stripe.
// X and Y are addressed through (row, column) strides, so row-major and column-major operands take
// the same kernel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace vbc {

// Padding row (no x row: never a valid row, m < 2^31).  Without HEAD it pads a panel to a multiple of
// 4 rows; with HEAD it is the single row of a stripe that stores none (its columns get beta * Y).
constexpr uint32_t kPanelSentinel = 0x7FFFFFFFu;

// One width bucket of the panel layout.
struct PanelBin {
    int32_t w;          // stripe width (1..16)
    int32_t S;          // stripes per panel = 16 / w
    int32_t range0;     // first range (wave) of this bucket in the launch
    int32_t nranges;
    int32_t out_affine;  // out[s] == out_base + s * out_stride
    int32_t out_base;
    int32_t out_stride;
    int32_t val_bytes;   // bytes of val (incl. tail padding), or 0x7FFFFFFF when >= 2 GiB (no BUF path)
    const uint32_t *key;  // rows (panel-padded): HEAD | x row, or kPanelSentinel
    const void *val;      // rows * w values
    const int32_t *out;   // per stripe: first y column
    const int32_t *rgrp;  // per range + 1: first 4-row group
    const int32_t *rseg;  // per range: first stripe
};

template <typename T>
struct MfmaAcc;
template <>
struct MfmaAcc<float> {
    typedef float v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(float a, float b, v4 c)
    {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // C/D map of the 16x16x4 f32 form: col = lane & 15, row = (lane >> 4) * 4 + reg
    static __device__ __forceinline__ int row(int lane, int reg) { return (lane >> 4) * 4 + reg; }
};
template <>
struct MfmaAcc<double> {
    typedef double v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(double a, double b, v4 c)
    {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // f64 16x16x4: col = lane & 15, row = (lane >> 4) + 4 * reg
    static __device__ __forceinline__ int row(int lane, int reg) { return (lane >> 4) + 4 * reg; }
};

__device__ __forceinline__ int panel_out(const PanelBin &b, int seg)
{
    return b.out_affine ? b.out_base + seg * b.out_stride : G(b.out)[seg];
}

// kPanelBatch groups (4 rows each) are loaded before any of them is multiplied: one coalesced key
// load per 64 rows, then every val and X load of the batch in flight together.
#ifndef VBC_PANEL_BATCH
#define VBC_PANEL_BATCH 16
#endif
constexpr int kPanelBatch = VBC_PANEL_BATCH;
#ifndef VBC_PANEL_VAL_AUX
#define VBC_PANEL_VAL_AUX 2  // val is streamed once: nt
#endif
constexpr int kPanelTail = 8 * kPanelBatch;
// Offset of a masked buffer access: at least every num_records used (operands < 2 GiB) and, plus any
// soffset below 2 GiB, still inside 32 bits -- the access is dropped (store) or reads 0 (load).
constexpr uint32_t kOobOff = 0x80000000u;  // padding rows after each bin (batch over-read + key prefetch)

// Raw buffer loads (32-bit offsets, hardware bounds check) for operands below 4 GiB.
// AUX = cache policy bits of the buffer instruction (2 = nt: streamed once, keep the caches for X).
template <typename T, int AUX = 0>
__device__ __forceinline__ T buf_load(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff)
{
    if constexpr (sizeof(T) == 4)
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, AUX));
    else
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, AUX));
}

template <typename T>
__device__ __forceinline__ void buf_store(T v, __amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff);
template <>
__device__ __forceinline__ void buf_store<float>(float v, __amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff)
{
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rs, voff, soff, 0);
}
template <>
__device__ __forceinline__ void buf_store<double>(double v, __amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff)
{
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, voff, soff, 0);
}

// diag (ablation, VBC_PANEL_DIAG; read by the VBC_ABLATION build only, 0 in the product library): 1 VALU path,
// 2 no Y stores, 4 X gathers hit cache, 8 val hits cache.
// BUF: X and the bins' val are addressed by 32-bit offsets through buffer descriptors (the host picks
// it when both, plus the column offsets, stay below 2 GiB); otherwise 64-bit global addresses.
// FAST (with BUF; beta = 0, affine stripe -> column map, Y below 2 GiB): a full panel is written by
// 4*NB buffer stores at per-lane constant offsets plus one uniform panel offset -- no address
// arithmetic, no loads, no branches in the flush.
template <typename T, int NB, bool BUF, bool FAST>
__global__ __launch_bounds__(kBlockThreads) void spmm_panel(const PanelBin *__restrict__ bins, int nbins,
                                                            int total_ranges, const T *__restrict__ X, int64_t sxr,
                                                            int64_t sxc, uint32_t xbytes, T *__restrict__ Y,
                                                            int64_t syr, int64_t syc, uint32_t ybytes, int nrhs,
                                                            T alpha, T beta, int rd_i, int diag)
{
    using M = MfmaAcc<T>;
    typedef typename M::v4 v4;
    __shared__ uint32_t xch[kWavesPerBlock][64][2];  // per wave: {X row offset, stripe-in-panel} of 64 rows
    const int wv = threadIdx.x >> 6;
    const int rg = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWavesPerBlock + wv));
    if (rg >= total_ranges) return;
    int bi = 0;
    while (bi + 1 < nbins && bins[bi + 1].range0 <= rg) bi++;
    const PanelBin b = bins[bi];
    const int r = rg - b.range0;
    const int g0 = __builtin_amdgcn_readfirstlane(b.rgrp[r]), g1 = __builtin_amdgcn_readfirstlane(b.rgrp[r + 1]);
    if (g0 >= g1) return;
    int seg_base = __builtin_amdgcn_readfirstlane(b.rseg[r]);
    const int lane = threadIdx.x & 63;
    const int w = b.w, S = b.S;
    constexpr int esz = (int)sizeof(T);
    // A-operand masking: fp64 masks by address (an out-of-range buffer offset reads 0, saving the
    // select and its registers); fp32 selects after the load (cheaper with many masked lanes).
    constexpr bool kOobMask = sizeof(T) == 8;
    // A operand: M row c = lane & 15 (stripe c / w of the panel, column c % w), k = lane >> 4.
    const int ca = lane & 15, kr = lane >> 4;
    const int sa = ca / w, cola = ca - sa * w;  // sa >= S: unused M row, never matches a stripe
    // B operand / C column: right-hand side j = lane & 15 (columns >= nrhs read a valid column and
    // only feed C columns that are never stored).
    const int j = lane & 15;
    // C rows held by this lane: stripe and column for each of the 4 accumulator registers.
    int cs[4], cc[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int c = M::row(lane, q);
        cs[q] = c / w;
        cc[q] = c - cs[q] * w;
        if (cs[q] >= S) cs[q] = 64;  // unused M row: never stored
    }
    uint32_t jofs[NB];
    int64_t jofs64[NB];
#pragma unroll
    for (int nb = 0; nb < NB; nb++) {
        const int jc = min(nb * 16 + j, nrhs - 1);
        jofs64[nb] = (int64_t)jc * sxc;
        jofs[nb] = (uint32_t)(jofs64[nb] * esz);
    }
    const uint32_t sxr_b = (uint32_t)(sxr * esz);
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const T> xg = G(X);
    gptr<T> yg = G(Y);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(X), 0, (int)xbytes, 0x00020000);
    // the bin's val pointer comes from memory: make its wave-uniformity explicit (no waterfall loop)
    const uint64_t vp = (uint64_t)(uintptr_t)b.val;
    const uint64_t vpu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(vp >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)vp);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)vpu, 0, b.val_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(Y, 0, (int)ybytes, 0x00020000);
    const uint32_t voff_lane = (uint32_t)((kr * w + cola) * esz);  // val offset of this lane's A element in a group
    // FAST flush: per-lane byte offset of C(reg) for right-hand side block 0 within a panel whose first
    // stripe is column out_base + seg_base * out_stride (past Y: the store is dropped)
    uint32_t yoff[4];
    const uint32_t ycol_b = (uint32_t)(16 * syc * esz);  // + per right-hand-side block
    const int32_t ostr = b.out_stride;
#pragma unroll
    for (int q = 0; q < 4; q++)
        yoff[q] = (cs[q] < S && j < nrhs) ? (uint32_t)((((int64_t)cs[q] * ostr + cc[q]) * syr + (int64_t)j * syc) * esz)
                                          : kOobOff;
    const T zero = T(0);

    v4 acc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; nb++) acc[nb] = v4{zero, zero, zero, zero};

    // general flush of the open panel holding `cnt` stripes (any map, beta, 64-bit addresses)
    auto flush_general = [&](int cnt) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (cs[q] < cnt) {
                const int64_t o = panel_out(b, seg_base + cs[q]) + cc[q];
#pragma unroll
                for (int nb = 0; nb < NB; nb++) {
                    const int jj = nb * 16 + j;
                    if (jj < nrhs && !VBC_ABL(diag & 2)) {
                        gptr<T> yo = yg + o * syr + (int64_t)jj * syc;
                        T v = alpha * acc[nb][q];
                        if (rd_i) v = fmadd(beta, *yo, v);
                        *yo = v;
                    }
                }
            }
        }
#pragma unroll
        for (int nb = 0; nb < NB; nb++) acc[nb] = v4{zero, zero, zero, zero};
    };
    // a full panel (S stripes) ends: FAST stores or the general flush
    auto flush_full = [&]() {
        if constexpr (FAST) {
            const uint32_t pb = (uint32_t)((int64_t)(b.out_base + (int64_t)seg_base * ostr) * syr * esz);
            if (!VBC_ABL(diag & 2)) {
#pragma unroll
                for (int nb = 0; nb < NB; nb++) {
                    if (nb * 16 < nrhs) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const uint32_t yo = (nb == 0 || nb * 16 + j < nrhs) ? yoff[q] : kOobOff;
                            buf_store<T>(alpha * acc[nb][q], yrs, yo, pb + (uint32_t)nb * ycol_b);
                        }
                    }
                }
            }
#pragma unroll
            for (int nb = 0; nb < NB; nb++) acc[nb] = v4{zero, zero, zero, zero};
        } else {
            flush_general(S);
        }
        seg_base += S;
    };

    // Loads are unconditional (no divergent branches, so the waitcnt pass keeps them all in flight):
    // the bin arrays carry kPanelTail padding rows, rows past the range are masked by value, and
    // the keys of batch b+1 are prefetched while batch b is multiplied.
    int segc = 0;  // stripes started in this range before the current batch
    uint32_t kraw = __builtin_nontemporal_load(key + (size_t)g0 * 4 + lane);
    for (int gb = g0; gb < g1; gb += kPanelBatch) {
        const int ng = min(kPanelBatch, g1 - gb);
        const uint32_t kv = lane < 4 * ng ? kraw : kPanelSentinel;
        kraw = __builtin_nontemporal_load(key + (size_t)(gb + kPanelBatch) * 4 + lane);
        const uint64_t hm = __ballot((kv & kHead) != 0);
        // per row (lane = row of the batch): X offset, stripe index within its panel, panel starts
        uint64_t fmask;  // bit 4q: a new panel starts at group q (flush the previous one first)
        {
            const bool head = (kv & kHead) != 0;
            const int hc = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u)) +
                           (int)head;
            const int gseg = segc + hc - 1;  // range-relative stripe of this row (ranges start at panels)
            const int rs = gseg - (gseg / S) * S;
            fmask = __ballot(head && rs == 0 && gseg > 0);
            const bool ok = (kv & ~kHead) != kPanelSentinel;
            uint32_t xo = ok ? (kv & ~kHead) * sxr_b : xbytes;  // past X: the buffer load returns 0
            if (VBC_ABL(diag & 4)) xo = ok ? (uint32_t)(lane & 3) * sxr_b : xbytes;  // ablation: X gathers hit cache
            xch[wv][lane][0] = xo;
            xch[wv][lane][1] = (uint32_t)rs;
        }
        segc += (int)__builtin_popcountll(hm);
        T av[kPanelBatch], xv[kPanelBatch][NB];
        uint32_t rsv[kPanelBatch];
#pragma unroll
        for (int q = 0; q < kPanelBatch; q++) {
            const uint32_t xo = xch[wv][4 * q + kr][0];
            rsv[q] = xch[wv][4 * q + kr][1];
            if constexpr (BUF) {
                const uint32_t vo = (!kOobMask || (int)rsv[q] == sa) ? voff_lane + (uint32_t)(q * 4 * w * esz) : kOobOff;
                av[q] = buf_load<T, VBC_PANEL_VAL_AUX>(vrs, vo, VBC_ABL(diag & 8) ? 0u : (uint32_t)((size_t)gb * 4 * w * esz));
#pragma unroll
                for (int nb = 0; nb < NB; nb++) xv[q][nb] = buf_load<T>(xrs, xo + jofs[nb], 0u);
            } else {
                const size_t row = (size_t)(gb + q) * 4 + kr;
                av[q] = __builtin_nontemporal_load(val + row * w + cola);
                const uint32_t rk = (uint32_t)__shfl((int)kv, 4 * q + kr, 64);
                const bool ok = (rk & ~kHead) != kPanelSentinel;
                const int64_t xr = ok ? (int64_t)(rk & ~kHead) * sxr : 0;
#pragma unroll
                for (int nb = 0; nb < NB; nb++) {
                    const T t = xg[xr + jofs64[nb]];
                    xv[q][nb] = ok ? t : zero;
                }
            }
        }
        // an Inf / NaN among the gathered X: x * 0 is NaN exactly for non-finite x (val is folded in
        // too, which keeps its loads ahead of this wait; a non-finite val only costs the VALU path)
        T chk = zero;
#pragma unroll
        for (int q = 0; q < kPanelBatch; q++) {
            chk = fmadd(av[q], zero, chk);
#pragma unroll
            for (int nb = 0; nb < NB; nb++) chk = fmadd(xv[q][nb], zero, chk);
        }
        const int any_bad = __builtin_amdgcn_readfirstlane(__ballot(chk != chk) != 0 || VBC_ABL(diag & 1) ? 1 : 0);
        if (!any_bad) {
#pragma unroll
            for (int q = 0; q < kPanelBatch; q++) {
                if (q < ng) {
                    if (__builtin_expect((fmask >> (4 * q)) & 1, 0)) flush_full();
                    const T a = (BUF && kOobMask) ? av[q] : ((int)rsv[q] == sa ? av[q] : zero);
#pragma unroll
                    for (int nb = 0; nb < NB; nb++) acc[nb] = M::mma(a, xv[q][nb], acc[nb]);
                }
            }
        } else {
            // VALU, one row at a time from memory: row k only feeds the accumulator rows of its own
            // stripe (rare: only batches whose X holds an Inf / NaN)
            for (int q = 0; q < ng; q++) {
                if ((fmask >> (4 * q)) & 1) flush_full();
                for (int k = 0; k < 4; k++) {
                    const uint32_t rk = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)kv, 4 * q + k, 64));
                    if ((rk & ~kHead) == kPanelSentinel) continue;
                    const int rsk = __builtin_amdgcn_readfirstlane((int)xch[wv][4 * q + k][1]);
                    const size_t row = (size_t)(gb + q) * 4 + k;
                    const int64_t xr = (int64_t)(rk & ~kHead) * sxr;
#pragma unroll
                    for (int reg = 0; reg < 4; reg++) {
                        if (cs[reg] != rsk) continue;
                        const T a = val[row * w + cc[reg]];
#pragma unroll
                        for (int nb = 0; nb < NB; nb++) {
                            const int jj = nb * 16 + j;
                            const T xval = jj < nrhs ? xg[xr + (int64_t)jj * sxc] : zero;
                            acc[nb][reg] = fmadd(a, xval, acc[nb][reg]);
                        }
                    }
                }
            }
        }
    }
    flush_general(segc - ((segc - 1) / S) * S);  // the last panel (the bin's last may hold < S stripes)
}

// Y rows of the stripes that store no row (and belong to no panel): beta * Y or 0.
template <typename T>
__global__ __launch_bounds__(kBlockThreads) void fill_rows_mm(const int32_t *__restrict__ fill, int nfill, T *__restrict__ Y,
                                                              int64_t syr, int64_t syc, int nrhs, T beta, int rd_i)
{
    const int64_t i = blockIdx.x * (int64_t)kBlockThreads + threadIdx.x;
    if (i >= (int64_t)nfill * nrhs) return;
    const int f = (int)(i / nrhs), jj = (int)(i - (int64_t)f * nrhs);
    T *yo = Y + (int64_t)fill[f] * syr + (int64_t)jj * syc;
    *yo = rd_i ? beta * *yo : T(0);
}

}  // namespace vbc
