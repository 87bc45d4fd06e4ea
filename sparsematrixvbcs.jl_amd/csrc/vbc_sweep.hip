// gfx950 row-swept SpMV kernel for mul!(y, B', x) on inputs without x locality.
//
// multiply_1DVBC.jl:90-134 folds each stripe's stored rows in row order: y[j:j+w-1] = sum over the
// stripe's rows i of val_row * x[i].  When the rows of neighbouring stripes are unrelated (the
// reference's own VBR generator, costs.jl:63-83, draws them uniformly) every x gather of the slotted
// or merge kernels is a random line fetch from an x far larger than L2, and the product runs at the
// random-access rate of the memory system, not at the stream rate.
//
// The swept layout reorders the work, not the arithmetic.  A wave owns a *tile* of S consecutive
// stripes whose w-wide accumulators sit in LDS (kSweepTileBytes per wave).  The tile's stored rows
// are sorted by x row and packed into 64-lane *steps*, each lane one stored row (gather index, stripe
// within the tile, w values); no stripe occurs twice in a step, so a step's LDS read-modify-writes
// never collide, and a stripe's rows stay in ascending row order across steps -- the per-stripe
// summation order of the reference.  Every resident wave therefore walks x from front to back at
// about the same pace: at any moment the grid's gathers fall into a narrow window of x that stays
// in L2 and each x line comes from HBM / MALL about once per XCD instead of once per gather.
// After its last step the wave writes y for its stripes once (alpha, beta applied there).
#include <hip/hip_runtime.h>

#include "vbc_kernels.h"

namespace vbc {

// One stored row of W_ values (16-B loads when the row is a multiple of 16 B, 8-B / scalar otherwise).
template <typename T, int W_>
__device__ __forceinline__ void ld_row(gptr<const T> p, T (&r)[W_])
{
    constexpr int B = W_ * (int)sizeof(T);
    if constexpr (B % 16 == 0) {
        constexpr int E = 16 / (int)sizeof(T);
        typedef T vt __attribute__((ext_vector_type(E)));
#pragma unroll
        for (int i = 0; i < W_ / E; i++) {
            const vt t = __builtin_nontemporal_load((gptr<const vt>)p + i);
#pragma unroll
            for (int e = 0; e < E; e++) r[i * E + e] = t[e];
        }
    } else if constexpr (sizeof(T) == 4 && B % 8 == 0) {
        typedef T vt __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int i = 0; i < W_ / 2; i++) {
            const vt t = __builtin_nontemporal_load((gptr<const vt>)p + i);
            r[2 * i] = t[0];
            r[2 * i + 1] = t[1];
        }
    } else {
#pragma unroll
        for (int e = 0; e < W_; e++) r[e] = __builtin_nontemporal_load(p + e);
    }
}

// U steps per pipeline stage; loads are unconditional (steps past the tile re-read its last step and
// are never folded), as in the slotted kernel.  DIAG (ablations, tools/ab.py only): 1 = gathers
// confined to a 1 MB window of x, 2 = no LDS fold (products summed in registers, one LDS store).
// KIND 0 (B'x): a lane gathers x[row] and folds its w products into its stripe's w accumulators.
// KIND 1 (Bx): a lane gathers the w-wide slice x[j ...] of its block's stripe and adds the block's
// dot product to its output row's accumulator -- per row the blocks come in stripe order, as in the
// reference's serial stripe loop (multiply_1DVBC.jl:62-71).
// PK (SweepBin::packed): one 32-bit key per entry = PAD | segment << lbits | (gather index - the step's
// base); the base is a scalar load per step.
template <typename T, int KIND, int W_, int U, int DIAG, bool PK>
__device__ __forceinline__ void run_sweep(const SweepBin &b, int t, int lane, const T *__restrict__ x,
                                          T *__restrict__ y, T alpha, T beta, bool rd, T *acc)
{
    constexpr int OW = KIND == 0 ? W_ : 1;  // accumulators per segment
    constexpr int XV = KIND == 0 ? 1 : W_;  // x values per entry
    const int s0 = t * b.S;
    const int ns = min(b.S, b.nseg - s0);
    const int nel = ns * OW;
    for (int i = lane; i < nel; i += 64) acc[i] = T(0);
    const int S0 = G(b.tstep)[t], S1 = G(b.tstep)[t + 1];
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const uint16_t> loc = G(b.loc);
    typedef __attribute__((address_space(4))) const uint32_t *cptr;  // scalar (constant) loads
    const cptr sbase = (cptr)b.sbase;
    const int lb = b.lbits;
    const uint32_t dmask = (1u << lb) - 1u;
    const gptr<const T> xg = G(x);
    // Three-phase software pipeline per half-iteration: values of stage i+1, gathers of stage i+1
    // (their keys arrived a half earlier), keys of stage i+2, then the fold of stage i -- so the gather
    // round trip of a stage overlaps the value stream of the next instead of following its key load.
    auto loadk = [&](int s, uint32_t (&kk)[U], uint32_t (&ll)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t p = (size_t)min(s + u, S1 - 1) * 64 + lane;
            kk[u] = __builtin_nontemporal_load(key + p);
            if constexpr (PK) ll[u] = sbase[min(s + u, S1 - 1)];
            else ll[u] = __builtin_nontemporal_load(loc + p);
        }
    };
    auto loadv = [&](int s, T (&v)[U][W_]) {
#pragma unroll
        for (int u = 0; u < U; u++) ld_row<T, W_>(val + ((size_t)min(s + u, S1 - 1) * 64 + lane) * W_, v[u]);
    };
    auto gather = [&](const uint32_t (&kk)[U], const uint32_t (&ll)[U], T (&xv)[U][XV], uint32_t (&fl)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t gi = (PK ? ll[u] + (kk[u] & dmask) : kk[u] & kSlotIdx) & (DIAG == 1 ? 0x1FFFFu : kSlotIdx);
#pragma unroll
            for (int e = 0; e < XV; e++) xv[u][e] = xg[gi + e];
            fl[u] = PK ? (((kk[u] & ~kPad) >> lb) | (kk[u] & kPad)) : (ll[u] | (kk[u] & kPad));
            // materialise fl here: otherwise the compiler sinks it past the next key loads, keeps the
            // old keys alive across them, and the register copies at the back edge cost a vmcnt(0)
            // drain per iteration
            asm volatile("" : "+v"(fl[u]));
        }
    };
    T racc = T(0);
    auto fold = [&](int s, const T (&v)[U][W_], const T (&xv)[U][XV], const uint32_t (&fl)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (s + u < S1 && !(fl[u] & kPad)) {
                if constexpr (DIAG == 2) {
#pragma unroll
                    for (int e = 0; e < W_; e++) racc = fmadd(v[u][e], xv[u][KIND == 0 ? 0 : e], racc + T(fl[u]));
                } else if constexpr (KIND == 0) {
                    T *a = acc + fl[u] * W_;
#pragma unroll
                    for (int e = 0; e < W_; e++) a[e] = fmadd(v[u][e], xv[u][0], a[e]);
                } else {
                    T d = v[u][0] * xv[u][0];
#pragma unroll
                    for (int e = 1; e < W_; e++) d = fmadd(v[u][e], xv[u][e], d);
                    acc[fl[u]] += d;
                }
            }
        }
    };
    if (S0 < S1) {
        uint32_t kA[U], lA[U], kB[U], lB[U], fA[U], fB[U];
        T vA[U][W_], vB[U][W_], xA[U][XV], xB[U][XV];
        loadk(S0, kA, lA);
        loadv(S0, vA);
        gather(kA, lA, xA, fA);
        loadk(S0 + U, kB, lB);
        for (int s = S0; s < S1; s += 2 * U) {
            loadv(s + U, vB);
            gather(kB, lB, xB, fB);
            loadk(s + 2 * U, kA, lA);
            fold(s, vA, xA, fA);
            loadv(s + 2 * U, vA);
            gather(kA, lA, xA, fA);
            loadk(s + 3 * U, kB, lB);
            fold(s + U, vB, xB, fB);
        }
    }
    if constexpr (DIAG == 2) acc[lane % max(nel, 1)] = racc;
    // y for the tile's segments, written once
    if (b.out_affine && b.out_stride == OW) {
        const gptr<T> yo = G(y) + b.out_base + (int64_t)s0 * OW;
        for (int i = lane; i < nel; i += 64) {
            T q = alpha * acc[i];
            if (rd) q = fmadd(beta, yo[i], q);
            yo[i] = q;
        }
    } else {
        for (int i = lane; i < nel; i += 64) {
            const int sl = i / OW, e = i - sl * OW;
            const int o = b.out_affine ? b.out_base + (s0 + sl) * b.out_stride : G(b.out)[s0 + sl];
            T q = alpha * acc[i];
            if (rd) q = fmadd(beta, G(y)[o + e], q);
            G(y)[o + e] = q;
        }
    }
}

// One wave per workgroup: the workgroup's LDS is exactly the wave's tile (TB bytes), so occupancy is
// LDS / TB waves per CU with no idle partner waves.
template <typename T, int KIND, int TB, int DIAG = 0>
__global__ __launch_bounds__(64) void spmv_sweep(const SweepBin *__restrict__ bins, int nbins, int total_tiles,
                                                 const T *__restrict__ x, T *__restrict__ y, T alpha, T beta, int rd_i)
{
    __shared__ __attribute__((aligned(16))) char lds[TB];
    const int g = (int)blockIdx.x;
    if (g >= total_tiles) return;
    const int lane = threadIdx.x;
    int bi = 0;
    while (bi + 1 < nbins && g >= bins[bi + 1].tile0) bi++;
    const SweepBin &b = bins[bi];
    const int t = g - b.tile0;
    T *acc = reinterpret_cast<T *>(lds);
    const bool rd = rd_i != 0;
    // Steps per stage: ~16 values per lane per buffer whatever the width (w = 4: 4 steps in flight).
    // Twice as many (up to 256 VGPRs; occupancy is set by the LDS tile anyway) measured the same.
#define U(W) (16 / W < 2 ? 2 : 16 / W > 8 ? 8 : 16 / W)
    switch (b.w) {
    case 1: if (b.packed) run_sweep<T, KIND, 1, U(1), DIAG, true>(b, t, lane, x, y, alpha, beta, rd, acc); else run_sweep<T, KIND, 1, U(1), DIAG, false>(b, t, lane, x, y, alpha, beta, rd, acc); break;
    case 2: if (b.packed) run_sweep<T, KIND, 2, U(2), DIAG, true>(b, t, lane, x, y, alpha, beta, rd, acc); else run_sweep<T, KIND, 2, U(2), DIAG, false>(b, t, lane, x, y, alpha, beta, rd, acc); break;
    case 3: if (b.packed) run_sweep<T, KIND, 3, U(3), DIAG, true>(b, t, lane, x, y, alpha, beta, rd, acc); else run_sweep<T, KIND, 3, U(3), DIAG, false>(b, t, lane, x, y, alpha, beta, rd, acc); break;
    case 4: if (b.packed) run_sweep<T, KIND, 4, U(4), DIAG, true>(b, t, lane, x, y, alpha, beta, rd, acc); else run_sweep<T, KIND, 4, U(4), DIAG, false>(b, t, lane, x, y, alpha, beta, rd, acc); break;
    case 5: if (b.packed) run_sweep<T, KIND, 5, U(5), DIAG, true>(b, t, lane, x, y, alpha, beta, rd, acc); else run_sweep<T, KIND, 5, U(5), DIAG, false>(b, t, lane, x, y, alpha, beta, rd, acc); break;
    case 6: if (b.packed) run_sweep<T, KIND, 6, U(6), DIAG, true>(b, t, lane, x, y, alpha, beta, rd, acc); else run_sweep<T, KIND, 6, U(6), DIAG, false>(b, t, lane, x, y, alpha, beta, rd, acc); break;
    case 7: if (b.packed) run_sweep<T, KIND, 7, U(7), DIAG, true>(b, t, lane, x, y, alpha, beta, rd, acc); else run_sweep<T, KIND, 7, U(7), DIAG, false>(b, t, lane, x, y, alpha, beta, rd, acc); break;
    case 8: if (b.packed) run_sweep<T, KIND, 8, U(8), DIAG, true>(b, t, lane, x, y, alpha, beta, rd, acc); else run_sweep<T, KIND, 8, U(8), DIAG, false>(b, t, lane, x, y, alpha, beta, rd, acc); break;
    default: break;
    }
#undef U
}

template <typename T, int KIND, int TB, int DIAG = 0>
static void launch_t(const SweepBin *d_bins, int nbins, int total_tiles, const void *x, void *y, double alpha,
                     double beta, bool rd, hipStream_t s)
{
    hipLaunchKernelGGL((spmv_sweep<T, KIND, TB, DIAG>), dim3(total_tiles), dim3(64), 0, s, d_bins, nbins, total_tiles,
                       static_cast<const T *>(x), static_cast<T *>(y), (T)alpha, (T)beta, (int)rd);
}

template <typename T, int KIND>
static void launch_any(const SweepBin *d_bins, int nbins, int total_tiles, int tile_bytes, int diag, const void *x,
                       void *y, double alpha, double beta, bool rd, hipStream_t s)
{
#ifdef VBC_ABLATION
    if constexpr (sizeof(T) == 8 && KIND == 0) {  // ablations (the VBC_ABLATION build only)
        if (diag == 1 && tile_bytes == 2 * kSweepTileBytes) return launch_t<T, KIND, 2 * kSweepTileBytes, 1>(d_bins, nbins, total_tiles, x, y, alpha, beta, rd, s);
        if (diag == 2 && tile_bytes == 2 * kSweepTileBytes) return launch_t<T, KIND, 2 * kSweepTileBytes, 2>(d_bins, nbins, total_tiles, x, y, alpha, beta, rd, s);
    }
#else
    (void)diag;
#endif
    if (tile_bytes >= 4 * kSweepTileBytes) launch_t<T, KIND, 4 * kSweepTileBytes>(d_bins, nbins, total_tiles, x, y, alpha, beta, rd, s);
    else if (tile_bytes >= 2 * kSweepTileBytes) launch_t<T, KIND, 2 * kSweepTileBytes>(d_bins, nbins, total_tiles, x, y, alpha, beta, rd, s);
    else launch_t<T, KIND, kSweepTileBytes>(d_bins, nbins, total_tiles, x, y, alpha, beta, rd, s);
}

int launch_sweep(int esz, int kind, const SweepBin *d_bins, int nbins, int total_tiles, int tile_bytes, int diag,
                 const void *x, void *y, double alpha, double beta, bool rd, hipStream_t stream)
{
    if (total_tiles <= 0) return hipSuccess;
#define VBC_SWEEP_ARGS d_bins, nbins, total_tiles, tile_bytes, diag, x, y, alpha, beta, rd, stream
    if (esz == 8) { if (kind == 0) launch_any<double, 0>(VBC_SWEEP_ARGS); else launch_any<double, 1>(VBC_SWEEP_ARGS); }
    else { if (kind == 0) launch_any<float, 0>(VBC_SWEEP_ARGS); else launch_any<float, 1>(VBC_SWEEP_ARGS); }
#undef VBC_SWEEP_ARGS
    return hipGetLastError();
}

}  // namespace vbc
