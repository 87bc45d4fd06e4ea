// gfx950 multi-RHS transposed product for SMALL dense tiles, one tile at a time (device code).
//
// Y = alpha * B' X + beta * Y for up to 16 right-hand sides per launch, for stripes of width w <= 4 whose
// stored rows come in tiles of u <= 4 consecutive x rows: the u x w blocks of a SparseMatrixVBC
// (constructors_VBC.jl:95-105, a 3D stiffness operator's 3 x 3 node tiles) or a 1DVBC's node runs.
// The reference's per-stripe loop (multiply_VBC.jl:93-147, `_VBR_mul!`) walks a stripe's blocks in stored
// order and, per block row Δi, adds val[q + wΔi : ...] * x[i + Δi] into the w-wide accumulator (:131); per
// right-hand side that is the same fma chain over (block, Δi), which this kernel keeps -- so every column
// equals the reference's column product bit for bit.
//
// The unit of work is the TILE, not the stored row (the MFMA panel of vbc_panel.h pays a key, a value
// row and a 64-B X gather per stored row and puts 3 of its 16 M rows to use on 3 x 3 tiles):
//   * a wave is 4 rows of 16 lanes; 16-lane row g walks its own *stream* -- a run of consecutive stripes
//     of the range -- one tile per step; lane j of the row owns right-hand side j, so the tile's u x 16
//     block of X (u contiguous 64-B rows of a row-major X with 16 RHS) is u coalesced dword loads;
//   * per tile ONE 32-bit key: the first x row of the tile slot, the present-row mask (bits 26..29: a
//     1DVBC run with a hole, or u < the slot height), VALID and LAST (the stripe's last tile);
//   * a stream's tiles and values are contiguous (stream-major inside the range), so a row loads NBT
//     tiles' values with ceil(NBT * u * w / 64) 16-B loads per lane and each lane takes the value it
//     needs from lane f of its row with a DPP row_newbcast (v_mov_b32_dpp row_newbcast:f);
//   * a LAST tile closes the row's stripe: its w x 16 sums go to the wave's LDS stage at the stripe's slot
//     (LDS only -- no store interrupts the vector-memory pipeline) and the range's outputs are written as
//     one contiguous run after the loop.
// Software pipeline: the keys run two batches ahead, the values and X gathers one batch ahead of the fold.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "vbc_kernels.h"
#include "vbc_panel.h"

namespace vbc {

constexpr uint32_t kTileLast = 0x80000000u;
constexpr uint32_t kTileValid = 0x40000000u;
constexpr int kTileMaskShift = 26;           // bits 26..29: rows of the slot the tile stores
constexpr uint32_t kTileRow = 0x00FFFFFFu;   // first x row of the tile slot (< 2^24 - 1); all ones: no tile
                                             // (an invalid key's row times the row stride lies past X)
constexpr int kTileStageBytes = 8192;        // largest LDS output stage per wave (the range's w x 16 sums per stripe)
constexpr int kTileStripes = 32;             // default stripes per range (c5-mesh 8 / 16 / 32: 338 / 327 / 298 us)
constexpr int kTileBatch = 8;                // default tiles per stream per pipeline stage (4 or 8: one key load per two)

// One width bucket of the tile layout (one launch per 16 right-hand sides).
struct TileBin {
    int32_t w;            // stripe width (1..4)
    int32_t ub;           // rows per tile slot (1..4)
    int32_t nranges;      // ranges = waves
    int32_t masku;        // some tile stores fewer rows than its slot (the kernel masks those x rows)
    int32_t out_affine;   // out[s] == out_base + s * out_stride
    int32_t out_base;
    int32_t out_stride;
    int32_t nbt;          // tiles per stream per pipeline stage (the kernel's NBT; streams padded to 2 NBT)
    int32_t depth;        // register sets of the kernel's pipeline (its D: 2, or 3 in the VBC_ABLATION build)
    int32_t stage_bytes;  // LDS output stage per wave: the most stripes of a range x w x 16 sums (dynamic LDS)
    int32_t diag;         // VBC_TILE_DIAG ablation (the VBC_ABLATION build only; 0 in the product library): 8 no output
                          // stores
    const uint32_t *key;  // per range: 4 streams x len keys, stream-major (+ over-read padding)
    const void *val;      // per range: 4 streams x len x (ub * w) values (+ padding)
    const int32_t *rinfo; // per range: {first tile slot, len, first stripe, stripes, stream 1..3 first stripe, 0}
    const int32_t *out;   // per stripe: first y column
};

// v from lane N of each 16-lane row (DPP row_newbcast, gfx90a+)
template <int N>
__device__ __forceinline__ int row_bcast_i(int v)
{
    return __builtin_amdgcn_mov_dpp(v, 0x150 + N, 0xF, 0xF, true);
}
__device__ __forceinline__ int row_bcast_rt(int v, int n)
{
    switch (n & 15) {
    case 0: return row_bcast_i<0>(v);
    case 1: return row_bcast_i<1>(v);
    case 2: return row_bcast_i<2>(v);
    case 3: return row_bcast_i<3>(v);
    case 4: return row_bcast_i<4>(v);
    case 5: return row_bcast_i<5>(v);
    case 6: return row_bcast_i<6>(v);
    case 7: return row_bcast_i<7>(v);
    case 8: return row_bcast_i<8>(v);
    case 9: return row_bcast_i<9>(v);
    case 10: return row_bcast_i<10>(v);
    case 11: return row_bcast_i<11>(v);
    case 12: return row_bcast_i<12>(v);
    case 13: return row_bcast_i<13>(v);
    case 14: return row_bcast_i<14>(v);
    default: return row_bcast_i<15>(v);
    }
}
template <typename T>
__device__ __forceinline__ T row_bcast(T v, int n)
{
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, row_bcast_rt(__builtin_bit_cast(int, v), n));
    } else {
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = (uint32_t)row_bcast_rt((int)(uint32_t)u, n);
        const uint32_t hi = (uint32_t)row_bcast_rt((int)(uint32_t)(u >> 32), n);
        return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
    }
}

// acc += (v from lane N of the row) * x in ONE instruction: v_fmac_f32 with a DPP row_newbcast source (the
// compiler keeps a separate v_mov_b32_dpp).  v is always a register a vector-memory load wrote (the tile's
// values), never a VALU result, so the DPP read-after-VALU-write hazard cannot arise; the checker in
// tools/isa_check.py verifies that in the built ISA.
template <int N>
__device__ __forceinline__ void fmac_bcast(float &acc, float v, float x)
{
    asm("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(v), "v"(x), "n"(N));
}
template <typename T>
__device__ __forceinline__ void fmac_bcast_rt(T &acc, T v, T x, int n)
{
    if constexpr (sizeof(T) == 4) {
        switch (n & 15) {
        case 0: fmac_bcast<0>(acc, v, x); break;
        case 1: fmac_bcast<1>(acc, v, x); break;
        case 2: fmac_bcast<2>(acc, v, x); break;
        case 3: fmac_bcast<3>(acc, v, x); break;
        case 4: fmac_bcast<4>(acc, v, x); break;
        case 5: fmac_bcast<5>(acc, v, x); break;
        case 6: fmac_bcast<6>(acc, v, x); break;
        case 7: fmac_bcast<7>(acc, v, x); break;
        case 8: fmac_bcast<8>(acc, v, x); break;
        case 9: fmac_bcast<9>(acc, v, x); break;
        case 10: fmac_bcast<10>(acc, v, x); break;
        case 11: fmac_bcast<11>(acc, v, x); break;
        case 12: fmac_bcast<12>(acc, v, x); break;
        case 13: fmac_bcast<13>(acc, v, x); break;
        case 14: fmac_bcast<14>(acc, v, x); break;
        default: fmac_bcast<15>(acc, v, x); break;
        }
    } else {
        acc = fmadd(row_bcast(v, n), x, acc);
    }
}

// BUF: X addressed by 32-bit buffer offsets (X below 2 GiB; an invalid key reads past the buffer: 0);
// else 64-bit addresses with the value selected to 0.  FAST: the range's outputs are one contiguous run of
// Y (affine stripe map with stride w, Y row-major with 16 contiguous right-hand sides): 16-B stores.
// D (round 6): register sets of the software pipeline.  D = 2 ping-pong (keys a pair of batches ahead, one
// load per two batches); D >= 3 a ring of D sets -- batch b's values and X gathers are issued D - 1 folds
// before batch b is folded, the next D batches' keys one whole ring ahead -- so a wave keeps D - 1 batches
// of gathers in flight instead of one (the kernel is bound by the memory latency per wave);
// streams are then padded to whole batches and a fold past a stream's end is skipped (uniform test).
template <typename T, int UB, int W, int NBT, bool MASKU, bool BUF, int D = 2>
__global__ __launch_bounds__(kBlockThreads) void spmm_tiles(const TileBin b, const T *__restrict__ X, int64_t sxr,
                                                            int64_t sxc, uint32_t xbytes, T *__restrict__ Y, int64_t syr,
                                                            int64_t syc, int nrhs, T alpha, T beta, int rd_i, int fast)
{
    constexpr int TV = UB * W;               // values per tile slot
    constexpr int EPL = 16 / (int)sizeof(T); // elements per lane per 16-B value load
    constexpr int PER = 16 * EPL;            // elements per value load per 16-lane row
    constexpr int NV = (NBT * TV + PER - 1) / PER;
    typedef T tv __attribute__((ext_vector_type(EPL)));
    extern __shared__ __attribute__((aligned(16))) char tile_stage[];  // kWavesPerBlock x b.stage_bytes
    const int wv = threadIdx.x >> 6;
    const int blk = xcd_block(blockIdx.x, gridDim.x);
    const int rg = __builtin_amdgcn_readfirstlane((int)(blk * kWavesPerBlock + wv));
    if (rg >= b.nranges) return;
    const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
    const gptr<const int32_t> ri = G(b.rinfo) + (size_t)rg * 8;
    const int tile0 = __builtin_amdgcn_readfirstlane(ri[0]), len = __builtin_amdgcn_readfirstlane(ri[1]);
    const int s0 = __builtin_amdgcn_readfirstlane(ri[2]), ns = __builtin_amdgcn_readfirstlane(ri[3]);
    int sidx = g == 0 ? 0 : ri[3 + g];  // this row's stripe (range-relative)
    const int64_t kb = (int64_t)tile0 + (int64_t)g * len;  // this row's first tile slot
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    constexpr int esz = (int)sizeof(T);
    const int jc = j < nrhs ? j : nrhs - 1;  // right-hand sides past nrhs: a valid column, never stored
    const uint32_t sxr_b = (uint32_t)(sxr * esz), jb = (uint32_t)(jc * sxc * esz);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(X), 0, (int)xbytes, 0x00020000);
    const gptr<const T> xg = G(X);
    T *st = reinterpret_cast<T *>(tile_stage + wv * b.stage_bytes);
    const T zero = T(0);
    T acc[W];
#pragma unroll
    for (int c = 0; c < W; c++) acc[c] = zero;

    // lane j of the row holds the key of step t0 + j, j < 2 NBT (the bin carries padding past its end)
    static_assert(2 * NBT <= 16 && D >= 2, "one key load covers two batches of a 16-lane row");
    auto load_keys = [&](int t0) -> uint32_t { return key[kb + t0 + (j < 2 * NBT ? j : 2 * NBT - 1)]; };
    // The batch's NBT * TV values of the row: the lanes of the last load past them (fp32 3 x 3, NBT = 8: 14 of
    // its 16) read lane 0's address -- a segment the load touches anyway; their registers are never read (the
    // fold's source lanes are < NBT TV).  They used to fetch the next batch's first values, which the
    // non-temporal stream had evicted again by the time that batch loaded them: ~40 % of the value bytes came
    // from HBM twice (c5-mesh FETCH_SIZE 785 -> 639 MB per product, 303 -> 270.5 us)
    auto load_vals = [&](int t0, tv (&V)[NV]) {
        const gptr<const T> p = val + (kb + t0) * TV;
#pragma unroll
        for (int v = 0; v < NV; v++) {
#ifdef VBC_TILE_VALS_ALL  // (A/B build, tools/exp/build_variant.sh: every lane loads its own 16 B)
            const int jj = j;
#else
            const int jj = v * PER + j * EPL < NBT * TV ? j : 0;
#endif
            V[v] = __builtin_nontemporal_load((gptr<const tv>)(p + v * PER + jj * EPL));
        }
    };
    auto load_x = [&](uint32_t K, int k0, T (&xs)[NBT][UB]) {
#pragma unroll
        for (int s = 0; s < NBT; s++) {
            const uint32_t ks = (uint32_t)row_bcast_rt((int)K, k0 + s);
            const bool ok = (ks & kTileValid) != 0;
            if constexpr (BUF) {
                // v_mad_u32_u24 reads the key's low 24 bits (the row): an invalid key's all-ones row lands
                // past X (the launcher guarantees it), whose buffer loads return 0 -- no select
                const uint32_t xo = __umul24(ks, sxr_b) + jb;
#pragma unroll
                for (int r = 0; r < UB; r++) xs[s][r] = buf_load<T>(xrs, xo, (uint32_t)r * sxr_b);
            } else {
                const int64_t xr = ok ? (int64_t)(ks & kTileRow) * sxr + (int64_t)jc * sxc : 0;
#pragma unroll
                for (int r = 0; r < UB; r++) {
                    // a slot row the tile does not store may lie past X: read row 0 of the slot instead
                    const bool has = !MASKU || ((ks >> (kTileMaskShift + r)) & 1);
                    const T t = xg[xr + (has ? (int64_t)r * sxr : 0)];
                    xs[s][r] = ok ? t : zero;
                }
            }
        }
    };
    // per key pair: bit 16 g + k of `lastm` = LAST of step k of row g (lanes k >= 2 NBT hold copies)
    auto fold = [&](int t0, uint32_t K, uint64_t lastm, int k0, const tv (&V)[NV], const T (&xs)[NBT][UB]) {
#pragma unroll
        for (int s = 0; s < NBT; s++) {
            // (every stream is padded to a whole number of key pairs: no step past its end)
#pragma unroll
            for (int r = 0; r < UB; r++) {
                T xr = xs[s][r];
                // a slot row the tile does not store: x taken as 0 (its values are 0), so a non-finite x
                // of a row the stripe does not store never reaches it, as in the reference
                if constexpr (MASKU) {
                    const uint32_t ks = (uint32_t)row_bcast_rt((int)K, k0 + s);
                    xr = ((ks >> (kTileMaskShift + r)) & 1) ? xr : zero;
                }
#pragma unroll
                for (int c = 0; c < W; c++) {
                    const int f = s * TV + r * W + c;  // value (r, c) of step s: lane (f % PER) / EPL of the row
                    fmac_bcast_rt(acc[c], V[f / PER][f % EPL], xr, (f % PER) / EPL);
                }
            }
            // a stripe of some row ends at this step (uniform test of the pair's ballot)
            if ((lastm >> (k0 + s)) & 0x0001000100010001ull) {
                const bool last = ((lastm >> (16 * g + k0 + s)) & 1) != 0;
                if (last) {
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        st[(sidx * W + c) * 16 + j] = acc[c];
                        acc[c] = zero;
                    }
                }
                sidx += last ? 1 : 0;
            }
        }
    };

    if constexpr (D == 2) {
        // Two register sets in ping-pong (copying a set would wait for its loads): while batch b is folded
        // from one set, batch b + 1's values and X gathers fill the other.  One key load covers two batches
        // (lane j of the row: step t0 + j), issued a pair ahead; the pair's register is copied only once its
        // keys have been consumed by the X gathers.
        uint32_t KA = load_keys(0);
        tv V0[NV], V1[NV];
        T X0[NBT][UB], X1[NBT][UB];
        load_vals(0, V0);
        load_x(KA, 0, X0);
        // (sched_barrier: the fold's DPP reads of a set must not be hoisted above the other set's loads,
        // which would make those loads wait for this set's data)
        for (int t0 = 0; t0 < len; t0 += 2 * NBT) {
            const uint32_t KB = load_keys(t0 + 2 * NBT);
            load_vals(t0 + NBT, V1);
            load_x(KA, NBT, X1);
            const uint64_t lastm = __builtin_amdgcn_ballot_w64((KA & kTileLast) != 0);
            __builtin_amdgcn_sched_barrier(0);
            fold(t0, KA, lastm, 0, V0, X0);
            __builtin_amdgcn_sched_barrier(0);
            load_vals(t0 + 2 * NBT, V0);
            load_x(KB, 0, X0);
            __builtin_amdgcn_sched_barrier(0);
            fold(t0 + NBT, KA, lastm, NBT, V1, X1);
            __builtin_amdgcn_sched_barrier(0);
            KA = KB;
        }
    } else {
        // A ring of D sets.  At step d of an iteration (batch t0 + d NBT folded from set d), the set freed by the
        // previous fold takes batch t0 + (d + D - 1) NBT, whose key is K[D - 1] for d = 0 and KN[d - 1] after.
        // Keys run a ring further ahead (KNN, issued when the iteration begins, consumed by the next one's
        // gathers), so no gather waits for a key load issued less than D folds earlier.  Lane j of a row holds
        // the key of step j of its batch (j < NBT).  Loads are unconditional (a load inside a branch would make
        // the compiler wait for every load in flight); a fold past the stream's end is skipped.
        auto load_keys1 = [&](int t0) -> uint32_t { return key[kb + t0 + (j < NBT ? j : NBT - 1)]; };
        uint32_t K[D], KN[D], KNN[D];
        tv V[D][NV];
        T Xs[D][NBT][UB];
#pragma unroll
        for (int d = 0; d < D; d++) {
            K[d] = load_keys1(d * NBT);
            KN[d] = load_keys1((D + d) * NBT);
        }
#pragma unroll
        for (int d = 0; d < D - 1; d++) {
            load_vals(d * NBT, V[d]);
            load_x(K[d], 0, Xs[d]);
        }
        for (int t0 = 0; t0 < len; t0 += D * NBT) {
#pragma unroll
            for (int d = 0; d < D; d++) KNN[d] = load_keys1(t0 + (2 * D + d) * NBT);
#pragma unroll
            for (int d = 0; d < D; d++) {
                const int e = (d + D - 1) % D;
                load_vals(t0 + (d + D - 1) * NBT, V[e]);
                load_x(d == 0 ? K[D - 1] : KN[d - 1], 0, Xs[e]);
                const uint64_t lastm = __builtin_amdgcn_ballot_w64((K[d] & kTileLast) != 0);
                __builtin_amdgcn_sched_barrier(0);
                if (t0 + d * NBT < len) fold(t0 + d * NBT, K[d], lastm, 0, V[d], Xs[d]);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int d = 0; d < D; d++) {
                K[d] = KN[d];
                KN[d] = KNN[d];
            }
        }
    }
    // the range's outputs (stripes s0 .. s0 + ns - 1, every slot written once) from the LDS stage
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int total = ns * W * 16;
    const bool rd = rd_i != 0;
    if (VBC_ABL(b.diag & 8)) return;  // (diag 8: no output stores -- the VBC_ABLATION build's ablation)
    if (fast == 2) {
        // Y row-major with 16 contiguous right-hand sides, stripes not contiguous columns (a bucket of a matrix
        // with several widths): each stripe's W x 16 block is contiguous -- 16-B pieces, not element stores
        constexpr int PPR = 16 / EPL;
        const gptr<const int32_t> outp = G(b.out) + s0;
        for (int p = lane; p < ns * W * PPR; p += 64) {
            const int i = p / (W * PPR), rem = p - i * (W * PPR);
            gptr<T> yo = G(Y) + (int64_t)outp[i] * 16 + rem * EPL;
            const tv v = *reinterpret_cast<const tv *>(st + i * W * 16 + rem * EPL);
            tv o;
#pragma unroll
            for (int q = 0; q < EPL; q++) o[q] = alpha * v[q];
            if (rd) {
                const tv yo0 = *(gptr<const tv>)yo;
#pragma unroll
                for (int q = 0; q < EPL; q++) o[q] = fmadd(beta, yo0[q], o[q]);
            }
            st_y((gptr<tv>)yo, o, VBC_ABL(b.diag & 16) != 0);
        }
    } else if (fast) {
        gptr<T> yb = G(Y) + ((int64_t)b.out_base + (int64_t)s0 * W) * 16;
        for (int e = lane * EPL; e < total; e += 64 * EPL) {
            tv v = *reinterpret_cast<const tv *>(st + e);
            tv o;
#pragma unroll
            for (int q = 0; q < EPL; q++) o[q] = alpha * v[q];
            if (rd) {
                const tv yo = *(gptr<const tv>)(yb + e);
#pragma unroll
                for (int q = 0; q < EPL; q++) o[q] = fmadd(beta, yo[q], o[q]);
            }
            st_y((gptr<tv>)(yb + e), o, VBC_ABL(b.diag & 16) != 0);
        }
    } else {
        for (int e = lane; e < total; e += 64) {
            const int i = e / (W * 16), rem = e - i * (W * 16), c = rem >> 4, jj = rem & 15;
            if (jj >= nrhs) continue;
            const int64_t col = (b.out_affine ? (int64_t)b.out_base + (int64_t)(s0 + i) * b.out_stride
                                              : (int64_t)G(b.out)[s0 + i]) + c;
            gptr<T> yo = G(Y) + col * syr + (int64_t)jj * syc;
            T o = alpha * st[e];
            if (rd) o = fmadd(beta, *yo, o);
            *yo = o;
        }
    }
}


}  // namespace vbc
