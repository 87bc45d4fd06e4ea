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

// Staged-X form (round 5b; TileBin::staged): one workgroup per CLUSTER of stripes that share block rows
constexpr int kTileXMaxWaves = 8;     // compute waves per cluster workgroup (4 or 8; the persistent kernel: 4)
constexpr int kTileXMaxStreams = 4 * kTileXMaxWaves;
// ints per cluster: {first stripe (out index), stripes, U, xrow offset, 8 x row stride of wave k's stream,
// 32 x first local stripe of stream k, 8 x first tile slot of wave k's segment (row 0), 8 x its length}
constexpr int kXiStride = 4, kXiSidx = kXiStride + kTileXMaxWaves, kXiSeg = kXiSidx + kTileXMaxStreams,
              kXiLen = kXiSeg + kTileXMaxWaves;
constexpr int kTileXInfo = 64;
constexpr uint32_t kTileXEnd = 0x40000000u;  // key bit 30: the last tile of a wave's segment of a cluster
constexpr int kTileXStreams = 16;     // 4 waves x 4 rows of 16 lanes (the persistent kernel's compute waves)
constexpr int kTileXBatch = 8;        // tiles per stream per pipeline stage
constexpr int kTileXDepth = 4;        // stages in flight (keys and values)
constexpr uint32_t kTileXSlot = 0xFFFFu;  // key bits 0..15: the tile's X slot in the cluster's LDS stage
constexpr int64_t kTileXLds = 65536;      // LDS per workgroup: X stage + output stage (4 compute waves)
constexpr int64_t kTileXLds8 = 80 * 1024; // ... 8 compute waves: two workgroups per CU
constexpr int kTileXPieces = 12;          // 16-B X pieces per thread of the staging (U + 1) x ub x 16 elements
constexpr int tile_x_pieces(int nw) { return nw == 8 ? 8 : kTileXPieces; }  // (8 waves: registers for 4 waves / SIMD)
constexpr int kTileXOutPieces = 4;        // 16-B output pieces per thread of the epilogue (stripes x w x 16 elements)

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
    int32_t stage_bytes;  // LDS output stage per wave: the most stripes of a range x w x 16 sums (dynamic LDS)
    int32_t diag;         // VBC_TILE_DIAG ablations (tools/ab.py only): 1 X tiles from 256 rows (cache-resident),
                          // 2 values from the range's first batch (cache-resident)
    const uint32_t *key;  // per range: 4 streams x len keys, stream-major (+ over-read padding)
    const void *val;      // per range: 4 streams x len x (ub * w) values (+ padding)
    const int32_t *rinfo; // per range: {first tile slot, len, first stripe, stripes, stream 1..3 first stripe, 0}
    const int32_t *out;   // per stripe: first y column
    // staged-X form: nranges = clusters (one workgroup each), rinfo = kTileXInfo ints per cluster, key bits
    // 0..15 an X slot of the cluster (slot U: the zero slot of padding), xrow = every cluster's slot base rows
    int32_t staged;
    int32_t xslots;       // largest U + 1 of a cluster (the LDS X stage: xslots x ub x 16 elements)
    const int32_t *xrow;
    int32_t nwaves;       // compute waves per cluster (spmm_tiles_x: 4 or 8; 4 streams each)
    int32_t nwg;          // persistent kernel (spmm_tiles_xp): workgroups, each a sequence of clusters
    const int32_t *wginfo;  // per workgroup: {first cluster, clusters}
    const void *zsrc;     // 16 zero bytes in device memory (the LDS-DMA source of zero pieces)
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
template <typename T, int UB, int W, int NBT, bool MASKU, bool BUF>
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
    static_assert(2 * NBT <= 16, "one key load covers two batches of a 16-lane row");
    auto load_keys = [&](int t0) -> uint32_t { return key[kb + t0 + (j < 2 * NBT ? j : 2 * NBT - 1)]; };
    auto load_vals = [&](int t0, tv (&V)[NV]) {
        const gptr<const T> p = val + (kb + t0) * TV + j * EPL;
#pragma unroll
        for (int v = 0; v < NV; v++) V[v] = __builtin_nontemporal_load((gptr<const tv>)(p + v * PER));
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
    // the range's outputs (stripes s0 .. s0 + ns - 1, every slot written once) from the LDS stage
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int total = ns * W * 16;
    const bool rd = rd_i != 0;
    if (b.diag & 8) return;  // (diag 8: no output stores -- an ablation, tools/ab.py)
    if (fast == 2) {
        // Y row-major with 16 contiguous right-hand sides, stripes not contiguous (a non-natural stripe order,
        // e.g. VBC_TILE_ORDER=1): each stripe's W x 16 block is contiguous -- 16-B pieces, not element stores
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
            *(gptr<tv>)yo = o;
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
            *(gptr<tv>)(yb + e) = o;
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


// The 16-B form (fp32, X row-major with 16 contiguous right-hand sides): the tile's u x 16 block of X is
// u x 64 contiguous bytes, loaded by ONE dwordx4 instruction per step -- lane j = 4 r + q of the row takes
// X[r][4q .. 4q+3] (lanes j >= 4 ub idle) -- instead of u dword loads (measured on gfx950,
// tools/exp/ta_probe.hip: a dword load of 4 x 64-B lines costs the CU 11 cycles of address / data path,
// a dwordx4 of 4 x 192 B 20: the dword form of a 3-row tile is 33).  Lane (r, q) then needs T[r][c], a
// value of its own row r of the tile: three DPP row_newbcast moves per column c, each writing only the
// lanes of bank r (bank_mask = 1 << r; the other banks keep what they hold), put T[r_lane][c] in one
// register, and the lane folds acc[c][k] += T[r][c] * X[r][4q + k] with packed fmas.  The u banks hold
// partial sums per slot row; a LAST tile adds them in the row (DPP row_shl 4 / 8 / 12: ((r0 + r1) + r2)
// + r3) and bank 0 stages the stripe's 16 x w sums.  Each column is the sum over the stripe's tiles of its
// per-slot-row chains -- the reference's products, associated by slot row (within fp32 rounding of the
// reference's single chain, multiply_VBC.jl:131).
template <int N, int BANK>
__device__ __forceinline__ float bank_bcast(float old, float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                                 0x150 + N, 0xF, 1 << BANK, false));
}
template <int BANK>
__device__ __forceinline__ float bank_bcast_rt(float old, float v, int n)
{
    switch (n & 15) {
    case 0: return bank_bcast<0, BANK>(old, v);
    case 1: return bank_bcast<1, BANK>(old, v);
    case 2: return bank_bcast<2, BANK>(old, v);
    case 3: return bank_bcast<3, BANK>(old, v);
    case 4: return bank_bcast<4, BANK>(old, v);
    case 5: return bank_bcast<5, BANK>(old, v);
    case 6: return bank_bcast<6, BANK>(old, v);
    case 7: return bank_bcast<7, BANK>(old, v);
    case 8: return bank_bcast<8, BANK>(old, v);
    case 9: return bank_bcast<9, BANK>(old, v);
    case 10: return bank_bcast<10, BANK>(old, v);
    case 11: return bank_bcast<11, BANK>(old, v);
    case 12: return bank_bcast<12, BANK>(old, v);
    case 13: return bank_bcast<13, BANK>(old, v);
    case 14: return bank_bcast<14, BANK>(old, v);
    default: return bank_bcast<15, BANK>(old, v);
    }
}
template <int R>
__device__ __forceinline__ float bank_bcast_r(float old, float v, int n)
{
    if constexpr (R == 0) return bank_bcast_rt<0>(old, v, n);
    else if constexpr (R == 1) return bank_bcast_rt<1>(old, v, n);
    else if constexpr (R == 2) return bank_bcast_rt<2>(old, v, n);
    else return bank_bcast_rt<3>(old, v, n);
}
// v from lane + N of the row (row_shl:N; lanes past the row's end read 0)
template <int N>
__device__ __forceinline__ float row_shl(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x100 + N, 0xF, 0xF, true));
}

template <int UB, int W, int NBT, bool MASKU>
__global__ __launch_bounds__(kBlockThreads) void spmm_tiles4(const TileBin b, const float *__restrict__ X, int64_t sxr,
                                                             uint32_t xbytes, float *__restrict__ Y, int64_t syr,
                                                             int64_t syc, float alpha, float beta, int rd_i, int fast)
{
    typedef float T;
    constexpr int TV = UB * W;
    constexpr int EPL = 4, PER = 64;
    constexpr int NV = (NBT * TV + PER - 1) / PER;
    typedef float tv __attribute__((ext_vector_type(4)));
    typedef float t2 __attribute__((ext_vector_type(2)));
    extern __shared__ __attribute__((aligned(16))) char tile_stage[];
    const int wv = threadIdx.x >> 6;
    const int blk = xcd_block(blockIdx.x, gridDim.x);
    const int rg = __builtin_amdgcn_readfirstlane((int)(blk * kWavesPerBlock + wv));
    if (rg >= b.nranges) return;
    const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15, rl = j >> 2, q = j & 3;
    const gptr<const int32_t> ri = G(b.rinfo) + (size_t)rg * 8;
    const int tile0 = __builtin_amdgcn_readfirstlane(ri[0]), len = __builtin_amdgcn_readfirstlane(ri[1]);
    const int s0 = __builtin_amdgcn_readfirstlane(ri[2]), ns = __builtin_amdgcn_readfirstlane(ri[3]);
    int sidx = g == 0 ? 0 : ri[3 + g];
    const int64_t kb = (int64_t)tile0 + (int64_t)g * len;
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const uint32_t sxr_b = (uint32_t)(sxr * 4);
    // lane (r, q): bytes r * row + 16 q of the tile's block; idle lanes (r >= ub) read past X: zeros
    const uint32_t lb = rl < UB ? (uint32_t)rl * sxr_b + (uint32_t)q * 16u : 0x80000000u;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(X), 0, (int)xbytes, 0x00020000);
    T *st = reinterpret_cast<T *>(tile_stage + wv * b.stage_bytes);
    t2 acc[W][2];
    float tc[W];  // this step's T[r_lane][c] (kept across steps: a bank only ever needs its own row)
#pragma unroll
    for (int c = 0; c < W; c++) {
        acc[c][0] = acc[c][1] = t2{0.f, 0.f};
        tc[c] = 0.f;
    }

    static_assert(2 * NBT <= 16, "one key load covers two batches of a 16-lane row");
    auto load_keys = [&](int t0) -> uint32_t { return key[kb + t0 + (j < 2 * NBT ? j : 2 * NBT - 1)]; };
    auto load_vals = [&](int t0, tv (&V)[NV]) {
#ifdef VBC_TILE_DIAG_BUILD
        const gptr<const T> p = val + (kb + ((b.diag & 2) ? 0 : t0)) * TV + j * EPL;
#else
        const gptr<const T> p = val + (kb + t0) * TV + j * EPL;
#endif
#pragma unroll
        for (int v = 0; v < NV; v++) V[v] = __builtin_nontemporal_load((gptr<const tv>)(p + v * PER));
    };
    auto load_x = [&](uint32_t K, int k0, tv (&xs)[NBT]) {
#pragma unroll
        for (int s = 0; s < NBT; s++) {
            const uint32_t ks = (uint32_t)row_bcast_rt((int)K, k0 + s);
            // (an invalid key's all-ones 24-bit row lands past X: zeros, see spmm_tiles)
#ifdef VBC_TILE_DIAG_BUILD
            const uint32_t xo = __umul24((b.diag & 1) ? (ks & 0xFFu) : ks, sxr_b) + lb;
#else
            const uint32_t xo = __umul24(ks, sxr_b) + lb;
#endif
            xs[s] = __builtin_bit_cast(tv, __builtin_amdgcn_raw_buffer_load_b128(xrs, xo, 0, 0));
        }
    };
    auto fold = [&](uint32_t K, uint64_t lastm, int k0, const tv (&V)[NV], const tv (&xs)[NBT]) {
#pragma unroll
        for (int s = 0; s < NBT; s++) {
            tv xv = xs[s];
            if constexpr (MASKU) {
                const uint32_t ks = (uint32_t)row_bcast_rt((int)K, k0 + s);
                if (!((ks >> (kTileMaskShift + rl)) & 1)) xv = tv{0.f, 0.f, 0.f, 0.f};
            }
            const t2 x01 = t2{xv[0], xv[1]}, x23 = t2{xv[2], xv[3]};
            // tc[c] = T[r_lane][c]: bank r receives row r's value (r outer: consecutive moves into one
            // register are W apart, past the DPP read-after-write distance).  The banks >= ub keep stale
            // values: their lanes load no X (zeros) and their partial sums are never read.
#pragma unroll
            for (int r = 0; r < UB; r++) {
#pragma unroll
                for (int c = 0; c < W; c++) {
                    const int f = s * TV + r * W + c;
                    if (r == 0) tc[c] = bank_bcast_r<0>(tc[c], V[f / PER][f % EPL], (f % PER) / EPL);
                    else if (r == 1) tc[c] = bank_bcast_r<1>(tc[c], V[f / PER][f % EPL], (f % PER) / EPL);
                    else if (r == 2) tc[c] = bank_bcast_r<2>(tc[c], V[f / PER][f % EPL], (f % PER) / EPL);
                    else tc[c] = bank_bcast_r<3>(tc[c], V[f / PER][f % EPL], (f % PER) / EPL);
                }
            }
#pragma unroll
            for (int c = 0; c < W; c++) {
                const t2 tt = t2{tc[c], tc[c]};
                acc[c][0] = __builtin_elementwise_fma(tt, x01, acc[c][0]);
                acc[c][1] = __builtin_elementwise_fma(tt, x23, acc[c][1]);
            }
            if ((lastm >> (k0 + s)) & 0x0001000100010001ull) {
                const bool last = ((lastm >> (16 * g + k0 + s)) & 1) != 0;
                if (last) {
#ifdef VBC_TILE_REDUCE_DPP
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        float o[4] = {acc[c][0][0], acc[c][0][1], acc[c][1][0], acc[c][1][1]};
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            float v = o[k];
                            if constexpr (UB > 1) v = v + row_shl<4>(o[k]);
                            if constexpr (UB > 2) v = v + row_shl<8>(o[k]);
                            if constexpr (UB > 3) v = v + row_shl<12>(o[k]);
                            o[k] = v;
                        }
                        if (rl == 0) *reinterpret_cast<tv *>(st + (sidx * W + c) * 16 + 4 * q) = tv{o[0], o[1], o[2], o[3]};
                        acc[c][0] = acc[c][1] = t2{0.f, 0.f};
                    }
#else
                    // each slot row's partial sums to the stage: [stripe][r][c][16 right-hand sides]
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        if (rl < UB)
                            *reinterpret_cast<tv *>(st + ((sidx * UB + rl) * W + c) * 16 + 4 * q) =
                                tv{acc[c][0][0], acc[c][0][1], acc[c][1][0], acc[c][1][1]};
                        acc[c][0] = acc[c][1] = t2{0.f, 0.f};
                    }
#endif
                }
                sidx += last ? 1 : 0;
            }
        }
    };

    uint32_t KA = load_keys(0);
    tv V0[NV], V1[NV];
    tv X0[NBT], X1[NBT];
    load_vals(0, V0);
    load_x(KA, 0, X0);
    for (int t0 = 0; t0 < len; t0 += 2 * NBT) {
        const uint32_t KB = load_keys(t0 + 2 * NBT);
        load_vals(t0 + NBT, V1);
        load_x(KA, NBT, X1);
        const uint64_t lastm = __builtin_amdgcn_ballot_w64((KA & kTileLast) != 0);
        __builtin_amdgcn_sched_barrier(0);
        fold(KA, lastm, 0, V0, X0);
        __builtin_amdgcn_sched_barrier(0);
        load_vals(t0 + 2 * NBT, V0);
        load_x(KB, 0, X0);
        __builtin_amdgcn_sched_barrier(0);
        fold(KA, lastm, NBT, V1, X1);
        __builtin_amdgcn_sched_barrier(0);
        KA = KB;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int total = ns * W * 16;
    const bool rd = rd_i != 0;
    // stripe i's sums: ((r0 + r1) + r2) + r3 of its slot rows' partials
    auto staged = [&](int e) -> tv {
        const int i = e / (W * 16), rem = e - i * (W * 16);
#ifdef VBC_TILE_REDUCE_DPP
        return *reinterpret_cast<const tv *>(st + e);
#else
        const T *p = st + i * UB * W * 16 + rem;
        tv v = *reinterpret_cast<const tv *>(p);
#pragma unroll
        for (int r = 1; r < UB; r++) v += *reinterpret_cast<const tv *>(p + r * W * 16);
        return v;
#endif
    };
    if (fast) {
        gptr<T> yb = G(Y) + ((int64_t)b.out_base + (int64_t)s0 * W) * 16;
        for (int e = lane * EPL; e < total; e += 64 * EPL) {
            const tv v = staged(e);
            tv o;
#pragma unroll
            for (int k = 0; k < 4; k++) o[k] = alpha * v[k];
            if (rd) {
                const tv yo = *(gptr<const tv>)(yb + e);
#pragma unroll
                for (int k = 0; k < 4; k++) o[k] = fmadd(beta, yo[k], o[k]);
            }
            *(gptr<tv>)(yb + e) = o;
        }
    } else {
        for (int e = lane * EPL; e < total; e += 64 * EPL) {
            const int i = e / (W * 16), rem = e - i * (W * 16), c = rem >> 4, jj = rem & 15;
            const int64_t col = (b.out_affine ? (int64_t)b.out_base + (int64_t)(s0 + i) * b.out_stride
                                              : (int64_t)G(b.out)[s0 + i]) + c;
            const tv v = staged(e);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                gptr<T> yo = G(Y) + col * syr + (int64_t)(jj + k) * syc;
                T o = alpha * v[k];
                if (rd) o = fmadd(beta, *yo, o);
                *yo = o;
            }
        }
    }
}

// Staged-X form (round 5b, TileBin::staged).  The unit of scheduling is a CLUSTER of stripes that gather the
// same X block rows (a compact ball of the stripe graph: a 3D operator's neighbouring nodes), one workgroup
// each.  A node's X block row is used by every stripe coupled to it -- ~16 tiles on the c5-mesh operator --
// and a cluster of ~50 neighbouring stripes gathers each of its U distinct block rows ~4 times, so:
//   * phase 1: the workgroup loads the cluster's U block rows (ub x 16 right-hand sides each, slot order =
//     ascending row) into LDS with full-line 16-B loads, plus one zero slot (U) for padding tiles;
//   * phase 2: 16 streams (4 waves x 4 rows of 16 lanes; lane j = right-hand side j) walk the cluster's
//     tiles, each tile's block read with ub ds_read_b32 from its slot (key bits 0..15) instead of ub
//     global gathers, the values streamed and DPP-broadcast exactly as spmm_tiles (the same fma chain per
//     column, so every column equals the reference's product bit for bit, multiply_VBC.jl:126-135);
//     keys and values run kTileXDepth batches ahead (no X registers to hold: the gathers are LDS reads);
//   * a LAST tile parks the stripe's w x 16 sums in the workgroup's output stage, written after a barrier.
// X4: 16 contiguous right-hand sides in 16-B aligned rows (16-B staging loads); else element loads.
template <typename T, int UB, int W, bool MASKU, bool X4, int NW>
__global__ __launch_bounds__(NW * 64) void spmm_tiles_x(const TileBin b, const T *__restrict__ X, int64_t sxr,
                                                              int64_t sxc, int64_t xrows, T *__restrict__ Y, int64_t syr,
                                                              int64_t syc, int nrhs, T alpha, T beta, int rd_i, int fast)
{
    constexpr int NB = kTileXBatch, D = kTileXDepth;
    constexpr int TV = UB * W;
    constexpr int EPL = 16 / (int)sizeof(T);  // elements per 16-B piece
    constexpr int PER = 16 * EPL;             // elements per value load of a 16-lane row
    constexpr int NV = (NB * TV + PER - 1) / PER;
    constexpr int PPR = 16 / EPL;             // 16-B pieces per X row of 16 right-hand sides
    typedef T tv __attribute__((ext_vector_type(EPL)));
    extern __shared__ __attribute__((aligned(16))) char tile_stage[];
    const int cl = xcd_block(blockIdx.x, gridDim.x);
    if (cl >= b.nranges) return;  // (the whole workgroup)
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, g = lane >> 4, j = lane & 15;
    // the cluster's info through the scalar cache (constant address space: uniform s_load)
    typedef __attribute__((address_space(4))) const int32_t *cptr;
    const cptr ci = (cptr)b.rinfo + (size_t)cl * kTileXInfo;
    const int s0 = __builtin_amdgcn_readfirstlane(ci[0]), ns = __builtin_amdgcn_readfirstlane(ci[1]);
    const int U = __builtin_amdgcn_readfirstlane(ci[2]), xo = __builtin_amdgcn_readfirstlane(ci[3]);
    // the wave's segment of the cluster: its own length (the longest of its 4 rows' streams, whole batches);
    // the rows of a wave are strided by the wave's whole stream (the persistent layout, spmm_tiles_xp)
    const int tile0 = __builtin_amdgcn_readfirstlane(ci[kXiSeg + wv]), len = __builtin_amdgcn_readfirstlane(ci[kXiLen + wv]);
    const int rstride = __builtin_amdgcn_readfirstlane(ci[kXiStride + wv]);
    const int stream = wv * 4 + g;
    int sidx = G(b.rinfo)[(size_t)cl * kTileXInfo + kXiSidx + stream];  // cluster-local index of this row's first stripe
                                                                  // (a stream's stripes are consecutive)
    const int64_t kb = (int64_t)tile0 + (int64_t)g * rstride;
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    T *xl = reinterpret_cast<T *>(tile_stage);
    T *st = reinterpret_cast<T *>(tile_stage + (size_t)b.xslots * UB * 16 * sizeof(T));
    const T zero = T(0);

    // keys and values of the first D batches first: their latency overlaps the X stage
    auto load_keys = [&](int t0) -> uint32_t { return key[kb + t0 + (j < NB ? j : NB - 1)]; };
    auto load_vals = [&](int t0, tv (&V)[NV]) {
        const gptr<const T> p = val + (kb + t0) * TV + j * EPL;
#pragma unroll
        for (int v = 0; v < NV; v++) V[v] = __builtin_nontemporal_load((gptr<const tv>)(p + v * PER));
    };
    uint32_t K[D];
    tv V[D][NV];
#pragma unroll
    for (int d = 0; d < D; d++) {
        K[d] = load_keys(d * NB);
        load_vals(d * NB, V[d]);
    }
    // the output columns of this thread's output pieces (the epilogue's), loaded now so that no round trip
    // follows the loop: piece p = tid + k * 256 of the ns x W x PPR pieces belongs to stripe p / (W * PPR)
    const gptr<const int32_t> outp = G(b.out) + s0;
    int ocol[kTileXOutPieces];
#pragma unroll
    for (int k = 0; k < kTileXOutPieces; k++) ocol[k] = outp[min((tid + k * (NW * 64)) / (W * PPR), max(ns - 1, 0))];

    // phase 1: the cluster's X block rows -> LDS [slot][r][16], slot U (and rows past X) zero.  Every load of
    // a thread is issued before the first LDS write, with clamped addresses and selects instead of branches
    // (a load inside a branch makes the compiler wait for every load in flight, the prefetched values
    // included): one round trip for the slots' rows, one for the stage.  At most kTileXPieces 16-B pieces
    // per thread (the builder caps U to fit).
    if (!(b.diag & 1)) {  // (diag 1: no staging -- an ablation, tools/ab.py)
        constexpr int MP = tile_x_pieces(NW);
        const gptr<const int32_t> xr = G(b.xrow) + xo;  // (xrow carries one entry past the last cluster's)
        if constexpr (X4) {
            const int np = (U + 1) * UB * PPR;
            int row[MP];
#pragma unroll
            for (int u = 0; u < MP; u++) {
                const int p = tid + u * (NW * 64);
                const int slot = min(p / (UB * PPR), U);
                const int rr = (p - slot * (UB * PPR)) / PPR;
                const int r0 = xr[slot] + rr;
                row[u] = ((p < np) & (slot < U) & (r0 < xrows)) ? r0 : -1;
            }
            tv v[MP];
#pragma unroll
            for (int u = 0; u < MP; u++) {
                const int p = tid + u * (NW * 64);
                const tv t = *(gptr<const tv>)(G(X) + (int64_t)max(row[u], 0) * sxr + (p % PPR) * EPL);
                v[u] = row[u] >= 0 ? t : tv{};
            }
#pragma unroll
            for (int u = 0; u < MP; u++) {
                const int p = tid + u * (NW * 64);
                // piece p of the stage is elements p * EPL .. p * EPL + EPL - 1: (slot, row r, RHS group q)
                if (p < np) *reinterpret_cast<tv *>(xl + p * EPL) = v[u];
            }
        } else {
            const int ne = (U + 1) * UB * 16;
            for (int e0 = 0; e0 < ne; e0 += MP * (NW * 64)) {
                int row[MP];
#pragma unroll
                for (int u = 0; u < MP; u++) {
                    const int e = e0 + tid + u * (NW * 64);
                    const int slot = min(e / (UB * 16), U);
                    const int r0 = xr[slot] + (e >> 4) - slot * UB;
                    row[u] = ((e < ne) & (slot < U) & (r0 < xrows) & ((e & 15) < nrhs)) ? r0 : -1;
                }
                T v[MP];
#pragma unroll
                for (int u = 0; u < MP; u++) {
                    const int jj = (e0 + tid + u * (NW * 64)) & 15;
                    const T t = G(X)[(int64_t)max(row[u], 0) * sxr + (int64_t)(row[u] >= 0 ? jj : 0) * sxc];
                    v[u] = row[u] >= 0 ? t : zero;
                }
#pragma unroll
                for (int u = 0; u < MP; u++)
                    if (e0 + tid + u * (NW * 64) < ne) xl[e0 + tid + u * (NW * 64)] = v[u];
            }
        }
    }
    __syncthreads();

    T acc[W];
#pragma unroll
    for (int c = 0; c < W; c++) acc[c] = zero;
    // per batch: bit 16 g + s of `lastm` = LAST of step s of row g (lanes s >= NB hold copies, never tested)
    auto fold = [&](uint32_t Kk, const tv (&Vv)[NV]) {
        const uint64_t lastm = __builtin_amdgcn_ballot_w64((Kk & kTileLast) != 0);
        T xs[NB][UB];
#pragma unroll
        for (int s = 0; s < NB; s++) {
            const uint32_t ks = (uint32_t)row_bcast_rt((int)Kk, s);
            const T *xp = xl + (ks & kTileXSlot) * (UB * 16) + j;
#pragma unroll
            for (int r = 0; r < UB; r++) {
                xs[s][r] = xp[r * 16];
                // a slot row the tile does not store: x taken as 0 (its values are 0), as in spmm_tiles
                if constexpr (MASKU) xs[s][r] = ((ks >> (kTileMaskShift + r)) & 1) ? xs[s][r] : zero;
            }
        }
#pragma unroll
        for (int s = 0; s < NB; s++) {
#pragma unroll
            for (int r = 0; r < UB; r++) {
#pragma unroll
                for (int c = 0; c < W; c++) {
                    const int f = s * TV + r * W + c;
                    fmac_bcast_rt(acc[c], Vv[f / PER][f % EPL], xs[s][r], (f % PER) / EPL);
                }
            }
            if ((lastm >> s) & 0x0001000100010001ull) {
                const bool last = ((lastm >> (16 * g + s)) & 1) != 0;
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
    // phase 2: batch t0 + d NB from ring slot d, refilled with batch t0 + (d + D) NB (streams are padded to
    // whole batches; the loads past a stream's end read the next stream or the layout's padding, unused)
    for (int t0 = 0; t0 < len; t0 += D * NB) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            // (the refill is unconditional: a load inside the branch would make every later fold wait for
            // all loads in flight; past the stream's end it reads the next stream or the padding, unused)
            __builtin_amdgcn_sched_barrier(0);
            if (t0 + d * NB < len) fold(K[d], V[d]);
            __builtin_amdgcn_sched_barrier(0);
            K[d] = load_keys(t0 + (d + D) * NB);
            load_vals(t0 + (d + D) * NB, V[d]);
        }
    }
    __syncthreads();

    // the cluster's outputs: stripe i (cluster-local) -> columns out[s0 + i] .. + W - 1
    const bool rd = rd_i != 0;
    if (b.diag & 2) return;  // (diag 2: no output stores -- an ablation)
    if (fast) {  // Y row-major with 16 contiguous right-hand sides: a stripe's W x 16 block is contiguous
        const int np = ns * W * PPR;  // (<= kTileXOutPieces x 256: the builder caps the stripes per cluster)
#pragma unroll
        for (int k = 0; k < kTileXOutPieces; k++) {
            const int p = tid + k * (NW * 64);
            if (p >= np) break;
            const int i = p / (W * PPR), rem = p - i * (W * PPR);
            gptr<T> yo = G(Y) + (int64_t)((b.diag & 4) ? (s0 + i) * W : ocol[k]) * 16 + rem * EPL;  // (diag 4: contiguous)
            const tv v = *reinterpret_cast<const tv *>(st + i * W * 16 + rem * EPL);
            tv o;
#pragma unroll
            for (int q = 0; q < EPL; q++) o[q] = alpha * v[q];
            if (rd) {
                const tv y0 = *(gptr<const tv>)yo;
#pragma unroll
                for (int q = 0; q < EPL; q++) o[q] = fmadd(beta, y0[q], o[q]);
            }
            *(gptr<tv>)yo = o;
        }
    } else {
        const int total = ns * W * 16;
        for (int e = tid; e < total; e += (NW * 64)) {
            const int i = e / (W * 16), rem = e - i * (W * 16), c = rem >> 4, jj = rem & 15;
            if (jj >= nrhs) continue;
            gptr<T> yo = G(Y) + ((int64_t)outp[i] + c) * syr + (int64_t)jj * syc;
            T o = alpha * st[e];
            if (rd) o = fmadd(beta, *yo, o);
            *yo = o;
        }
    }
}

// Persistent staged-X form (round 5b, spmm_tiles_xp; fp32, 16 contiguous right-hand sides in X and Y).  The
// per-workgroup costs of spmm_tiles_x -- dispatch, the chain cluster info -> row groups -> X -> LDS before the
// first tile, the output stores draining at the end (c5-mesh ablations: staging 60 us, stores 58 us of 303) --
// are taken off the compute waves:
//   * one workgroup per resident slot (TileBin::nwg) walks a sequence of clusters (wginfo); its 4 compute waves
//     each read ONE continuous stream per row (the clusters' segments back to back), so the keys and values run
//     kTileXDepth batches ahead across cluster boundaries;
//   * a stager wave fills the other half of a double-buffered LDS X stage with the next cluster's row groups
//     (LDS-DMA, global_load_lds_dwordx4: no registers, all pieces in flight at once) while the compute waves
//     fold the current cluster;
//   * a writer wave stores the previous cluster's outputs from the other half of a double-buffered output stage;
//   * the END key bit (the last tile of a wave's segment) closes a cluster: one barrier of all six waves, then
//     both halves swap.  Every wave passes 1 + K barriers.
// Each column keeps the reference's fma chain per stripe (the fold is spmm_tiles_x's): bit for bit.
// A workgroup barrier that orders LDS only: __syncthreads()'s workgroup fence would also wait for every
// global load in flight (vmcnt(0): the compute waves' value prefetch, drained at each cluster boundary).
// The LDS-DMA stage is waited for by the stager itself (vmcnt(0)) before it joins the barrier.
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
constexpr int kTileXPWaves = 6;                         // 4 compute, 1 stager, 1 writer
constexpr int64_t kTileXPLds = 160 * 1024 - 1024;       // LDS of the CU shared by the persistent workgroups
constexpr int kTileXPThreads = kTileXPWaves * 64;
constexpr int kTileXPLoad = 32;                         // 16-B X pieces per stager lane per cluster (at most)
constexpr int kTileXPOut = 24;                          // 16-B output pieces per writer lane per cluster
template <int UB, int W, bool MASKU>
__global__ __launch_bounds__(kTileXPThreads) void spmm_tiles_xp(const TileBin b, const float *__restrict__ X, int64_t sxr,
                                                                int64_t xrows, float *__restrict__ Y, float alpha,
                                                                float beta, int rd_i)
{
    typedef float T;
    constexpr int NB = kTileXBatch, D = kTileXDepth;
    constexpr int TV = UB * W;
    constexpr int EPL = 4, PER = 64, PPR = 4;
    constexpr int NV = (NB * TV + PER - 1) / PER;
    typedef float tv __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(4))) const int32_t *cptr;
    extern __shared__ __attribute__((aligned(16))) char tile_stage[];
    const int xfl = b.xslots * UB * 16;          // floats per X half
    const int sfl = b.stage_bytes / 4;           // floats per output half
    T *xbuf = reinterpret_cast<T *>(tile_stage);
    T *sbuf = xbuf + 2 * xfl;
    int *sinfo = reinterpret_cast<int *>(sbuf + 2 * sfl);  // [2][16]: first local stripe of each stream
    const int L = xcd_block(blockIdx.x, gridDim.x);
    const cptr wg = (cptr)b.wginfo + 2 * L;
    const int c0 = wg[0], K = wg[1];
    if (K == 0) return;  // (the whole workgroup)
    const cptr cinfo = (cptr)b.rinfo;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;

    if (wv == 4) {  // ---- stager
        // rows of cluster c's pieces p = i * 64 + lane (-1: a zero piece), loaded one cluster ahead of its DMA
        auto load_rows = [&](int c, int (&row)[kTileXPLoad]) {
            const cptr ci = cinfo + (size_t)c * kTileXInfo;
            const int U = ci[2];
            const gptr<const int32_t> xr = G(b.xrow) + ci[3];
#pragma unroll
            for (int i = 0; i < kTileXPLoad; i++) {
                const int p = i * 64 + lane;
                const int slot = min(p / (UB * PPR), U);
                const int r0 = xr[slot] + (p - slot * (UB * PPR)) / PPR;
                // (bitwise &, not &&: a short-circuit test becomes a branch, the load is sunk into it and waited
                // for on the spot, one round trip per piece)
                const bool ok = (slot < U) & (r0 < xrows);
                row[i] = ok ? r0 : -1;
            }
        };
        auto dma = [&](int c, int half, const int (&row)[kTileXPLoad]) {
            const cptr ci = cinfo + (size_t)c * kTileXInfo;
            const int np = (ci[2] + 1) * UB * PPR;
            if (lane < kTileXStreams) sinfo[half * kTileXStreams + lane] = G(b.rinfo)[(size_t)c * kTileXInfo + kXiSidx + lane];
            // LDS byte address of this half (M0 of the DMA: lane l of piece round i lands at M0 + l * 16)
            const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)(xbuf + half * xfl);
#pragma unroll
            for (int i = 0; i < kTileXPLoad; i++) {
                const int p = i * 64 + lane;
                if (i * 64 < np) {  // (uniform)
                    const void *src = (row[i] >= 0 && p < np) ? (const void *)(X + (int64_t)row[i] * sxr + (p % PPR) * EPL) : b.zsrc;
                    // inline asm: the compiler's own LDS-DMA tracking waited for each piece before issuing the
                    // next (vmcnt(0)); the stager waits once for all of them before the cluster barrier.  Lanes
                    // past np are exec-masked off (the DMA writes only active lanes' pieces).
                    if (p < np)
                        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                                     :: "s"(dst + (uint32_t)i * 1024u), "v"(src) : "memory");
                }
            }
        };
        int row[kTileXPLoad];
        load_rows(c0, row);
        dma(c0, 0, row);
        if (K > 1) load_rows(c0 + 1, row);
        __builtin_amdgcn_s_waitcnt(0);
        lds_barrier();
        for (int k = 0; k < K; k++) {
            if (k + 1 < K) {
                dma(c0 + k + 1, (k + 1) & 1, row);        // (addresses read at issue)
                if (k + 2 < K) load_rows(c0 + k + 2, row);  // in flight with the DMA: one round trip per cluster
            }
            __builtin_amdgcn_s_waitcnt(0);  // (the LDS-DMA pieces landed)
            lds_barrier();  // cluster k done; cluster k + 1's stage in place
        }
        return;
    }
    if (wv == 5) {  // ---- writer
        const bool rd = rd_i != 0;
        lds_barrier();
        for (int k = 0; k < K; k++) {
            const cptr ci = cinfo + (size_t)(c0 + k) * kTileXInfo;
            const int s0 = ci[0], ns = ci[1];
            const int np = ns * W * PPR;
            const gptr<const int32_t> outp = G(b.out) + s0;
            int ocol[kTileXPOut];
#pragma unroll
            for (int i = 0; i < kTileXPOut; i++) ocol[i] = outp[min((i * 64 + lane) / (W * PPR), max(ns - 1, 0))];
            lds_barrier();  // cluster k's sums in output half k & 1
            const T *st = sbuf + (k & 1) * sfl;
#pragma unroll
            for (int i = 0; i < kTileXPOut; i++) {
                const int p = i * 64 + lane;
                if (i * 64 >= np) break;  // (uniform)
                if (p < np) {
                    const int si = p / (W * PPR), rem = p - si * (W * PPR);
                    gptr<T> yo = G(Y) + (int64_t)ocol[i] * 16 + rem * EPL;
                    const tv v = *reinterpret_cast<const tv *>(st + si * W * 16 + rem * EPL);
                    tv o;
#pragma unroll
                    for (int q = 0; q < EPL; q++) o[q] = alpha * v[q];
                    if (rd) {
                        const tv y0 = *(gptr<const tv>)yo;
#pragma unroll
                        for (int q = 0; q < EPL; q++) o[q] = fmadd(beta, y0[q], o[q]);
                    }
                    *(gptr<tv>)yo = o;
                }
            }
        }
        return;
    }
    // ---- compute waves
    const int g = lane >> 4, j = lane & 15, stream = wv * 4 + g;
    const cptr ci0 = cinfo + (size_t)c0 * kTileXInfo;
    const int len = ci0[kXiStride + wv];  // the wave's whole stream (its segments of the K clusters)
    const int64_t kb = (int64_t)ci0[kXiSeg + wv] + (int64_t)g * len;
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const T zero = T(0);
    auto load_keys = [&](int t0) -> uint32_t { return key[kb + t0 + (j < NB ? j : NB - 1)]; };
    auto load_vals = [&](int t0, tv (&V)[NV]) {
        const gptr<const T> p = val + (kb + t0) * TV + j * EPL;
#pragma unroll
        for (int v = 0; v < NV; v++) V[v] = __builtin_nontemporal_load((gptr<const tv>)(p + v * PER));
    };
    uint32_t Kr[D];
    tv V[D][NV];
#pragma unroll
    for (int d = 0; d < D; d++) {
        Kr[d] = load_keys(d * NB);
        load_vals(d * NB, V[d]);
    }
    lds_barrier();  // cluster 0's stage in place
    int half = 0;
    int sidx = sinfo[stream];
    T acc[W];
#pragma unroll
    for (int c = 0; c < W; c++) acc[c] = zero;
    auto fold = [&](uint32_t Kk, const tv (&Vv)[NV]) {
        const T *xl = xbuf + half * xfl;
        T *st = sbuf + half * sfl;
        const uint64_t lastm = __builtin_amdgcn_ballot_w64((Kk & kTileLast) != 0);
        T xs[NB][UB];
#pragma unroll
        for (int s = 0; s < NB; s++) {
            const uint32_t ks = (uint32_t)row_bcast_rt((int)Kk, s);
            const T *xp = xl + (ks & kTileXSlot) * (UB * 16) + j;
#pragma unroll
            for (int r = 0; r < UB; r++) {
                xs[s][r] = xp[r * 16];
                if constexpr (MASKU) xs[s][r] = ((ks >> (kTileMaskShift + r)) & 1) ? xs[s][r] : zero;
            }
        }
#pragma unroll
        for (int s = 0; s < NB; s++) {
#pragma unroll
            for (int r = 0; r < UB; r++) {
#pragma unroll
                for (int c = 0; c < W; c++) {
                    const int f = s * TV + r * W + c;
                    fmac_bcast_rt(acc[c], Vv[f / PER][f % EPL], xs[s][r], (f % PER) / EPL);
                }
            }
            if ((lastm >> s) & 0x0001000100010001ull) {
                const bool last = ((lastm >> (16 * g + s)) & 1) != 0;
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
        // the segment's last batch (every row of every compute wave has END at step NB - 1 of it)
        const uint32_t ke = (uint32_t)__builtin_amdgcn_readfirstlane(row_bcast_i<NB - 1>((int)Kk));
        if (ke & kTileXEnd) {
            lds_barrier();  // every wave done with this cluster; the next one's stage in place
            half ^= 1;
            sidx = sinfo[half * kTileXStreams + stream];
        }
    };
    for (int t0 = 0; t0 < len; t0 += D * NB) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            __builtin_amdgcn_sched_barrier(0);
            if (t0 + d * NB < len) fold(Kr[d], V[d]);
            __builtin_amdgcn_sched_barrier(0);
            Kr[d] = load_keys(t0 + (d + D) * NB);
            load_vals(t0 + (d + D) * NB, V[d]);
        }
    }
}

}  // namespace vbc
