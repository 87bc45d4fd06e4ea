// gfx950 planar slotted kernel for mul!(y, B', x) with stripes 3..8 columns wide (device code,
// included by vbc_planar.hip only).
//
// The slotted layout of vbc_slots.h gives a segment (stripe) LPR = w / V lanes when a stored row is
// wider than one 16-B lane vector: fp64 w = 3 runs 3 lanes per stripe with 8-B loads, 21 stripes per
// 63-lane wave, and the three lanes of a stripe gather the same x element.  Irregular 3-dof operators
// (SuiteSparse ldoor / 3D stiffness matrices: every node column a w = 3 stripe) then issue one
// 8-B-per-lane load, one key load and one gather per 21 stripe-rows -- request-rate bound (0.3-0.5 of
// the HBM roofline).  The *planar* chunk keeps one stripe per lane (64 stripes per chunk, RPI = 64) and
// stores each chunk row column-group-major: for the 16-B column groups g of the row (fp64: columns
// {0,1}, {2,3}, ...; fp32: {0..3}, {4..7}; the last group narrower), the 64 lanes' group-g values are
// contiguous, so every value load is one fully coalesced sweep (1 KiB for a 16-B group) and a lane
// holds its stripe's whole row.  Per stored row a lane issues cld(w, 16 B / sizeof(T)) value loads,
// one key load and one x gather (x[idx[Q]], multiply_1DVBC.jl:102) for 64 stripe-rows, folds the
// w columns serially in stored (reference) row order, and at the chunk's LAST row writes its w
// outputs (y[j : j+w-1], :114-116).  PAD / LAST / compressed keys, ranges of whole chunks, the
// two-stage pipeline and LDS-staged contiguous y writes follow vbc_slots.h.
#pragma once
#include "vbc_kernels.h"

namespace vbc {

// Column groups of a W_-wide row: 16-B groups of G = 16 / sizeof(T) elements, the last one narrower.
template <typename T>
__host__ __device__ constexpr int planar_g() { return 16 / (int)sizeof(T); }
template <typename T, int W_>
__host__ __device__ constexpr int planar_ngroups() { return (W_ + planar_g<T>() - 1) / planar_g<T>(); }
template <typename T, int W_, int GI>
__host__ __device__ constexpr int planar_vg() { return (W_ - GI * planar_g<T>()) < planar_g<T>() ? (W_ - GI * planar_g<T>()) : planar_g<T>(); }

// Element offset of (slot s, column c) inside a planar chunk row of width w (host and device).
__host__ __device__ inline int64_t planar_off(int esz, int w, int s, int c)
{
    const int G = 16 / esz, g = c / G, vg = (w - g * G) < G ? (w - g * G) : G;
    return (int64_t)64 * g * G + (int64_t)s * vg + (c - g * G);
}

// VG consecutive elements of a group (non-temporal: the value stream is read once); a 12-B group
// (fp32, 3 columns) is one dwordx3 load.
template <typename T, int VG, bool NT = true>
__device__ __forceinline__ void ld_group(gptr<const T> p, T *r)
{
    if constexpr (!NT && VG == 1) {  // cached loads (small matrices that stay in L2 between products)
        r[0] = *p;
    } else if constexpr (!NT && VG != 3) {
        typedef T vt __attribute__((ext_vector_type(VG)));
        const vt t = *(gptr<const vt>)p;
#pragma unroll
        for (int e = 0; e < VG; e++) r[e] = t[e];
    } else if constexpr (VG == 3) {
        struct __attribute__((packed, aligned(4))) p3 { T a, b, c; };
        const __attribute__((address_space(1))) p3 *q = (const __attribute__((address_space(1))) p3 *)p;
        r[0] = q->a;  // merged into one dwordx3 load
        r[1] = q->b;
        r[2] = q->c;
    } else if constexpr (VG == 1) {
        r[0] = __builtin_nontemporal_load(p);
    } else {
        typedef T vt __attribute__((ext_vector_type(VG)));
        const vt t = __builtin_nontemporal_load((gptr<const vt>)p);
#pragma unroll
        for (int e = 0; e < VG; e++) r[e] = t[e];
    }
}

template <typename T, int W_, int GI, bool NT = true>
__device__ __forceinline__ void ld_row(gptr<const T> row, int lane, T (&v)[W_])
{
    if constexpr (GI < planar_ngroups<T, W_>()) {
        constexpr int G = planar_g<T>(), VG = planar_vg<T, W_, GI>();
        ld_group<T, VG, NT>(row + 64 * GI * G + lane * VG, v + GI * G);
        ld_row<T, W_, GI + 1, NT>(row, lane, v);
    }
}

// RUN consecutive elements of x from one lane: one gather of RUN * sizeof(T) bytes (fp64 RUN = 3:
// dwordx4 + dwordx2; fp32 RUN = 3: dwordx3) instead of RUN separate requests.  Only element
// alignment is known (a run starts at any x row).
template <typename T, int RUN>
__device__ __forceinline__ void ld_run(gptr<const T> p, T (&r)[RUN])
{
    if constexpr (RUN == 1) {
        r[0] = *p;
    } else {
        struct __attribute__((packed, aligned(sizeof(T)))) pr { T e[RUN]; };
        const __attribute__((address_space(1))) pr *q = (const __attribute__((address_space(1))) pr *)p;
#pragma unroll
        for (int d = 0; d < RUN; d++) r[d] = q->e[d];  // merged into wide loads
    }
}

// fp64 runs of 3 (24 B at 8-B alignment: a node's x entries) gathered by lane PAIRS (round 6; PAIRS = true:
// the lane-stream kernel, FE-3D 214.8 / 213.6 -> 210.9 / 210.9 us B'x / B·x, profiles/r06o_*.log; the split
// kernels of small shards, latency-bound, keep one gather per lane -- the cross-lane swap waits for both
// loads: ldoor 1/8 forward shard 15.9 -> 17.9 us with pairs).  Each lane
// still folds its own run, but the pair (l, l ^ 1) loads both runs with two 16-B loads per lane -- load A
// the even lane's run, load B the odd lane's, the even lane at the run's first element and the odd lane at
// its second -- instead of one 16-B and one 8-B load per lane: every load instruction then touches 32 runs'
// lines, not 64 (the vector-memory path costs ≈ 2.4 CU cycles per distinct line: 306 -> 169 cycles per 64
// runs, tools/exp/ta_probe.hip shapes 12-14).  The slots: A's pair (x0, x1) or (x1, x2), B's likewise; a
// DPP quad_perm swap gives each lane the element its partner loaded (xrun_values).  Every lane of the wave
// must be active (the kernels call these at wave-uniform points); a dead or padding lane's index is the
// in-range index it would have gathered anyway.  Other eltypes / run lengths: ld_run, RUN slots.
template <typename T, int RUN, bool PAIRS = false>
__host__ __device__ constexpr bool xrun_pairs()
{
#ifdef VBC_XRUN_SINGLE  // (A/B build, tools/exp/build_variant.sh: each lane gathers its own run)
    return false;
#else
    return PAIRS && sizeof(T) == 8 && RUN == 3;
#endif
}
template <typename T, int RUN, bool PAIRS = false>
__host__ __device__ constexpr int xrun_slots() { return xrun_pairs<T, RUN, PAIRS>() ? 4 : RUN; }

__device__ __forceinline__ uint32_t pair_swap(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ double pair_swap(double v)
{
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint64_t lo = pair_swap((uint32_t)u), hi = pair_swap((uint32_t)(u >> 32));
    return __builtin_bit_cast(double, lo | (hi << 32));
}

template <typename T, int RUN, bool PAIRS = false>
__device__ __forceinline__ void ld_xrun(gptr<const T> xg, uint32_t idx, T (&r)[xrun_slots<T, RUN, PAIRS>()])
{
    if constexpr (xrun_pairs<T, RUN, PAIRS>()) {
        const uint32_t odd = threadIdx.x & 1, other = pair_swap(idx);
        const uint32_t ia = (odd ? other : idx) + odd, ib = (odd ? idx : other) + odd;
        struct __attribute__((packed, aligned(8))) d2p { double a, b; };
        typedef const __attribute__((address_space(1))) d2p *pp;
        const pp A = (pp)(xg + ia), B = (pp)(xg + ib);  // (member reads merge into one 16-B load each)
        r[0] = A->a;
        r[1] = A->b;
        r[2] = B->a;
        r[3] = B->b;
    } else {
        ld_run<T, RUN>(xg + idx, r);
    }
}

// The lane's own run from ld_xrun's slots (even lane: A = its (x0, x1), the odd lane's A.b = its x2; odd
// lane: B = its (x1, x2), the even lane's B.a = its x0).
template <typename T, int RUN, bool PAIRS = false>
__device__ __forceinline__ void xrun_values(const T (&r)[xrun_slots<T, RUN, PAIRS>()], T (&x)[RUN])
{
    if constexpr (xrun_pairs<T, RUN, PAIRS>()) {
        const bool odd = (threadIdx.x & 1) != 0;
        const double pa = pair_swap(r[1]), pb = pair_swap(r[2]);
        x[0] = odd ? pb : r[0];
        x[1] = odd ? r[2] : r[1];
        x[2] = odd ? r[3] : pa;
    } else {
#pragma unroll
        for (int d = 0; d < RUN; d++) x[d] = r[d];
    }
}

// One range (wave): chunks [rchunk[r], rchunk[r+1]), rows [rrow[r], rrow[r+1]).
// RUN > 1 (b.run): every lane's rows come in aligned runs of RUN consecutive x rows (a node's dof
// rows in a 3-dof stiffness operator): keys and the chunk's LAST flag are read from each run's first
// row only, and the run's x values are one RUN-wide gather.
// FASTE: affine y map and beta = 0 (no loads on the write path); NB > 0 (FASTE, contiguous chunk
// outputs): NB finished chunks staged in LDS and written as one run of 16-B stores.
// MASK (SlotBin::mask): lanes >= nlive[row] are padding; they read lane 0's key and values (lines lane 0
// fetches anyway) and fold nothing, so a chunk's padding rows cost no memory lines.
template <typename T, int W_, int U, bool FASTE, int NB, bool KC, int RUN, bool MASK = false>
__device__ __forceinline__ void run_planar(const SlotBin &b, int r, int lane, const T *__restrict__ x,
                                           T *__restrict__ y, T alpha, T beta, bool rd, char *lds_wave, int *lds_out)
{
    const int R0 = G(b.rrow)[r], R1 = G(b.rrow)[r + 1];
    if (R0 >= R1) return;
    int c = G(b.rchunk)[r];
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> xg = G(x);
    typedef __attribute__((address_space(4))) const uint32_t *cptr;
    const cptr bases = (cptr)b.base;
    const cptr doffs = (cptr)b.kdoff;
    const cptr nlive = (cptr)b.nlive;
    constexpr int NR = U / RUN;  // runs per step (ranges start and end on run boundaries)
    static_assert(NR * RUN == U, "a step holds whole runs");
    auto load = [&](int R, uint32_t (&kk)[NR], uint32_t (&bs)[NR], int (&nl)[NR], T (&v)[U][W_]) {
#pragma unroll
        for (int j = 0; j < NR; j++) {
            const int Rk = min(R + j * RUN, R1 - RUN);  // the run's first row (clamped: rows past the range)
            int ln = lane;
            if constexpr (MASK) {
                nl[j] = (int)nlive[Rk];
                ln = lane < nl[j] ? lane : 0;
            }
            if constexpr (KC) {
                kk[j] = (uint32_t)(int32_t)((gptr<const int16_t>)key)[(size_t)doffs[Rk] + ln];
                bs[j] = bases[Rk];
            } else {
                kk[j] = __builtin_nontemporal_load(key + (size_t)Rk * 64 + ln);
                bs[j] = 0;
            }
#pragma unroll
            for (int d = 0; d < RUN; d++) {
                const int Rc = min(R + j * RUN + d, R1 - 1);
                ld_row<T, W_, 0>(val + (size_t)Rc * 64 * W_, ln, v[j * RUN + d]);
            }
        }
    };
    constexpr uint32_t kPad16 = 0xFFFF8000u;
    auto gather = [&](const uint32_t (&kk)[NR], const uint32_t (&bs)[NR], T (&xv)[NR][xrun_slots<T, RUN>()]) {
#pragma unroll
        for (int j = 0; j < NR; j++) {
            const uint32_t gi = KC ? (bs[j] & kSlotIdx) + (kk[j] == kPad16 ? 0u : kk[j]) : kk[j] & kSlotIdx;
            ld_xrun<T, RUN>(xg, gi, xv[j]);
        }
    };
    T acc[W_];
#pragma unroll
    for (int e = 0; e < W_; e++) acc[e] = T(0);
    int nbuf = 0, cfirst = c;
    const int c0 = c;
    if constexpr (!FASTE) {
        if (!b.out_affine) {
            const int n = min(kSlotOutEntries, b.nseg - c0 * 64);
            for (int i = lane; i < n; i += 64) lds_out[i] = G(b.out)[c0 * 64 + i];
        }
    }
    // staged chunks [cfirst, cfirst + nbuf) -> y: one contiguous run of 64 * W_ values per chunk
    auto write_out = [&]() {
        const int64_t segs = min((int64_t)nbuf * 64, (int64_t)b.nseg - (int64_t)cfirst * 64);
        const int64_t bytes = segs * W_ * (int64_t)sizeof(T);
        char *dst = reinterpret_cast<char *>(y + b.out_base + (int64_t)cfirst * 64 * W_);
        if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            for (int64_t off = (int64_t)lane * 16; off < bytes; off += 1024) {
                if (off + 16 <= bytes) {
                    st_y((gptr<u4>)(dst + off), *reinterpret_cast<const u4 *>(lds_wave + off), VBC_ABL(b.diag & 16) != 0);
                } else {
                    for (int64_t q = off; q < bytes; q += sizeof(T))
                        *(gptr<T>)(dst + q) = *reinterpret_cast<const T *>(lds_wave + q);
                }
            }
        } else {
            for (int64_t off = (int64_t)lane * sizeof(T); off < bytes; off += 64 * sizeof(T))
                *(gptr<T>)(dst + off) = *reinterpret_cast<const T *>(lds_wave + off);
        }
        nbuf = 0;
    };
    auto flush = [&]() {
        const int seg = c * 64 + lane;
        if constexpr (NB > 0) {
            T *st = reinterpret_cast<T *>(lds_wave) + ((size_t)nbuf * 64 + lane) * W_;
#pragma unroll
            for (int e = 0; e < W_; e++) st[e] = alpha * acc[e];
            if (nbuf == 0) cfirst = c;
        } else if (seg < b.nseg) {
            const int o = (FASTE || b.out_affine) ? b.out_base + seg * b.out_stride : lds_out[(c - c0) * 64 + lane];
            gptr<T> yo = G(y) + o;
            const int lim = b.wst;  // padding columns (w > wst) are never written
#pragma unroll
            for (int e = 0; e < W_; e++) {
                if (e < lim) {
                    T q = alpha * acc[e];
                    if (!FASTE && rd) q = fmadd(beta, yo[e], q);
                    yo[e] = q;
                }
            }
        }
#pragma unroll
        for (int e = 0; e < W_; e++) acc[e] = T(0);
        c++;
        if constexpr (NB > 0) {
            if (++nbuf == NB) write_out();
        }
    };
    int R1v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(R1v) : "s"(R1));
    auto compute = [&](int R, const uint32_t (&kk)[NR], const uint32_t (&bs)[NR], const int (&nl)[NR],
                       const T (&v)[U][W_], const T (&xv)[NR][xrun_slots<T, RUN>()]) {
#pragma unroll
        for (int j = 0; j < NR; j++) {
            const bool pad = MASK ? lane >= nl[j] : (KC ? kk[j] == kPad16 : (kk[j] & kPad) != 0);
            const bool live = R + j * RUN < R1v && !(MASK && pad);  // MASK: lane 0's values, never folded
            T xr[RUN];
            xrun_values<T, RUN>(xv[j], xr);
#pragma unroll
            for (int d = 0; d < RUN; d++) {  // the run's rows in stored (reference) order
                const T xe = pad ? T(0) : xr[d];
#pragma unroll
                for (int e = 0; e < W_; e++) {
                    const T nv = fmadd(v[j * RUN + d][e], xe, acc[e]);
                    acc[e] = live ? nv : acc[e];
                }
            }
            const uint32_t lastw = KC ? bs[j] : (uint32_t)__builtin_amdgcn_readfirstlane((int)kk[j]);
            if (R + j * RUN < R1 && (lastw & kLast)) flush();
        }
    };
    uint32_t kA[NR], kB[NR], bA[NR], bB[NR];
    int nA[NR], nB[NR];
    T vA[U][W_], vB[U][W_], xv[NR][xrun_slots<T, RUN>()];
    load(R0, kA, bA, nA, vA);
    __builtin_amdgcn_s_waitcnt(0);
    for (int R = R0; R < R1; R += 2 * U) {
        gather(kA, bA, xv);
        load(R + U, kB, bB, nB, vB);
        compute(R, kA, bA, nA, vA, xv);
        gather(kB, bB, xv);
        load(R + 2 * U, kA, bA, nA, vA);
        compute(R + U, kB, bB, nB, vB, xv);
    }
    if constexpr (NB > 0) {
        if (nbuf > 0) write_out();
    }
}

// Rows per pipeline step: about 24 values per lane per stage (fp64 w = 3: 8 rows), whole runs.
// Values per lane per stage: fp64 24 (36 / 48 measured the same on ldoor and fe3d), fp32 with row
// runs 36 (ldoor stand-in 49.5 -> 44.7 us against 24; 48 the same; without runs 36 spills SGPRs:
// one scalar base per row).  A/B builds: -DVBC_PLANAR_VALS=...
// values per lane per step of the split products (spmv_planar_split, spmv_planar_fwd_split)
#ifndef VBC_SPLIT_VALS
#define VBC_SPLIT_VALS 9
#endif
#ifndef VBC_PLANAR_VALS
#define VBC_PLANAR_VALS (sizeof(T) == 8 || RUN == 1 ? 24 : 36)
#endif
template <typename T, int W_, int RUN>
__host__ __device__ constexpr int planar_step()
{
    constexpr int vals = VBC_PLANAR_VALS;
    constexpr int u = (vals / W_) < 2 ? 2 : ((vals / W_) > 12 ? 12 : (vals / W_));
    return u / RUN * RUN < RUN ? RUN : u / RUN * RUN;
}
// Chunks staged per y write: 8 KB of LDS per wave.
template <typename T, int W_>
__host__ __device__ constexpr int planar_nb()
{
    return (8192 / (64 * W_ * (int)sizeof(T))) > 8 ? 8 : (8192 / (64 * W_ * (int)sizeof(T)));
}

template <typename T, int W_, bool FASTE, int NB, bool KC, int RUN, bool MASK = false>
__global__ __launch_bounds__(kBlockThreads) void spmv_planar(const SlotBin b, const T *__restrict__ x,
                                                             T *__restrict__ y, T alpha, T beta, int rd_i)
{
    const int blk = b.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int rg = __builtin_amdgcn_readfirstlane((int)(blk * kWavesPerBlock + (threadIdx.x >> 6)));
    if (rg >= b.nranges) return;
    const int lane = threadIdx.x & 63;
    __shared__ __attribute__((aligned(16))) char stage[NB > 0 ? kWavesPerBlock * 8192 : 16];
    char *lds = stage + (NB > 0 ? (threadIdx.x >> 6) * 8192 : 0);
    __shared__ int outs[FASTE ? 1 : kWavesPerBlock * kSlotOutEntries];
    int *lds_out = outs + (FASTE ? 0 : (threadIdx.x >> 6) * kSlotOutEntries);
    run_planar<T, W_, planar_step<T, W_, RUN>(), FASTE, NB, KC, RUN, MASK>(b, rg, lane, x, y, alpha, beta, rd_i != 0,
                                                                            lds, lds_out);
}

// Per-lane compacted streams (SlotBin::lanes).  The masked chunk layout above steps every chunk
// through its longest stripe's rows: on an irregular operator (FE-3D: 1..12 runs per stripe) a third
// of its lane-rows are dead.  Here a range (one wave) is a *tile* of consecutive stripes
// [s0, s0 + ns), dealt to the 64 lanes as contiguous sub-blocks balanced by rows; lane l walks its
// sub-block's stored rows back to back -- stripe after stripe, each in stored (reference) row order
// (multiply_1DVBC.jl:101-104) -- so a tile holds ~5 % dead lane-rows instead of ~38 %.  Lanes are
// ordered by decreasing stream length: the live lanes of every step are a prefix (nlive; dead lanes
// read lane 0's lines, as MASK).  A run whose key has LAST closes the lane's current stripe: the lane
// stores its W_ sums into the wave's LDS tile buffer at that stripe's slot and moves to its next
// stripe (an empty stripe is one zero run with PAD | LAST).  Every slot of the tile is written exactly
// once; after the loop the wave writes the tile's ns * W_ outputs y[j : j+w-1] (:114-116) as one
// contiguous run of 16-B stores, α and β applied there.  (Writing the 24-B outputs straight from the
// lanes measured 213 -> 275 us on FE-3D: partial-line writes; no global store sits inside the loop,
// so the compiler's vmcnt accounting stays exact.)  DEEP: keys two steps ahead, the gathers one step
// ahead of their fold.
#ifndef VBC_LANE_TILE_BYTES
#define VBC_LANE_TILE_BYTES 8192
#endif
constexpr int kLaneTileBytes = VBC_LANE_TILE_BYTES;  // LDS tile buffer per wave (4 workgroups of 4 waves per
                                                     // CU, as the VGPR limit)

template <typename T, int W_, int U, int RUN, bool DEEP, bool RD, int DIAG = 0>
__device__ __forceinline__ void run_planar_lanes(const SlotBin &b, int r, int lane, const T *__restrict__ x,
                                                 T *__restrict__ y, T alpha, T beta, T *buf)
{
    typedef __attribute__((address_space(4))) const uint32_t *cptr;
    const int R0 = G(b.rrow)[r], R1 = G(b.rrow)[r + 1];
    if (R0 >= R1) return;
    const int s0 = G(b.tseg)[r];
    const int ns = G(b.tseg)[r + 1] - s0;
    int cur = (int)G(b.lseg)[(size_t)r * 64 + lane];  // the lane's current stripe, relative to s0
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> xg = G(x);
    const cptr nlive = (cptr)b.nlive;
    constexpr int NR = U / RUN;
    static_assert(NR * RUN == U, "a step holds whole runs");
    T acc[W_];
#pragma unroll
    for (int e = 0; e < W_; e++) acc[e] = T(0);
    int R1v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(R1v) : "s"(R1));
    // fold a step; kk: the runs' keys (or just their PAD / LAST bits)
    auto compute = [&](int R, const uint32_t (&kk)[NR], const int (&nl)[NR], const T (&v)[U][W_],
                       const T (&xv)[NR][xrun_slots<T, RUN, true>()]) {
#pragma unroll
        for (int j = 0; j < NR; j++) {
            const bool live = R + j * RUN < R1v && lane < nl[j];  // dead lanes hold lane 0's values
            const bool kpad = (kk[j] & kPad) != 0;                // an empty stripe's zero run
            T xr[RUN];
            xrun_values<T, RUN, true>(xv[j], xr);
#pragma unroll
            for (int d = 0; d < RUN; d++) {  // the run's rows in stored (reference) order
                const T xe = kpad ? T(0) : xr[d];
#pragma unroll
                for (int e = 0; e < W_; e++) {
                    const T nv = fmadd(v[j * RUN + d][e], xe, acc[e]);
                    acc[e] = live ? nv : acc[e];
                }
            }
            const bool fl = live && (kk[j] & kLast) != 0;
            if (DIAG != 3 && fl) {
#pragma unroll
                for (int e = 0; e < W_; e++) buf[cur * W_ + e] = acc[e];
            }
#pragma unroll
            for (int e = 0; e < W_; e++) acc[e] = fl ? T(0) : acc[e];
            cur += fl ? 1 : 0;
        }
    };
    auto load_keys = [&](int R, uint32_t (&kk)[NR], int (&nl)[NR]) {
#pragma unroll
        for (int j = 0; j < NR; j++) {
            const int Rk = min(R + j * RUN, R1 - RUN);  // the run's first row (clamped: rows past the range)
            nl[j] = (int)nlive[Rk];
            kk[j] = __builtin_nontemporal_load(key + (size_t)Rk * 64 + (lane < nl[j] ? lane : 0));
        }
    };
    auto load_vals = [&](int R, const int (&nl)[NR], T (&v)[U][W_]) {
#pragma unroll
        for (int j = 0; j < NR; j++) {
            const int ln = lane < nl[j] ? lane : 0;
#pragma unroll
            for (int d = 0; d < RUN; d++)
                ld_row<T, W_, 0>(val + (size_t)min(R + j * RUN + d, R1 - 1) * 64 * W_, ln, v[j * RUN + d]);
        }
    };
    // DIAG (tools/ab.py ablations, VBC_DIAG): 1 = no x gathers (x taken as 1), 2 = gathers confined to
    // the first 16 K rows of x (L2-resident), 3 = no LDS stores of finished stripes
    auto gather = [&](const uint32_t (&kk)[NR], T (&xv)[NR][xrun_slots<T, RUN, true>()]) {
#pragma unroll
        for (int j = 0; j < NR; j++) {
            if constexpr (DIAG == 1) {
#pragma unroll
                for (int d = 0; d < xrun_slots<T, RUN, true>(); d++) xv[j][d] = T(1);
            } else {
                ld_xrun<T, RUN, true>(xg, kk[j] & (DIAG == 2 ? 0x3FFFu : kSlotIdx), xv[j]);
            }
        }
    };
    if constexpr (!DEEP) {
        uint32_t kA[NR], kB[NR];
        int nA[NR], nB[NR];
        T vA[U][W_], vB[U][W_], xv[NR][xrun_slots<T, RUN, true>()];
        load_keys(R0, kA, nA);
        load_vals(R0, nA, vA);
        __builtin_amdgcn_s_waitcnt(0);
        for (int R = R0; R < R1; R += 2 * U) {
            gather(kA, xv);
            load_keys(R + U, kB, nB);
            load_vals(R + U, nB, vB);
            compute(R, kA, nA, vA, xv);
            gather(kB, xv);
            load_keys(R + 2 * U, kA, nA);
            load_vals(R + 2 * U, nA, vA);
            compute(R + U, kB, nB, vB, xv);
        }
    } else {
        // a step's key buffer is free once its gathers are issued (PAD / LAST move to a flags word), so
        // two key buffers rotate with the two value and gather buffers
        auto issue = [&](const uint32_t (&kk)[NR], T (&xv)[NR][xrun_slots<T, RUN, true>()], uint32_t (&fl)[NR]) {
            gather(kk, xv);
#pragma unroll
            for (int j = 0; j < NR; j++) {
                fl[j] = kk[j] & (kPad | kLast);
                asm volatile("" : "+v"(fl[j]));  // materialise now: kk's register is reloaded next step
            }
        };
        uint32_t kA[NR], kB[NR], fA[NR], fB[NR];
        int nA[NR], nB[NR];
        T vA[U][W_], vB[U][W_], xA[NR][xrun_slots<T, RUN, true>()], xB[NR][xrun_slots<T, RUN, true>()];
        load_keys(R0, kA, nA);
        load_keys(R0 + U, kB, nB);
        load_vals(R0, nA, vA);
        issue(kA, xA, fA);
        for (int R = R0; R < R1; R += 2 * U) {
            int nC[NR], nD[NR];
            load_keys(R + 2 * U, kA, nC);  // step R: keys(R + 2U); gathers and values of R + U; fold R
            issue(kB, xB, fB);
            load_vals(R + U, nB, vB);
            compute(R, fA, nA, vA, xA);
#pragma unroll
            for (int j = 0; j < NR; j++) nA[j] = nC[j];
            load_keys(R + 3 * U, kB, nD);  // step R + U
            issue(kA, xA, fA);
            load_vals(R + 2 * U, nA, vA);
            compute(R + U, fB, nB, vB, xB);
#pragma unroll
            for (int j = 0; j < NR; j++) nB[j] = nD[j];
        }
    }
    // the tile's outputs -> y: one contiguous run (every slot was written once by its lane)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    T *dst = y + b.out_base + (int64_t)s0 * W_;
    const int n = ns * W_;
    constexpr int VE = 16 / (int)sizeof(T);
    typedef T vt __attribute__((ext_vector_type(VE)));
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        for (int i = lane * VE; i < n; i += 64 * VE) {
            if (i + VE <= n) {
                vt q = *reinterpret_cast<const vt *>(buf + i) * alpha;
                if constexpr (RD) {
                    const vt yo = *(gptr<const vt>)(dst + i);
#pragma unroll
                    for (int e = 0; e < VE; e++) q[e] = fmadd(beta, yo[e], q[e]);
                }
                st_y((gptr<vt>)(dst + i), q, VBC_ABL(b.diag & 16) != 0);
            } else {
                for (int e = i; e < n; e++) {
                    T q = alpha * buf[e];
                    if constexpr (RD) q = fmadd(beta, G(dst)[e], q);
                    G(dst)[e] = q;
                }
            }
        }
    } else {
        for (int e = lane; e < n; e += 64) {
            T q = alpha * buf[e];
            if constexpr (RD) q = fmadd(beta, G(dst)[e], q);
            G(dst)[e] = q;
        }
    }
}

template <typename T, int W_, int RUN, bool DEEP, bool RD, int DIAG = 0>
__global__ __launch_bounds__(kBlockThreads) void spmv_planar_lanes(const SlotBin b,
                                                                   const T *__restrict__ x, T *__restrict__ y,
                                                                   T alpha, T beta)
{
    const int blk = b.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int rg = __builtin_amdgcn_readfirstlane((int)(blk * kWavesPerBlock + (threadIdx.x >> 6)));
    if (rg >= b.nranges) return;
    __shared__ __attribute__((aligned(16))) T tilebuf[kWavesPerBlock][kLaneTileBytes / sizeof(T)];
    run_planar_lanes<T, W_, planar_step<T, W_, RUN>(), RUN, DEEP, RD, DIAG>(b, rg, threadIdx.x & 63, x, y, alpha, beta,
                                                                      tilebuf[threadIdx.x >> 6]);
}

// Planar forward product with row runs (SlotBin kind 1, run = R): mul!(y, B, x) for node-blocked rows.
// A lane owns a segment of R consecutive output rows whose stripe lists are identical; per block (chunk
// row) it loads the block's R x w values (column-group-major, planar_off width R*w), gathers the
// stripe's w-wide x slice once (x[j .. j+w-1], multiply_1DVBC.jl:27 -- one gather for R rows instead
// of R), and adds the R dot products to its R accumulators, blocks in stripe order as the reference's
// serial stripe loop (:62-71).  At the LAST row the lane writes y[R*q .. R*q+R-1] (contiguous, LDS-
// staged in runs of NB chunks when FASTE).
// MASK (SlotBin::mask): lanes >= nlive[row] read lane 0's key and values and add nothing.
template <typename T, int W_, int R, int U, bool FASTE, int NB, bool KC, bool MASK = false>
__device__ __forceinline__ void run_planar_fwd(const SlotBin &b, int r, int lane, const T *__restrict__ x,
                                               T *__restrict__ y, T alpha, T beta, bool rd, char *lds_wave)
{
    constexpr int WV = R * W_;
    const int R0 = G(b.rrow)[r], R1 = G(b.rrow)[r + 1];
    if (R0 >= R1) return;
    int c = G(b.rchunk)[r];
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> xg = G(x);
    typedef __attribute__((address_space(4))) const uint32_t *cptr;
    const cptr bases = (cptr)b.base;
    const cptr doffs = (cptr)b.kdoff;
    const cptr nlive = (cptr)b.nlive;
    auto load = [&](int Rr, uint32_t (&kk)[U], uint32_t (&bs)[U], int (&nl)[U], T (&v)[U][WV]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int Rc = min(Rr + u, R1 - 1);
            int ln = lane;
            if constexpr (MASK) {
                nl[u] = (int)nlive[Rc];
                ln = lane < nl[u] ? lane : 0;
            }
            if constexpr (KC) {
                kk[u] = (uint32_t)(int32_t)((gptr<const int16_t>)key)[(size_t)doffs[Rc] + ln];
                bs[u] = bases[Rc];
            } else {
                kk[u] = __builtin_nontemporal_load(key + (size_t)Rc * 64 + ln);
                bs[u] = 0;
            }
            ld_row<T, WV, 0>(val + (size_t)Rc * 64 * WV, ln, v[u]);
        }
    };
    constexpr uint32_t kPad16 = 0xFFFF8000u;
    auto gather = [&](const uint32_t (&kk)[U], const uint32_t (&bs)[U], T (&xv)[U][xrun_slots<T, W_>()]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t gi = KC ? (bs[u] & kSlotIdx) + (kk[u] == kPad16 ? 0u : kk[u]) : kk[u] & kSlotIdx;
            ld_xrun<T, W_>(xg, gi, xv[u]);
        }
    };
    T acc[R];
#pragma unroll
    for (int q = 0; q < R; q++) acc[q] = T(0);
    int nbuf = 0, cfirst = c;
    auto write_out = [&]() {
        const int64_t segs = min((int64_t)nbuf * 64, (int64_t)b.nseg - (int64_t)cfirst * 64);
        const int64_t bytes = segs * R * (int64_t)sizeof(T);
        char *dst = reinterpret_cast<char *>(y + b.out_base + (int64_t)cfirst * 64 * R);
        if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            for (int64_t off = (int64_t)lane * 16; off < bytes; off += 1024) {
                if (off + 16 <= bytes) st_y((gptr<u4>)(dst + off), *reinterpret_cast<const u4 *>(lds_wave + off), VBC_ABL(b.diag & 16) != 0);
                else
                    for (int64_t q = off; q < bytes; q += sizeof(T))
                        *(gptr<T>)(dst + q) = *reinterpret_cast<const T *>(lds_wave + q);
            }
        } else {
            for (int64_t off = (int64_t)lane * sizeof(T); off < bytes; off += 64 * sizeof(T))
                *(gptr<T>)(dst + off) = *reinterpret_cast<const T *>(lds_wave + off);
        }
        nbuf = 0;
    };
    auto flush = [&]() {
        const int seg = c * 64 + lane;
        if constexpr (NB > 0) {
            T *st = reinterpret_cast<T *>(lds_wave) + ((size_t)nbuf * 64 + lane) * R;
#pragma unroll
            for (int q = 0; q < R; q++) st[q] = alpha * acc[q];
            if (nbuf == 0) cfirst = c;
        } else if (seg < b.nseg) {  // affine (natural order) or the table of a length-sorted layout
            gptr<T> yo = G(y) + (b.out_affine ? b.out_base + (int64_t)seg * R : (int64_t)G(b.out)[seg]);
#pragma unroll
            for (int q = 0; q < R; q++) {
                T v = alpha * acc[q];
                if (!FASTE && rd) v = fmadd(beta, yo[q], v);
                yo[q] = v;
            }
        }
#pragma unroll
        for (int q = 0; q < R; q++) acc[q] = T(0);
        c++;
        if constexpr (NB > 0) {
            if (++nbuf == NB) write_out();
        }
    };
    int R1v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(R1v) : "s"(R1));
    auto compute = [&](int Rr, const uint32_t (&kk)[U], const uint32_t (&bs)[U], const int (&nl)[U],
                       const T (&v)[U][WV], const T (&xv)[U][xrun_slots<T, W_>()]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool live = Rr + u < R1v;
            const bool pad = MASK ? lane >= nl[u] : (KC ? kk[u] == kPad16 : (kk[u] & kPad) != 0);
            T xr[W_];
            xrun_values<T, W_>(xv[u], xr);
#pragma unroll
            for (int q = 0; q < R; q++) {  // one dot product per output row of the run
                T d = v[u][q * W_] * xr[0];
#pragma unroll
                for (int e = 1; e < W_; e++) d = fmadd(v[u][q * W_ + e], xr[e], d);
                acc[q] = (live && !pad) ? acc[q] + d : acc[q];
            }
            const uint32_t lastw = KC ? bs[u] : (uint32_t)__builtin_amdgcn_readfirstlane((int)kk[u]);
            if (Rr + u < R1 && (lastw & kLast)) flush();
        }
    };
    uint32_t kA[U], kB[U], bA[U], bB[U];
    int nA[U], nB[U];
    T vA[U][WV], vB[U][WV], xv[U][xrun_slots<T, W_>()];
    load(R0, kA, bA, nA, vA);
    __builtin_amdgcn_s_waitcnt(0);
    for (int Rr = R0; Rr < R1; Rr += 2 * U) {
        gather(kA, bA, xv);
        load(Rr + U, kB, bB, nB, vB);
        compute(Rr, kA, bA, nA, vA, xv);
        gather(kB, bB, xv);
        load(Rr + 2 * U, kA, bA, nA, vA);
        compute(Rr + U, kB, bB, nB, vB, xv);
    }
    if constexpr (NB > 0) {
        if (nbuf > 0) write_out();
    }
}

template <typename T, int W_, int R, bool FASTE, int NB, bool KC, bool MASK = false>
__global__ __launch_bounds__(kBlockThreads) void spmv_planar_fwd(const SlotBin b, const T *__restrict__ x,
                                                                 T *__restrict__ y, T alpha, T beta, int rd_i)
{
    const int blk = b.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int rg = __builtin_amdgcn_readfirstlane((int)(blk * kWavesPerBlock + (threadIdx.x >> 6)));
    if (rg >= b.nranges) return;
    const int lane = threadIdx.x & 63;
    __shared__ __attribute__((aligned(16))) char stage[NB > 0 ? kWavesPerBlock * 8192 : 16];
    char *lds = stage + (NB > 0 ? (threadIdx.x >> 6) * 8192 : 0);
#ifndef VBC_FWD_VALS
#define VBC_FWD_VALS 24  // values per lane per stage (A/B builds: -DVBC_FWD_VALS=...)
#endif
    // blocks per stage: ~VBC_FWD_VALS values per lane (fp64 R = 3, w = 3: 2 blocks)
    constexpr int U = (VBC_FWD_VALS / (R * W_)) < 2 ? 2 : (VBC_FWD_VALS / (R * W_));
    run_planar_fwd<T, W_, R, U, FASTE, NB, KC, MASK>(b, rg, lane, x, y, alpha, beta, rd_i != 0, lds);
}

// Split planar forward product (SlotBin kind 1, run = R, split = P > 1; ranges are single chunks of the
// natural-order layout): the forward counterpart of spmv_planar_split for matrices with few chunks
// (ct20stif: 273 chunks of ~19 blocks).  Wave k of workgroup c folds the blocks [R0 + k*S, R0 + (k+1)*S)
// of chunk c in stripe order, one block per step (keys and values, then the w-wide x gather, then the R
// dot products), keys and values through the cache as in spmv_planar_split; the P partial sums meet in
// LDS and wave 0 writes y[R*q .. R*q+R-1] = alpha * (((p0 + p1) + p2) + ...) + beta * y.
template <typename T, int W_, int R, int P>
__global__ __launch_bounds__(64 * P) void spmv_planar_fwd_split(const SlotBin b, const T *__restrict__ x,
                                                                T *__restrict__ y, T alpha, T beta, int rd_i)
{
    constexpr int WV = R * W_;
    constexpr int U = (VBC_SPLIT_VALS / WV) < 1 ? 1 : (VBC_SPLIT_VALS / WV);
    const int c = blockIdx.x;
    if (c >= b.nranges) return;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int R0 = G(b.rrow)[c], R1 = G(b.rrow)[c + 1];
    const int S = (R1 - R0 + P - 1) / P;
    const int a = __builtin_amdgcn_readfirstlane(min(R1, R0 + wv * S)), e = __builtin_amdgcn_readfirstlane(min(R1, a + S));
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> xg = G(x);
    T acc[R];
#pragma unroll
    for (int q = 0; q < R; q++) acc[q] = T(0);
    for (int Rr = a; Rr < e; Rr += U) {
        uint32_t kk[U];
        T v[U][WV], xv[U][xrun_slots<T, W_>()];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int Rc = min(Rr + u, e - 1);
            kk[u] = key[(size_t)Rc * 64 + lane];
            ld_row<T, WV, 0, false>(val + (size_t)Rc * 64 * WV, lane, v[u]);
        }
#pragma unroll
        for (int u = 0; u < U; u++) ld_xrun<T, W_>(xg, kk[u] & kSlotIdx, xv[u]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool live = Rr + u < e && (kk[u] & kPad) == 0;
            T xr[W_];
            xrun_values<T, W_>(xv[u], xr);
#pragma unroll
            for (int q = 0; q < R; q++) {
                T d = v[u][q * W_] * xr[0];
#pragma unroll
                for (int k = 1; k < W_; k++) d = fmadd(v[u][q * W_ + k], xr[k], d);
                acc[q] = live ? acc[q] + d : acc[q];
            }
        }
    }
    __shared__ T part[P - 1][64 * R];
    if (wv > 0) {
#pragma unroll
        for (int q = 0; q < R; q++) part[wv - 1][q * 64 + lane] = acc[q];
    }
    __syncthreads();
    if (wv != 0) return;
#pragma unroll
    for (int p = 0; p < P - 1; p++)
#pragma unroll
        for (int q = 0; q < R; q++) acc[q] += part[p][q * 64 + lane];
    const int seg = c * 64 + lane;
    if (seg >= b.nseg) return;
    gptr<T> yo = G(y) + b.out_base + (int64_t)seg * R;
#pragma unroll
    for (int q = 0; q < R; q++) {
        T t = alpha * acc[q];
        if (rd_i) t = fmadd(beta, yo[q], t);
        yo[q] = t;
    }
}

// Lane-pair planar product (SlotBin::pair: fp64, 3-wide stripes, rows in runs of 3 -- a 3-dof
// stiffness operator).  A run's three x values are 24 B: one lane needs a dwordx4 + dwordx2 gather
// (two requests).  Here lanes 2s and 2s+1 share stripe s: they gather x[g .. g+1] and x[g+1 .. g+2]
// with ONE dwordx4 instruction (same 64-B line, merged by the addresser) and swap the element the
// other one lacks over DPP.  The even lane owns columns 0 and 1, the odd lane column 2, each folding
// its columns' three rows in stored order (multiply_1DVBC.jl:101-104), so every output is still the
// reference's serial sum.  A chunk is 32 stripes; a row of the layout is a *run-row* (one run of every
// stripe, 288 values, no padding): A = 64 lanes x {r0c0, r0c1 | r0c2, r1c2}, B = 32 x {r1c0, r1c1},
// C = 32 x r2c2, D = 32 x {r2c0, r2c1}; three dwordx4 loads per lane per run-row (the odd lane's
// second one reads C and its neighbour, its third the even partner's D line: merged requests).
// MASK (SlotBin::mask): stripe slots >= nlive[run-row] are padding; their lanes read pair 0's keys and
// values (lane parity kept) and fold nothing.
// DOT (SlotBin::dot, the forward product mul!(y, B, x) of 3 x 3 node blocks, round 6): the layout is that of
// the blocks TRANSPOSED -- a "stripe" is an output node run of 3 rows, a run-row one block of it (stripes in
// order), its "rows" the block's 3 columns gathering x[j .. j+2] -- and each lane adds, per block, the dot
// product of its output row with the x slice to its accumulator: y[i] += (B[i][j] x[j] + B[i][j+1] x[j+1]) +
// B[i][j+2] x[j+2], blocks in stripe order -- the association of the reference's serial forward loop
// (multiply_1DVBC.jl:34, :62-71) and of run_planar_fwd, so the forward product stays bit-identical to it.
template <int NRS, bool FASTE, int NB, bool KC, bool MASK = false, bool DOT = false>
__device__ __forceinline__ void run_pair(const SlotBin &b, int r, int lane, const double *__restrict__ x,
                                         double *__restrict__ y, double alpha, double beta, bool rd, char *lds_wave,
                                         int *lds_out)
{
    typedef double d2 __attribute__((ext_vector_type(2)));
    const int R0 = G(b.rrow)[r], R1 = G(b.rrow)[r + 1];
    if (R0 >= R1) return;
    int c = G(b.rchunk)[r];
    const bool odd = (lane & 1) != 0;
    const int ps = lane >> 1;  // stripe slot of the pair
    const gptr<const double> val = G(static_cast<const double *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const double> xg = G(x);
    typedef __attribute__((address_space(4))) const uint32_t *cptr;
    const cptr bases = (cptr)b.base;
    const cptr doffs = (cptr)b.kdoff;
    const cptr nlive = (cptr)b.nlive;
    // per-lane element offsets of the three value loads inside a run-row
    const int o0 = 2 * lane, o1 = odd ? 192 + ps : 128 + 2 * ps, o2 = 224 + 2 * ps;
    auto load = [&](int R, uint32_t (&kk)[NRS], uint32_t (&bs)[NRS], int (&nl)[NRS], d2 (&v)[NRS][3]) {
#pragma unroll
        for (int j = 0; j < NRS; j++) {
            const int Rc = min(R + j, R1 - 1);
            int mps = ps, m0 = o0, m1 = o1, m2 = o2;
            if constexpr (MASK) {  // dead pairs: pair 0's addresses (lane parity kept)
                nl[j] = (int)nlive[Rc];
                const bool dead = ps >= nl[j];
                mps = dead ? 0 : ps;
                m0 = dead ? (odd ? 1 : 0) * 2 : o0;
                m1 = dead ? (odd ? 192 : 128) : o1;
                m2 = dead ? 224 : o2;
            }
            if constexpr (KC) {
                kk[j] = (uint32_t)(int32_t)((gptr<const int16_t>)key)[(size_t)doffs[Rc] + mps];
                bs[j] = bases[Rc];
            } else {
                kk[j] = key[(size_t)Rc * 32 + mps];
                bs[j] = 0;
            }
            const gptr<const double> rowp = val + (size_t)Rc * 288;
            v[j][0] = __builtin_nontemporal_load((gptr<const d2>)(rowp + m0));
            v[j][1] = *(const __attribute__((address_space(1))) d2 *)(rowp + m1);  // 8-B aligned (odd lanes)
            v[j][2] = __builtin_nontemporal_load((gptr<const d2>)(rowp + m2));
        }
    };
    constexpr uint32_t kPad16 = 0xFFFF8000u;
    auto gather = [&](const uint32_t (&kk)[NRS], const uint32_t (&bs)[NRS], d2 (&xv)[NRS]) {
#pragma unroll
        for (int j = 0; j < NRS; j++) {
            const uint32_t gi = KC ? (bs[j] & kSlotIdx) + (kk[j] == kPad16 ? 0u : kk[j]) : kk[j] & kSlotIdx;
            xv[j] = *(const __attribute__((address_space(1))) d2 *)(xg + gi + (odd ? 1 : 0));  // 8-B aligned
        }
    };
    double acc0 = 0.0, acc1 = 0.0;  // even: columns 0, 1; odd: column 2 in acc0
    int nbuf = 0, cfirst = c;
    const int c0 = c;
    if constexpr (!FASTE) {
        if (!b.out_affine) {
            const int n = min(kSlotOutEntries, b.nseg - c0 * 32);
            for (int i = lane; i < n; i += 64) lds_out[i] = G(b.out)[c0 * 32 + i];
        }
    }
    // staged chunks [cfirst, cfirst + nbuf) -> y: one contiguous run of 32 * 3 values per chunk
    auto write_out = [&]() {
        const int64_t segs = min((int64_t)nbuf * 32, (int64_t)b.nseg - (int64_t)cfirst * 32);
        const int64_t bytes = segs * 3 * (int64_t)sizeof(double);
        char *dst = reinterpret_cast<char *>(y + b.out_base + (int64_t)cfirst * 32 * 3);
        if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            for (int64_t off = (int64_t)lane * 16; off < bytes; off += 1024) {
                if (off + 16 <= bytes) st_y((gptr<u4>)(dst + off), *reinterpret_cast<const u4 *>(lds_wave + off), VBC_ABL(b.diag & 16) != 0);
                else
                    for (int64_t q = off; q < bytes; q += 8)
                        *(gptr<double>)(dst + q) = *reinterpret_cast<const double *>(lds_wave + q);
            }
        } else {
            for (int64_t off = (int64_t)lane * 8; off < bytes; off += 512)
                *(gptr<double>)(dst + off) = *reinterpret_cast<const double *>(lds_wave + off);
        }
        nbuf = 0;
    };
    auto flush = [&]() {
        const int seg = c * 32 + ps;
        if constexpr (NB > 0) {
            double *st = reinterpret_cast<double *>(lds_wave) + ((size_t)nbuf * 32 + ps) * 3;
            if (odd) st[2] = alpha * acc0;
            else {
                st[0] = alpha * acc0;
                st[1] = alpha * acc1;
            }
            if (nbuf == 0) cfirst = c;
        } else if (seg < b.nseg) {
            const int o = (FASTE || b.out_affine) ? b.out_base + seg * b.out_stride : lds_out[(c - c0) * 32 + ps];
            gptr<double> yo = G(y) + o;
            if (odd) {
                double q = alpha * acc0;
                if (!FASTE && rd) q = fmadd(beta, yo[2], q);
                yo[2] = q;
            } else {
                double q0 = alpha * acc0, q1 = alpha * acc1;
                if (!FASTE && rd) {
                    q0 = fmadd(beta, yo[0], q0);
                    q1 = fmadd(beta, yo[1], q1);
                }
                yo[0] = q0;
                yo[1] = q1;
            }
        }
        acc0 = acc1 = 0.0;
        c++;
        if constexpr (NB > 0) {
            if (++nbuf == NB) write_out();
        }
    };
    int R1v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(R1v) : "s"(R1));
    auto compute = [&](int R, const uint32_t (&kk)[NRS], const uint32_t (&bs)[NRS], const int (&nl)[NRS],
                       const d2 (&v)[NRS][3], const d2 (&xv)[NRS]) {
#pragma unroll
        for (int j = 0; j < NRS; j++) {
            const bool pad = MASK ? ps >= nl[j] : (KC ? kk[j] == kPad16 : (kk[j] & kPad) != 0);
            const bool live = R + j < R1v && !(MASK && pad);  // MASK: pair 0's values, never folded
            // even sends x[g] (its .x), odd sends x[g+2] (its .y); each receives the element it lacks
            const double t = odd ? xv[j].y : xv[j].x;
            const uint64_t tb = __builtin_bit_cast(uint64_t, t);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)tb, 0xB1, 0xF, 0xF, true);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(tb >> 32), 0xB1, 0xF, 0xF, true);
            const double other = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
            double x0 = odd ? other : xv[j].x, x1 = odd ? xv[j].x : xv[j].y, x2 = odd ? xv[j].y : other;
            if (pad) x0 = x1 = x2 = 0.0;
            // even: v[0] = {r0c0, r0c1}, v[1] = {r1c0, r1c1}, v[2] = {r2c0, r2c1}
            // odd:  v[0] = {r0c2, r1c2}, v[1].x = r2c2
            if constexpr (DOT) {
                const double d0 = odd ? fmadd(v[j][1].x, x2, fmadd(v[j][0].y, x1, v[j][0].x * x0))
                                      : fmadd(v[j][2].x, x2, fmadd(v[j][1].x, x1, v[j][0].x * x0));
                const double d1 = fmadd(v[j][2].y, x2, fmadd(v[j][1].y, x1, v[j][0].y * x0));
                acc0 = (live && !pad) ? acc0 + d0 : acc0;
                acc1 = (live && !pad) ? acc1 + d1 : acc1;
            } else {
                const double n0 = odd ? fmadd(v[j][1].x, x2, fmadd(v[j][0].y, x1, fmadd(v[j][0].x, x0, acc0)))
                                      : fmadd(v[j][2].x, x2, fmadd(v[j][1].x, x1, fmadd(v[j][0].x, x0, acc0)));
                const double n1 = fmadd(v[j][2].y, x2, fmadd(v[j][1].y, x1, fmadd(v[j][0].y, x0, acc1)));
                acc0 = live ? n0 : acc0;
                acc1 = live ? n1 : acc1;
            }
            const uint32_t lastw = KC ? bs[j] : (uint32_t)__builtin_amdgcn_readfirstlane((int)kk[j]);
            if (R + j < R1 && (lastw & kLast)) flush();
        }
    };
    uint32_t kA[NRS], kB[NRS], bA[NRS], bB[NRS];
    int nA[NRS], nB[NRS];
    d2 vA[NRS][3], vB[NRS][3], xv[NRS];
    load(R0, kA, bA, nA, vA);
    __builtin_amdgcn_s_waitcnt(0);
    for (int R = R0; R < R1; R += 2 * NRS) {
        gather(kA, bA, xv);
        load(R + NRS, kB, bB, nB, vB);
        compute(R, kA, bA, nA, vA, xv);
        gather(kB, bB, xv);
        load(R + 2 * NRS, kA, bA, nA, vA);
        compute(R + NRS, kB, bB, nB, vB, xv);
    }
    if constexpr (NB > 0) {
        if (nbuf > 0) write_out();
    }
}

template <bool FASTE, int NB, bool KC, bool MASK = false, bool DOT = false>
__global__ __launch_bounds__(kBlockThreads) void spmv_planar_pair(const SlotBin b,
                                                                  const double *__restrict__ x, double *__restrict__ y,
                                                                  double alpha, double beta, int rd_i)
{
    const int blk = b.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int rg = __builtin_amdgcn_readfirstlane((int)(blk * kWavesPerBlock + (threadIdx.x >> 6)));
    if (rg >= b.nranges) return;
    const int lane = threadIdx.x & 63;
    __shared__ __attribute__((aligned(16))) char stage[NB > 0 ? kWavesPerBlock * 8192 : 16];
    char *lds = stage + (NB > 0 ? (threadIdx.x >> 6) * 8192 : 0);
    __shared__ int outs[FASTE ? 1 : kWavesPerBlock * kSlotOutEntries];
    int *lds_out = outs + (FASTE ? 0 : (threadIdx.x >> 6) * kSlotOutEntries);
#ifndef VBC_PAIR_NRS
#define VBC_PAIR_NRS 4  // run-rows per pipeline stage (ldoor stand-in: 2 -> 82, 3 -> 80, 4 -> 77 us)
#endif
    run_pair<VBC_PAIR_NRS, FASTE, NB, KC, MASK, DOT>(b, rg, lane, x, y, alpha, beta, rd_i != 0, lds, lds_out);
}

// Lane-pair streams (SlotBin::lanes with pair: fp64, 3-wide stripes, rows in runs of 3 -- FE-3D): the
// lane-stream layout with a lane PAIR per stream, so a run's 24 B of x are ONE dwordx4 gather per lane
// (the pair reads x[g .. g+1] and x[g+1 .. g+2], one line, merged by the addresser) instead of a
// dwordx4 + dwordx2 per lane: the lane-stream kernel is bound by L1 -> L2 requests, of which the x
// gathers are two thirds (FE-3D ablation: no gathers 157 us, L2-resident gathers 197, real 204).
// A tile's stripes are cut into 32 streams; a layout row is a run-row of the 32 streams in the pair
// kernel's 288-value form (segments A, B, C, D, run_pair), keys and nlive per run-row; the even lane
// folds columns 0-1, the odd lane column 2, each in stored row order, and a LAST run stores them into
// the wave's LDS tile buffer at the stream's current stripe slot.  After the loop the wave writes the
// tile's outputs as one contiguous run (α, β applied there).
template <int NRS, bool RD>
__device__ __forceinline__ void run_pair_lanes(const SlotBin &b, int r, int lane, const double *__restrict__ x,
                                               double *__restrict__ y, double alpha, double beta, double *buf)
{
    typedef double d2 __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(4))) const uint32_t *cptr;
    const int R0 = G(b.rrow)[r], R1 = G(b.rrow)[r + 1];
    if (R0 >= R1) return;
    const int s0 = G(b.tseg)[r];
    const int ns = G(b.tseg)[r + 1] - s0;
    const bool odd = (lane & 1) != 0;
    const int ps = lane >> 1;  // stream slot of the pair
    int cur = (int)G(b.lseg)[(size_t)r * 64 + ps];
    const gptr<const double> val = G(static_cast<const double *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const double> xg = G(x);
    const cptr nlive = (cptr)b.nlive;
    const int o0 = 2 * lane, o1 = odd ? 192 + ps : 128 + 2 * ps, o2 = 224 + 2 * ps;
    auto load = [&](int R, uint32_t (&kk)[NRS], int (&nl)[NRS], d2 (&v)[NRS][3]) {
#pragma unroll
        for (int j = 0; j < NRS; j++) {
            const int Rc = min(R + j, R1 - 1);
            nl[j] = (int)nlive[Rc];
            const bool dead = ps >= nl[j];  // dead pairs: pair 0's addresses (lane parity kept)
            const int mps = dead ? 0 : ps;
            const int m0 = dead ? (odd ? 2 : 0) : o0, m1 = dead ? (odd ? 192 : 128) : o1, m2 = dead ? 224 : o2;
            kk[j] = key[(size_t)Rc * 32 + mps];
            const gptr<const double> rowp = val + (size_t)Rc * 288;
            v[j][0] = __builtin_nontemporal_load((gptr<const d2>)(rowp + m0));
            v[j][1] = *(const __attribute__((address_space(1))) d2 *)(rowp + m1);  // 8-B aligned (odd lanes)
            v[j][2] = __builtin_nontemporal_load((gptr<const d2>)(rowp + m2));
        }
    };
    auto gather = [&](const uint32_t (&kk)[NRS], d2 (&xv)[NRS]) {
#pragma unroll
        for (int j = 0; j < NRS; j++)
            xv[j] = *(const __attribute__((address_space(1))) d2 *)(xg + (kk[j] & kSlotIdx) + (odd ? 1 : 0));
    };
    double acc0 = 0.0, acc1 = 0.0;  // even: columns 0, 1; odd: column 2 in acc0
    int R1v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(R1v) : "s"(R1));
    auto compute = [&](int R, const uint32_t (&kk)[NRS], const int (&nl)[NRS], const d2 (&v)[NRS][3],
                       const d2 (&xv)[NRS]) {
#pragma unroll
        for (int j = 0; j < NRS; j++) {
            const bool live = R + j < R1v && ps < nl[j];  // dead pairs hold pair 0's values
            const bool kpad = (kk[j] & kPad) != 0;        // an empty stripe's zero run
            // even sends x[g] (its .x), odd sends x[g+2] (its .y); each receives the element it lacks
            const double t = odd ? xv[j].y : xv[j].x;
            const uint64_t tb = __builtin_bit_cast(uint64_t, t);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)tb, 0xB1, 0xF, 0xF, true);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(tb >> 32), 0xB1, 0xF, 0xF, true);
            const double other = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
            double x0 = odd ? other : xv[j].x, x1 = odd ? xv[j].x : xv[j].y, x2 = odd ? xv[j].y : other;
            if (kpad) x0 = x1 = x2 = 0.0;
            // even: v[0] = {r0c0, r0c1}, v[1] = {r1c0, r1c1}, v[2] = {r2c0, r2c1}
            // odd:  v[0] = {r0c2, r1c2}, v[1].x = r2c2
            const double n0 = odd ? fmadd(v[j][1].x, x2, fmadd(v[j][0].y, x1, fmadd(v[j][0].x, x0, acc0)))
                                  : fmadd(v[j][2].x, x2, fmadd(v[j][1].x, x1, fmadd(v[j][0].x, x0, acc0)));
            const double n1 = fmadd(v[j][2].y, x2, fmadd(v[j][1].y, x1, fmadd(v[j][0].y, x0, acc1)));
            acc0 = live ? n0 : acc0;
            acc1 = live ? n1 : acc1;
            const bool fl = live && (kk[j] & kLast) != 0;
            if (fl) {
                if (odd) buf[cur * 3 + 2] = acc0;
                else {
                    buf[cur * 3 + 0] = acc0;
                    buf[cur * 3 + 1] = acc1;
                }
            }
            acc0 = fl ? 0.0 : acc0;
            acc1 = fl ? 0.0 : acc1;
            cur += fl ? 1 : 0;
        }
    };
    uint32_t kA[NRS], kB[NRS];
    int nA[NRS], nB[NRS];
    d2 vA[NRS][3], vB[NRS][3], xv[NRS];
    load(R0, kA, nA, vA);
    __builtin_amdgcn_s_waitcnt(0);
    for (int R = R0; R < R1; R += 2 * NRS) {
        gather(kA, xv);
        load(R + NRS, kB, nB, vB);
        compute(R, kA, nA, vA, xv);
        gather(kB, xv);
        load(R + 2 * NRS, kA, nA, vA);
        compute(R + NRS, kB, nB, vB, xv);
    }
    // the tile's outputs -> y: one contiguous run (every slot was written once by its pair)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double *dst = y + b.out_base + (int64_t)s0 * 3;
    const int n = ns * 3;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        for (int i = lane * 2; i < n; i += 128) {
            if (i + 2 <= n) {
                d2 q = *reinterpret_cast<const d2 *>(buf + i) * alpha;
                if constexpr (RD) {
                    const d2 yo = *(gptr<const d2>)(dst + i);
                    q.x = fmadd(beta, yo.x, q.x);
                    q.y = fmadd(beta, yo.y, q.y);
                }
                *(gptr<d2>)(dst + i) = q;
            } else {
                double q = alpha * buf[i];
                if constexpr (RD) q = fmadd(beta, G(dst)[i], q);
                G(dst)[i] = q;
            }
        }
    } else {
        for (int e = lane; e < n; e += 64) {
            double q = alpha * buf[e];
            if constexpr (RD) q = fmadd(beta, G(dst)[e], q);
            G(dst)[e] = q;
        }
    }
}

template <bool RD>
__global__ __launch_bounds__(kBlockThreads) void spmv_pair_lanes(const SlotBin b, const double *__restrict__ x,
                                                                 double *__restrict__ y, double alpha, double beta)
{
    const int blk = b.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int rg = __builtin_amdgcn_readfirstlane((int)(blk * kWavesPerBlock + (threadIdx.x >> 6)));
    if (rg >= b.nranges) return;
    __shared__ __attribute__((aligned(16))) double tilebuf[kWavesPerBlock][kLaneTileBytes / sizeof(double)];
#ifndef VBC_PAIR_LANES_NRS
#define VBC_PAIR_LANES_NRS 4  // run-rows per pipeline stage (as VBC_PAIR_NRS)
#endif
    run_pair_lanes<VBC_PAIR_LANES_NRS, RD>(b, rg, threadIdx.x & 63, x, y, alpha, beta, tilebuf[threadIdx.x >> 6]);
}

// Split planar product (SlotBin::split = P > 1; ranges are single chunks): workgroup c = chunk c, wave k
// folds the rows [R0 + k*S, R0 + (k+1)*S) of it (S a whole number of runs) in stored order, the P
// partial accumulators meet in LDS and wave 0 writes y = alpha * (((p0 + p1) + p2) + ...) + beta * y.
// For matrices with fewer chunks than the chip has wave slots (ct20stif: 273 chunks of ~48 rows),
// where one wave per chunk leaves the product latency-bound.  Same keys, values and gathers as
// run_planar; summation order is per slice, then across slices.
// Rows per step of the split product: about VBC_SPLIT_VALS values per lane, whole runs (fp64 w = 3,
// runs of 3: one run).  Short steps measured fastest (cached loads, NS = 1, graph-timed,
// profiles/r03_splitu_*.log): ct20stif stand-in P = 4: 9 / 18 / 36 values 5.9 / 6.3 / 7.1 us; ldoor's 1/8
// stripe shard P = 4: 11.0 / 12.0 / 13.3 us.
template <typename T, int W_, int RUN>
__host__ __device__ constexpr int planar_split_step()
{
    constexpr int cap = 8 * RUN;  // <= 8 runs: their scalar key bases stay in SGPRs
    constexpr int u = (VBC_SPLIT_VALS / W_) / RUN * RUN;
    return u < RUN ? RUN : (u > cap ? cap / RUN * RUN : u);
}

// The split product's view of a bin: what one chunk's workgroup reads (SlotBin fields, or a part of a
// fused launch, SplitMulti below).
struct SplitView {
    const int32_t *rrow;
    const uint32_t *key;
    const void *val;
    const uint32_t *base;
    const uint32_t *kdoff;
    const int32_t *out;
    int32_t nseg, out_affine, out_base, out_stride, wst, holes, ks;
};

// Keys and values are CACHED loads here (the streaming kernels use non-temporal ones): a split bucket
// is small by construction, and its layout stays in L2 / MALL from one product to the next (ct20stif
// stand-in, 25 MB, graph-timed: 8.8 -> 6.2 us; ldoor's 1/8 stripe shard, 52 MB: 11.5 -> 11.0 us).
// DIAG (A/B ablations, tools/ab.py VBC_DIAG): 1 no x gathers, 2 gathers confined to 2 KB of x,
// 3 no y store, 4 non-temporal key / value loads.
// One chunk c by the P waves of a workgroup (wave wv); `part` = (P - 1) x 64 x W_ LDS partials.
// PIPE: a two-stage pipeline over the wave's slice (the keys and values of step i+1 are issued before
// the fold of step i, the gathers of step i right after its keys arrive) -- for slices of several
// steps (medium matrices of a fused split launch, where each wave streams tens of rows); the one-phase
// form issues a step's loads, gathers and fold back to back.
// MODE 2 (batched): NB runs of the slice at a time -- all their keys, then all their values, then all
// their gathers (each gather waits for its key only: the loads are counted in issue order), then the
// folds in stored order -- so a batch costs two memory round trips (keys, gathers) with the value
// stream under them, instead of two per step; NB keeps ~24 (fp64) / 48 (fp32) values per lane in flight.
#ifndef VBC_SPLIT_BATCH_VALS
#define VBC_SPLIT_BATCH_VALS (sizeof(T) == 8 ? 24 : 48)
#endif
template <typename T, int W_, int RUN>
__host__ __device__ constexpr int split_batch_runs()
{
    constexpr int nb = (int)(VBC_SPLIT_BATCH_VALS) / (W_ * RUN);
    return nb < 2 ? 2 : (nb > 16 ? 16 : nb);
}

template <typename T, int W_, bool KC, int RUN, int P, int DIAG = 0, int MODE = 0>
__device__ __forceinline__ void split_chunk(const SplitView &b, int c, int wv, int lane, const T *__restrict__ x,
                                            T *__restrict__ y, T alpha, T beta, int rd_i, T *part)
{
    constexpr int U = planar_split_step<T, W_, RUN>(), NR = U / RUN;
    const int R0 = G(b.rrow)[c], R1 = G(b.rrow)[c + 1];
    const int S = ((R1 - R0 + P - 1) / P + RUN - 1) / RUN * RUN;
    const int a = __builtin_amdgcn_readfirstlane(min(R1, R0 + wv * S)), e = __builtin_amdgcn_readfirstlane(min(R1, a + S));
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> xg = G(x);
    typedef __attribute__((address_space(4))) const uint32_t *cptr;
    const cptr bases = (cptr)b.base;
    const cptr doffs = (cptr)b.kdoff;
    constexpr uint32_t kPad16 = 0xFFFF8000u;
    T acc[W_];
#pragma unroll
    for (int k = 0; k < W_; k++) acc[k] = T(0);
    const uint32_t imask = b.holes ? kHoleIdx : kSlotIdx;  // runs with holes: the row mask sits above the index
    // NS steps at a time go through three phases -- all keys and values, then all gathers, then the
    // folds in stored order.  NS = 1 measured fastest (ct20stif stand-in P = 2: NS 1 / 2 / 3 / 4 =
    // 8.7 / 8.8 / 9.5 / 11.1 us; ldoor 1/8 shard 11.4 / 13.1 / 13.7 / 16.3 us,
    // profiles/archive/r03_splitns_*.log): a longer phase only adds clamped duplicate rows at the slice end.
#ifndef VBC_SPLIT_NS
#define VBC_SPLIT_NS 1
#endif
    constexpr int NS = VBC_SPLIT_NS;
    if constexpr ((MODE == 2 || MODE == 3) && !KC && DIAG == 0) {
        constexpr int NB = split_batch_runs<T, W_, RUN>();
        constexpr bool NT = MODE == 3;  // a layout larger than the Infinity Cache streams non-temporally
        // (a form that issues batch i+1's keys with batch i's values measured slower: 248 VGPRs, ct20stif
        // strict 9.1 -> 11.5 us, 'min blocks' 14.7 -> 15.4 us, profiles/r04_ab3_*.log)
        for (int R = a; R < e; R += NB * RUN) {
            uint32_t kk[NB];
            T v[NB][RUN][W_], xv[NB][xrun_slots<T, RUN>()];
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const size_t o = (size_t)min(R + j * RUN, e - RUN) * 64 + lane;
                kk[j] = NT ? __builtin_nontemporal_load(key + o) : key[o];
            }
#pragma unroll
            for (int j = 0; j < NB; j++)
#pragma unroll
                for (int d = 0; d < RUN; d++)
                    ld_row<T, W_, 0, NT>(val + (size_t)min(R + j * RUN + d, e - 1) * 64 * W_, lane, v[j][d]);
#pragma unroll
            for (int j = 0; j < NB; j++) ld_xrun<T, RUN>(xg, kk[j] & imask, xv[j]);
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const bool live = R + j * RUN < e;
                const bool pad = (kk[j] & kPad) != 0;
                T xr[RUN];
                xrun_values<T, RUN>(xv[j], xr);
#pragma unroll
                for (int d = 0; d < RUN; d++) {
                    const bool hole = b.holes && !((kk[j] >> (kHoleShift + d)) & 1u);
                    const T xe = (pad || hole) ? T(0) : xr[d];
#pragma unroll
                    for (int k = 0; k < W_; k++) {
                        const T nv = fmadd(v[j][d][k], xe, acc[k]);
                        acc[k] = live ? nv : acc[k];
                    }
                }
            }
        }
    } else if constexpr (MODE == 1 && !KC && DIAG == 0) {
        uint32_t kA[NR], kB[NR];
        T vA[U][W_], vB[U][W_], xv[NR][xrun_slots<T, RUN>()];
        // rows past the slice are clamped to its last run (loaded, folded as no-ops): no branch in the
        // loop body, so the compiler's waits stay counted
        auto load = [&](int R, uint32_t (&kk)[NR], T (&v)[U][W_]) {
#pragma unroll
            for (int j = 0; j < NR; j++) {
                kk[j] = key[(size_t)min(R + j * RUN, e - RUN) * 64 + lane];
#pragma unroll
                for (int d = 0; d < RUN; d++)
                    ld_row<T, W_, 0, false>(val + (size_t)min(R + j * RUN + d, e - 1) * 64 * W_, lane, v[j * RUN + d]);
            }
        };
        auto gather = [&](const uint32_t (&kk)[NR]) {
#pragma unroll
            for (int j = 0; j < NR; j++) ld_xrun<T, RUN>(xg, kk[j] & imask, xv[j]);
        };
        auto fold = [&](int R, const uint32_t (&kk)[NR], const T (&v)[U][W_]) {
#pragma unroll
            for (int j = 0; j < NR; j++) {
                const bool live = R + j * RUN < e;
                const bool pad = (kk[j] & kPad) != 0;
                T xr[RUN];
                xrun_values<T, RUN>(xv[j], xr);
#pragma unroll
                for (int d = 0; d < RUN; d++) {
                    const bool hole = b.holes && !((kk[j] >> (kHoleShift + d)) & 1u);
                    const T xe = (pad || hole) ? T(0) : xr[d];
#pragma unroll
                    for (int k = 0; k < W_; k++) {
                        const T nv = fmadd(v[j * RUN + d][k], xe, acc[k]);
                        acc[k] = live ? nv : acc[k];
                    }
                }
            }
        };
        load(a, kA, vA);
        for (int R = a; R < e; R += 2 * U) {
            gather(kA);
            load(R + U, kB, vB);
            fold(R, kA, vA);
            gather(kB);
            load(R + 2 * U, kA, vA);
            fold(R + U, kB, vB);
        }
    } else
    for (int R = a; R < e; R += NS * U) {
        uint32_t kk[NS][NR], bs[NS][NR];
        T v[NS][U][W_], xv[NS][NR][xrun_slots<T, RUN>()];
#pragma unroll
        for (int t = 0; t < NS; t++)
#pragma unroll
            for (int j = 0; j < NR; j++) {
                const int Rk = min(R + t * U + j * RUN, e - RUN);
                if constexpr (KC) {
                    kk[t][j] = (uint32_t)(int32_t)((gptr<const int16_t>)key)[(size_t)doffs[Rk] + lane];
                    bs[t][j] = bases[Rk];
                } else {
                    kk[t][j] = DIAG != 4 ? key[(size_t)Rk * 64 + lane] : __builtin_nontemporal_load(key + (size_t)Rk * 64 + lane);
                    bs[t][j] = 0;
                }
#pragma unroll
                for (int d = 0; d < RUN; d++)
                    ld_row<T, W_, 0, DIAG == 4>(val + (size_t)min(R + t * U + j * RUN + d, e - 1) * 64 * W_, lane, v[t][j * RUN + d]);
            }
#pragma unroll
        for (int t = 0; t < NS; t++)
#pragma unroll
            for (int j = 0; j < NR; j++) {
                const uint32_t gi = KC ? (bs[t][j] & kSlotIdx) + (kk[t][j] == kPad16 ? 0u : kk[t][j]) : kk[t][j] & imask;
                if constexpr (DIAG == 1) {
#pragma unroll
                    for (int d = 0; d < xrun_slots<T, RUN>(); d++) xv[t][j][d] = T(1) + T(gi & 1);
                } else {
                    ld_xrun<T, RUN>(xg, DIAG == 2 ? (gi & 0xFFu) : gi, xv[t][j]);
                }
            }
#pragma unroll
        for (int t = 0; t < NS; t++)
#pragma unroll
            for (int j = 0; j < NR; j++) {
                const bool live = R + t * U + j * RUN < e;
                const bool pad = KC ? kk[t][j] == kPad16 : (kk[t][j] & kPad) != 0;
                T xr[RUN];
                xrun_values<T, RUN>(xv[t][j], xr);
#pragma unroll
                for (int d = 0; d < RUN; d++) {
                    const bool hole = !KC && b.holes && !((kk[t][j] >> (kHoleShift + d)) & 1u);
                    const T xe = (pad || hole) ? T(0) : xr[d];
#pragma unroll
                    for (int k = 0; k < W_; k++) {
                        const T nv = fmadd(v[t][j * RUN + d][k], xe, acc[k]);
                        acc[k] = live ? nv : acc[k];
                    }
                }
            }
    }
    if (wv > 0) {
#pragma unroll
        for (int k = 0; k < W_; k++) part[((wv - 1) * W_ + k) * 64 + lane] = acc[k];
    }
    __syncthreads();
    if (wv != 0) return;
#pragma unroll
    for (int q = 0; q < P - 1; q++)
#pragma unroll
        for (int k = 0; k < W_; k++) acc[k] += part[(q * W_ + k) * 64 + lane];
    // stripes cut into ks parts (SlotBin::ks): part h of stripe i sits in lane h * m + i; a fixed tree
    // over the lanes (m apart, then 2m, ...) sums them, the same order for every stripe and every call
    const int m = b.ks > 1 ? 64 / b.ks : 64;
    for (int d = m; d < 64; d *= 2)
#pragma unroll
        for (int k = 0; k < W_; k++) acc[k] += __shfl_xor(acc[k], d, 64);
    if (lane >= m) return;
    const int seg = c * m + lane;
    if (seg >= b.nseg) return;
    if (DIAG == 3 && acc[0] != T(-12345.678)) return;
    const int o = b.out_affine ? b.out_base + seg * b.out_stride : G(b.out)[seg];
    gptr<T> yo = G(y) + o;
#pragma unroll
    for (int k = 0; k < W_; k++) {
        if (k < b.wst) {
            T q = alpha * acc[k];
            if (rd_i) q = fmadd(beta, yo[k], q);
            yo[k] = q;
        }
    }
}

template <typename T, int W_, bool KC, int RUN, int P, int DIAG = 0>
__global__ __launch_bounds__(64 * P) void spmv_planar_split(const SlotBin b, const T *__restrict__ x,
                                                            T *__restrict__ y, T alpha, T beta, int rd_i)
{
    const int c = b.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    if (c >= b.nranges) return;
    __shared__ T part[(P > 1 ? P - 1 : 1) * 64 * W_];
    const SplitView v{b.rrow, b.key, b.val, b.base, b.kdoff, b.out, b.nseg, b.out_affine, b.out_base, b.out_stride, b.wst,
                      b.holes, b.ks};
    if (!KC && DIAG == 0 && b.deep == 1)  // SlotBin::deep on a split bin: 1 pipelined, 2 batched slice loop
        split_chunk<T, W_, KC, RUN, P, DIAG, 1>(v, c, threadIdx.x >> 6, threadIdx.x & 63, x, y, alpha, beta, rd_i, part);
    else if (!KC && DIAG == 0 && b.deep == 2)
        split_chunk<T, W_, KC, RUN, P, DIAG, 2>(v, c, threadIdx.x >> 6, threadIdx.x & 63, x, y, alpha, beta, rd_i, part);
    else if (!KC && DIAG == 0 && b.deep == 3)
        split_chunk<T, W_, KC, RUN, P, DIAG, 3>(v, c, threadIdx.x >> 6, threadIdx.x & 63, x, y, alpha, beta, rd_i, part);
    else
        split_chunk<T, W_, KC, RUN, P, DIAG>(v, c, threadIdx.x >> 6, threadIdx.x & 63, x, y, alpha, beta, rd_i, part);
}

// ONE launch for every split bin of a small mixed-width matrix (Launch::fuse_split): workgroup c is
// chunk c of the concatenated bins; the part holding it is found by a scalar scan of the (<= 8) parts,
// all kernel arguments, so no descriptor load precedes the chunk's first key load.  Each wave runs
// the split body of its part's width and row run (a switch, every workgroup one case).  A matrix of
// several width buckets then costs one launch instead of one per planar bucket plus the slotted and
// merge launches (the ct20stif stand-in's strict stripes have widths 1..6).
template <typename T, int P, int MODE>
__global__ __launch_bounds__(64 * P) void spmv_split_multi(const SplitMulti M, const T *__restrict__ x,
                                                           T *__restrict__ y, T alpha, T beta, int rd_i)
{
    const int c = blockIdx.x;
    if (c >= M.nchunks) return;
    int i = 0;
#pragma unroll
    for (int k = 1; k < kSplitParts; k++) i = (k < M.nparts && M.p[k].chunk0 <= c) ? k : i;
    i = __builtin_amdgcn_readfirstlane(i);
    int w = 0, run = 0, chunk0 = 0;
    SplitView v{};
    // a switch over the part index keeps every field a kernel argument (no dynamic indexing)
#define VBC_PART(K)                                                                                               \
    case K: {                                                                                                     \
        const SplitPart &q = M.p[K];                                                                              \
        w = q.w; run = q.run; chunk0 = q.chunk0;                                                                  \
        v = SplitView{q.rrow, q.key, q.val, nullptr, nullptr, q.out, q.nseg, q.out_affine, q.out_base, q.out_stride, q.wst, q.holes, q.ks}; \
        break;                                                                                                    \
    }
    switch (i) {
        VBC_PART(0) VBC_PART(1) VBC_PART(2) VBC_PART(3) VBC_PART(4) VBC_PART(5) VBC_PART(6) VBC_PART(7)
        VBC_PART(8) VBC_PART(9) VBC_PART(10) VBC_PART(11) VBC_PART(12) VBC_PART(13) VBC_PART(14) VBC_PART(15)
    }
#undef VBC_PART
    __shared__ T part[(P > 1 ? P - 1 : 1) * 64 * 8];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, cc = c - chunk0;
#define VBC_WR(W, R) \
    case W * 4 + R: split_chunk<T, W, false, R, P, 0, MODE>(v, cc, wv, lane, x, y, alpha, beta, rd_i, part); break;
    switch (w * 4 + run) {
        VBC_WR(1, 1) VBC_WR(2, 1) VBC_WR(3, 1) VBC_WR(4, 1) VBC_WR(5, 1) VBC_WR(6, 1) VBC_WR(7, 1) VBC_WR(8, 1)
        VBC_WR(1, 2) VBC_WR(2, 2) VBC_WR(3, 2) VBC_WR(4, 2) VBC_WR(5, 2) VBC_WR(6, 2) VBC_WR(7, 2) VBC_WR(8, 2)
        VBC_WR(1, 3) VBC_WR(2, 3) VBC_WR(3, 3) VBC_WR(4, 3) VBC_WR(5, 3) VBC_WR(6, 3) VBC_WR(7, 3) VBC_WR(8, 3)
    default: break;
    }
#undef VBC_WR
}

}  // namespace vbc
