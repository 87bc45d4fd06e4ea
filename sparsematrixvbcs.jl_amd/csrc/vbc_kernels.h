// gfx950 variable-block SpMV kernels (device code, included by vbc_device.hip only).
//
// Merge-based, flat streaming design.  Per width bucket w the stored w-wide rows of
// the product are one stream of *entries*, ordered by output *segment*:
//   kind 0, mul!(y, B', x)  (multiply_1DVBC.jl:90-134, multiply_VBC.jl:93-147, TrSpMV.jl:1-20):
//       segment = stripe, entry = stored row; y[j : j+w-1] += val_row * x[row].
//   kind 1, mul!(y, B, x)   (multiply_1DVBC.jl:13-83, multiply_VBC.jl:7-87):
//       segment = output row i of B, entry = (i, stripe) block; y[i] += val_row · x[j : j+w-1].
// Each entry's 32-bit key holds its gather index (kind 0: x row; kind 1: first x column) and, in
// bit 31, a HEAD flag marking the first entry of a segment.  The stream is cut into tiles of
// RPI x K entries: a wave's 64 lanes form RPI = 64/LPR row *slots* of LPR lanes (V consecutive
// columns per lane, 16 B per lane where w allows); slot s owns the K consecutive entries
// s*K .. s*K+K-1 of the tile, stored k-major so every load instruction is one contiguous, fully
// coalesced sweep of the stream.  A slot accumulates its entries serially (HEAD restarts the sum;
// segments that close inside the slot are written at once), a segmented scan across the slots
// (wavefront shuffles) joins segments that cross slots, and the open segment flows into the next
// tile in registers.  Every wave owns a contiguous range of tiles; a segment is written by the wave
// that holds its HEAD (it applies beta); the partial of a segment continued from an earlier range is
// written to the range's carry slot and added by the fix-up kernel in range order -- results are
// deterministic.  val and keys are read once: non-temporal loads keep x resident in the caches.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "vbc_internal.h"  // VBC_ABL

namespace vbc {

constexpr int kBlockThreads = 256;
constexpr int kWavesPerBlock = kBlockThreads / 64;
constexpr int kTileKDefault = 8;  // entries per slot per tile (runtime choice: 4 or 8)
constexpr int kPipeDefault = 2;   // software-pipeline depth (runtime choice: 2 or 3)
constexpr uint32_t kHead = 0x80000000u;

// Global-address-space views: the Bin's pointers are loaded from memory, so without these the
// compiler emits flat_* accesses (which also count in lgkmcnt and force conservative waits).
template <typename T>
using gptr = __attribute__((address_space(1))) T *;
template <typename T>
__device__ __forceinline__ gptr<T> G(T *p) { return (gptr<T>)p; }
template <typename T>
__device__ __forceinline__ gptr<const T> G(const T *p) { return (gptr<const T>)p; }

// A 16-B (or narrower) piece of y: a plain store, or a non-temporal one when `nt` (SlotBin / TileBin diag
// bit 16 -- the VBC_ABLATION build's A/B of streaming y stores; the product library passes false).
template <typename V>
__device__ __forceinline__ void st_y(gptr<V> p, V v, bool nt)
{
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Fused multiply-add in T (__builtin_fma is the double version: on floats it would widen).
__device__ __forceinline__ float fmadd(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fmadd(double a, double b, double c) { return __builtin_fma(a, b, c); }

// One width bucket of a fused launch (read through the scalar cache).
struct Bin {
    int32_t kind;     // 0: B'x, 1: Bx
    int32_t wkey;     // dispatch width: 1..8, or 0 = runtime width (w > 8)
    int32_t w;        // entry width as laid out (padded: a w = 3 bucket may be stored 4 wide)
    int32_t wst;      // columns actually written (the stripes' width, <= w)
    int32_t rpi;      // slots per tile (64 / lanes-per-entry)
    int32_t range0;   // first range (wave) of this bucket in the launch
    int32_t nranges;  // ranges of this bucket
    int32_t tiles_per_range;
    int32_t ntiles;   // tiles of this bucket
    int32_t tile_k;   // entries per slot per tile (4 or 8)
    int32_t pipe;     // software-pipeline depth (2 or 3)
    int32_t diag;     // ablation variant (0 = production)
    int32_t out_affine;  // 1: out[s] == out_base + s * out_stride (no table lookup)
    int32_t out_base;
    int32_t out_stride;
    const uint32_t *key;  // entries (tile-permuted): HEAD | gather index
    const void *val;      // entries * w values, 16-B aligned
    const int32_t *rseg;  // per range: number of HEADs before the range (segment base)
    const int32_t *out;   // per segment: kind 0 -> first y column; kind 1 -> y row
    void *carry;          // per range: w (kind 0) or 1 (kind 1) partial values
    int32_t *carry_seg;   // per range: continued segment, or -1
};

// One width bucket in the slotted layout (vbc_slots.h): chunks of RPI segments, one slot each.
struct SlotBin {
    int32_t kind;        // 0: B'x, 1: Bx
    int32_t wkey;        // dispatch width: 1..8, or 0 = runtime width (w > 8)
    int32_t w;           // entry width as laid out
    int32_t wst;         // columns actually written (<= w)
    int32_t rpi;         // slots per chunk
    int32_t range0;      // first range (wave) of this bucket in the launch
    int32_t nranges;
    int32_t nseg;        // segments (the last chunk may be partial)
    int32_t out_affine;  // 1: out[s] == out_base + s * out_stride
    int32_t out_base;
    int32_t out_stride;
    int32_t u;           // rows per pipeline step of the launch (4 / 8 fp64, 8 / 16 fp32)
    int32_t diag;        // ablation variant (0 = production)
    int32_t contig;      // affine and chunk outputs contiguous in y (LDS-staged writes allowed)
    int32_t kc;          // compressed keys: per-row base + int16 per-slot deltas
    int32_t spl;         // segments per lane (narrow B'x rows: 16 / (w * sizeof(T))), else 1
    int32_t planar;      // 1: planar chunk rows (vbc_planar.h: one stripe per lane, column groups)
    int32_t run;         // planar: every segment's rows come in runs of `run` consecutive x rows (1 = none);
                         // keys / LAST are read from each run's first row, x gathered `run` elements wide
    int32_t split;       // planar: > 1 = one chunk per workgroup of `split` waves, each folding a slice of
                         // the chunk's rows, partials summed in LDS (small matrices: more waves in flight)
    int32_t pair;        // planar fp64 w = 3, run = 3: a lane pair per stripe, 32 stripes per chunk, rows =
                         // run-rows of 288 values (vbc_planar.h run_pair)
    int32_t xcd;         // planar: XCD-contiguous workgroup order (xcd_block)
    int32_t holes;       // planar split runs with holes: a run's first key holds, in bits 27..29, which of its
                         // RUN rows the stripe stores (the others: zero values, x taken as 0); index bits 0..26
    int32_t fused;       // planar split bin run inside the fused split launch (Launch::multi), not on its own
    int32_t ks;          // planar split: > 1 = every stripe cut into ks parts of whole runs, part h of the
                         // chunk's stripe i in lane h * (64 / ks) + i (long stripes of the fused split; the
                         // parts are summed across lanes before the store), out / nseg per stripe
    int32_t mask;        // planar: chunk-local length order (lanes of a chunk by decreasing length, the chunk's
                         // 64 stripes kept) and nlive[row] = live lanes of the chunk row; dead lanes read
                         // lane 0's key and values (no extra lines fetched) and fold nothing (vbc_planar.h)
    const uint32_t *key;   // rows * rpi: PAD | LAST | gather index  (kc: int16 deltas, INT16_MIN = PAD)
    const uint32_t *base;  // kc: per row, LAST | base gather index
    const uint32_t *kdoff; // kc: per row, offset (int16 units) of its delta pattern in key
    const void *val;       // rows * rpi * w values
    const int32_t *out;    // per segment (when not affine)
    const int32_t *rrow;   // per range: first row, nranges + 1 entries
    const int32_t *rchunk; // per range: first chunk
    const uint32_t *nlive; // mask: per row, live lanes (a prefix: lanes are in decreasing length order)
    // lanes (planar B'x, vbc_planar.h run_planar_lanes): per-lane compacted streams.  A tile is a run of
    // consecutive stripes dealt to the 64 lanes as contiguous sub-blocks balanced by rows; rchunk[r] is
    // the range's first tile, rrow[r] its first row.
    int32_t lanes;         // 1: per-lane streams (then mask = 1: nlive per row, dead lanes a suffix)
    int32_t ntiles;
    int32_t deep;          // lanes: 1 = keys two steps ahead, gathers one step ahead of their fold
    int32_t nowonly;       // slotted: 1 = keep the all-width kernel even when every bin has one width (A/B)
    const int32_t *trow;   // ntiles + 1: first row of each tile
    const int32_t *tseg;   // ntiles + 1: first segment of each tile
    const int16_t *lseg;   // ntiles * 64: lane's first segment inside its tile (== stripes of the tile: none)
    int32_t dot;           // pair layout of a forward product (vbc_planar.h run_pair DOT): per block, each output
                           // row's dot product with the x slice is added to its sum (the reference's forward order)
    int32_t pad_dot;
};

// Runs with holes (SlotBin::holes): the run's stored-row mask above the gather index of its first key.
constexpr uint32_t kHoleIdx = (1u << 27) - 1;
constexpr int kHoleShift = 27;

// The parts of a fused split launch (vbc_planar.h spmv_split_multi): up to kSplitParts planar split
// bins of a small matrix, their chunks concatenated (part k owns chunks [chunk0, next chunk0)).  A width
// bucket may give up to three parts (its stripes cut into ks = 1, 2 or 4 parts, SlotBin::ks).
constexpr int kSplitParts = 16;
struct SplitPart {
    int32_t w, run, chunk0, nseg, out_affine, out_base, out_stride, wst, holes, ks;
    const int32_t *rrow;
    const uint32_t *key;
    const void *val;
    const int32_t *out;
};
struct SplitMulti {
    int32_t nparts, nchunks, pad0, pad1;
    SplitPart p[kSplitParts];
};

// XCD-aware workgroup order: the hardware deals workgroups round-robin over the 8 XCDs, so logical
// block xcd * (nb / 8) + i -- a contiguous run of ranges, whose x gathers overlap -- is given to the
// workgroups of one XCD, which share its L2.  Blocks past the last full round keep their index.
__device__ __forceinline__ int xcd_block(int blk, int nb)
{
    const int full = nb & ~7;
    return blk < full ? (blk & 7) * (full >> 3) + (blk >> 3) : blk;
}

__device__ __forceinline__ int out_of_slots(const SlotBin &b, int seg)
{
    return b.out_affine ? b.out_base + seg * b.out_stride : G(b.out)[seg];
}

constexpr uint32_t kPad = 0x80000000u;   // slotted layout: padding row (x taken as 0)
constexpr uint32_t kLast = 0x40000000u;  // slotted layout: last row of a chunk
constexpr uint32_t kSlotIdx = 0x3FFFFFFFu;
constexpr int kSlotOutEntries = 1024;  // y offsets per range of a table-mapped slotted bin (LDS-staged)
constexpr int64_t kSlotIdxLimit = int64_t(1) << 30;  // gather indices of the slotted layout (30 bits)

// One width bucket in the row-swept layout (vbc_sweep.hip): tiles of S consecutive segments (B'x:
// stripes; Bx: output rows) whose y accumulators live in LDS; a tile's entries are packed into 64-lane
// steps in ascending gather order (no segment twice in a step), so the whole grid sweeps x front to
// back and the gathers of the concurrently resident waves fall into a narrow window of x.
struct SweepBin {
    int32_t kind;        // 0: B'x (segment = stripe, w outputs), 1: Bx (segment = output row)
    int32_t pad_;
    int32_t w;           // entry width (1..8)
    int32_t tile0;       // first tile (wave) of this bucket in the launch
    int32_t ntiles;
    int32_t S;           // stripes per tile (the last tile may hold fewer)
    int32_t nseg;        // stripes of the bucket
    int32_t out_affine;  // 1: out[s] == out_base + s * out_stride
    int32_t out_base;
    int32_t out_stride;
    int32_t packed;      // 1: key = PAD | segment << lbits | (gather index - sbase[step]), one 32-bit load
    int32_t lbits;       // packed: bits of the gather-index delta (31 - bits of the segment)
    const int32_t *tstep;  // ntiles + 1: first step of each tile
    const uint32_t *key;   // steps * 64: PAD | gather index (B'x: x row; Bx: first x column), or packed
    const uint16_t *loc;   // steps * 64: segment within the tile (not packed)
    const uint32_t *sbase; // packed: steps: the step's smallest gather index (its first lane's)
    const void *val;       // steps * 64 * w values
    const int32_t *out;    // per stripe: first y column (when not affine)
};
constexpr int kSweepTileBytes = 8192;  // LDS accumulators per wave: VBC_SWEEP_TILE = 8 / 16 / 32 (KB)

// Launches spmv_sweep (vbc_sweep.hip): returns the hipError_t of the launch.
int launch_sweep(int esz, int kind, const SweepBin *d_bins, int nbins, int total_tiles, int tile_bytes, int diag, const void *x,
                 void *y, double alpha, double beta, bool rd, hipStream_t stream);

constexpr int kWonlyNarrow2 = 102;  // spmv_slots WONLY: fp32 B'x w = 2 folded two segments per lane (run_slots_narrow)
// Launches spmv_slots (vbc_slots.hip): returns the hipError_t of the launch.
int launch_slots(int esz, int kind, const SlotBin *d_bins, int nbins, int total_ranges, bool faste, int xcd, int u, int diag, int stage, bool kc,
                 int wonly, const void *x, void *y, double alpha, double beta, bool rd, hipStream_t stream);
int occupancy_slots(int esz, int kind);
// vbc_planar.hip
int launch_planar(int esz, const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                  double alpha, double beta, bool rd, hipStream_t s);
int occupancy_planar(int esz);
int occupancy_split_multi(int esz, int P);
int launch_split_multi(int esz, const SplitMulti &M, int P, const void *x, void *y, double alpha, double beta, bool rd,
                       hipStream_t s);
int occupancy_lanes(int esz);

__host__ __device__ constexpr int vec_elems(int esz, int w)
{
    return esz == 8 ? (w % 2 == 0 ? 2 : 1) : (w % 4 == 0 ? 4 : (w % 2 == 0 ? 2 : 1));
}

// Grouped tile layout.  Keys: each lane's 4 consecutive entries (k = 4g .. 4g+3) are contiguous, one
// 16-B load: entry (slot s, k) of a tile at (k/4)*RPI*4 + s*4 + k%4.  Values: when one lane holds a
// whole row (LPR = 1) narrower than 16 B, G = 16 / (V*esz) consecutive entries of the lane are
// contiguous (entry at (k/G)*RPI*G + s*G + k%G) so those loads are 16 B too; otherwise G = 1.
constexpr int kKeyGroup = 4;
__host__ __device__ constexpr int val_group(int esz, int w)
{
    return (w >= 1 && w <= 8 && w / vec_elems(esz, w) == 1 && vec_elems(esz, w) * esz < 16)
               ? 16 / (vec_elems(esz, w) * esz) : 1;
}
__host__ __device__ constexpr size_t key_pos(size_t tile_base, int k, int s, int RPI)
{
    return tile_base + (size_t)(k / kKeyGroup) * RPI * kKeyGroup + (size_t)s * kKeyGroup + (k % kKeyGroup);
}
__host__ __device__ constexpr size_t val_pos(size_t tile_base, int k, int s, int RPI, int G)
{
    return tile_base + (size_t)(k / G) * RPI * G + (size_t)s * G + (k % G);
}

template <typename T, int V>
__device__ __forceinline__ void ld_stream(gptr<const T> p, T (&r)[V])
{
    if constexpr (V == 1) {
        r[0] = __builtin_nontemporal_load(p);
    } else {
        typedef T vt __attribute__((ext_vector_type(V)));
        const vt t = __builtin_nontemporal_load((gptr<const vt>)p);
#pragma unroll
        for (int e = 0; e < V; e++) r[e] = t[e];
    }
}

// DPP moves (VALU, no LDS traffic): CTRL = row_shr:n (0x110+n), row_bcast:15 (0x142),
// row_bcast:31 (0x143), wave_shr:1 (0x138); lanes outside RM rows / the row receive 0.
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp32(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM, typename T>
__device__ __forceinline__ T dppv(T v)
{
    if constexpr (sizeof(T) == 8) {
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        const uint64_t lo = dpp32<CTRL, RM>((uint32_t)u), hi = dpp32<CTRL, RM>((uint32_t)(u >> 32));
        return __builtin_bit_cast(T, lo | (hi << 32));
    } else {
        return __builtin_bit_cast(T, dpp32<CTRL, RM>(__builtin_bit_cast(uint32_t, v)));
    }
}
template <typename T>
__device__ __forceinline__ T readlane(T v, int l)
{
    if constexpr (sizeof(T) == 8) {
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        const uint64_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
        const uint64_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
        return __builtin_bit_cast(T, lo | (hi << 32));
    } else {
        return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
    }
}
// One step of the segmented inclusive scan (f = segment restarts here).
template <int CTRL, int RM, typename T, int V>
__device__ __forceinline__ void seg_step(bool cond, bool &f, T (&s)[V])
{
    const bool of = dpp32<CTRL, RM>((uint32_t)f) != 0;
    T os[V];
#pragma unroll
    for (int e = 0; e < V; e++) os[e] = dppv<CTRL, RM>(s[e]);
    if (cond) {
        if (!f) {
#pragma unroll
            for (int e = 0; e < V; e++) s[e] += os[e];
        }
        f = f || of;
    }
}

// Kind 1 keeps per-lane column partials; the LPR lanes of a slot (lane stride SS) are summed when a
// segment is written.  Called with the whole slot active (its lanes share every control decision).
template <typename T, int V>
__device__ __forceinline__ T slot_sum(const T (&v)[V], int lane, int sub, int LPR, int SS)
{
    T s = T(0);
#pragma unroll
    for (int e = 0; e < V; e++) s += v[e];
    for (int d = 1; d < LPR; d <<= 1) {
        const T t = __shfl(s, (lane + d * SS) & 63, 64);
        if (sub + d < LPR) s += t;
    }
    return s;
}

// Owner write of one segment: y = alpha * v (+ beta * y).
__device__ __forceinline__ int out_of(const Bin &b, int seg)
{
    return b.out_affine ? b.out_base + seg * b.out_stride : G(b.out)[seg];
}

// FASTE (every bin affine, beta = 0): no loads at all -- a load here would make the waitcnt pass
// drain the software pipeline's in-flight stream at every owner write.
template <typename T, int KIND, int V, bool FASTE = false>
__device__ __forceinline__ void emit(const Bin &b, int seg, const T (&v)[V], int sub, int LPR, int SS, int lane,
                                     T *__restrict__ y, T alpha, T beta, bool rd)
{
    const int o = FASTE ? b.out_base + seg * b.out_stride : out_of(b, seg);
    if constexpr (KIND == 0) {
        gptr<T> yo = G(y) + o + sub * V;
        const int lim = b.wst - sub * V;  // padding columns (w > wst) are never written
#pragma unroll
        for (int e = 0; e < V; e++) {
            if (e >= lim) break;
            T r = alpha * v[e];
            if (!FASTE && rd) r = fmadd(beta, yo[e], r);
            yo[e] = r;
        }
    } else {
        const T s = slot_sum<T, V>(v, lane, sub, LPR, SS);
        if (sub == 0) {
            gptr<T> yo = G(y) + o;
            T r = alpha * s;
            if (!FASTE && rd) r = fmadd(beta, *yo, r);
            *yo = r;
        }
    }
}

// Hand a continued segment's partial to the fix-up pass.
template <typename T, int KIND, int V>
__device__ __forceinline__ void hand_off(const Bin &b, int r, int seg, const T (&v)[V], int sub, int LPR,
                                         int SS, int lane, int w)
{
    if constexpr (KIND == 0) {
        gptr<T> c = G(static_cast<T *>(b.carry)) + (size_t)r * w + sub * V;
#pragma unroll
        for (int e = 0; e < V; e++) c[e] = v[e];
    } else {
        const T s = slot_sum<T, V>(v, lane, sub, LPR, SS);
        if (sub == 0) G(static_cast<T *>(b.carry))[r] = s;
    }
    if (sub == 0) G(b.carry_seg)[r] = seg;
}

// DIAG (ablation builds only; never selected by default): 1 = loads and gathers but no segmented
// reduction (a plain fold keeps the loads live), 2 = no x gathers (x taken as 1).
template <typename T, int KIND, int W_, int K, int P, int DIAG = 0, bool FASTE = false>
__device__ __forceinline__ void run_range(const Bin &b, int r, int lane, const T *__restrict__ x,
                                          T *__restrict__ y, T alpha, T beta, bool rd)
{
    constexpr bool kGeneric = (W_ == 0);
    constexpr int V = kGeneric ? 1 : vec_elems(sizeof(T), W_);
    const int w = kGeneric ? b.w : W_;
    const int LPR = w / V;
    const int RPI = b.rpi;
    // DPP path: compile-time power-of-two slot count filling the wave; lanes are sub-major
    // (lane = sub * RPI + slot) so each column's slots are contiguous lanes for row_shr/row_bcast.
    constexpr int cLPR = kGeneric ? 0 : W_ / V;
    constexpr int cRPI = kGeneric ? 0 : 64 / (cLPR > 0 ? cLPR : 1);
    constexpr bool kDpp = !kGeneric && (cRPI & (cRPI - 1)) == 0 && cRPI * cLPR == 64 && cRPI >= 8;
    const int slot = kDpp ? (lane & (cRPI - 1)) : lane / LPR;
    const int sub = kDpp ? (lane / cRPI) : lane - slot * LPR;
    const int SS = kDpp ? cRPI : 1;  // lane stride between the columns of one slot
    const bool active = kDpp || (slot < RPI && sub < LPR);
    const int t0 = r * b.tiles_per_range;
    const int t1 = min(t0 + b.tiles_per_range, b.ntiles);
    if (t0 >= t1) return;
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> xg_ = G(x);
    const size_t tile_rows = (size_t)RPI * K;

    int seg_base = G(b.rseg)[r];  // segments whose HEAD precedes the current tile
    // A range that does not start at a HEAD continues the segment open before it.
    const bool starts_at_head = (key[(size_t)t0 * tile_rows] & kHead) != 0;
    T carry[V];                // value of the segment open when entering the tile
#pragma unroll
    for (int e = 0; e < V; e++) carry[e] = T(0);
    bool owned = false;        // the open segment's HEAD lies in this range

    // Stage 1: keys and values of a tile (one coalesced sweep per k).  Loads are unconditional --
    // a tile past the range re-reads the range's last tile (never reduced), idle lanes read slot 0
    // and drop it -- so no branch hides them from the waitcnt pass (which would otherwise wait for
    // the whole in-flight stream at the merge).
    const int lslot = active ? slot : 0, lsub = active ? sub : 0;
    constexpr int GV = kGeneric ? 1 : val_group((int)sizeof(T), W_);
    auto load_stream = [&](int t, uint32_t (&kk)[K], T (&v)[K][V]) {
        const size_t tb = (size_t)min(t, t1 - 1) * tile_rows;
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int g = 0; g < K / kKeyGroup; g++) {
            const u4 q = __builtin_nontemporal_load((gptr<const u4>)(key + key_pos(tb, g * kKeyGroup, lslot, RPI)));
#pragma unroll
            for (int i = 0; i < kKeyGroup; i++) kk[g * kKeyGroup + i] = q[i];
        }
        if constexpr (GV == 1) {
#pragma unroll
            for (int k = 0; k < K; k++) ld_stream<T, V>(val + val_pos(tb, k, lslot, RPI, 1) * w + lsub * V, v[k]);
        } else {  // one row per lane, GV entries per 16-B load
            typedef T vt __attribute__((ext_vector_type(GV * V)));
#pragma unroll
            for (int g = 0; g < K / GV; g++) {
                const vt q = __builtin_nontemporal_load((gptr<const vt>)(val + val_pos(tb, g * GV, lslot, RPI, GV) * w));
#pragma unroll
                for (int i = 0; i < GV; i++)
#pragma unroll
                    for (int e = 0; e < V; e++) v[g * GV + i][e] = q[i * V + e];
            }
        }
        if constexpr (!kDpp) {
#pragma unroll
            for (int k = 0; k < K; k++) {
                kk[k] = active ? kk[k] : 0u;
#pragma unroll
                for (int e = 0; e < V; e++) v[k][e] = active ? v[k][e] : T(0);
            }
        }
    };
    // Stage 2: the x gathers of a tile whose keys have arrived (kind 0: one x per entry).
    constexpr int XV = KIND == 0 ? 1 : V;
    // `ok` = the tile lies inside the range (wave-uniform).  A tile past the range is gathered at x[0]
    // and reduced as a tile of zeros without HEADs -- a no-op on every output and on the carried sum --
    // so the pipelined loops below have one exit and straight-line bodies: no branch around a stage,
    // hence no vmcnt(0) drain at the loop header (the slotted kernels' rule).
    auto gather = [&](int t, const uint32_t (&kk)[K], T (&xv)[K][XV], bool ok = true) {
        (void)t;
        if constexpr (DIAG == 2) {
#pragma unroll
            for (int k = 0; k < K; k++)
#pragma unroll
                for (int e = 0; e < XV; e++) xv[k][e] = T(1);
        } else {
#pragma unroll
            for (int k = 0; k < K; k++) {
                const uint32_t gi = ok ? kk[k] & ~kHead : 0u;
                if constexpr (KIND == 0) {
                    xv[k][0] = xg_[gi];
                } else {
#pragma unroll
                    for (int e = 0; e < V; e++) xv[k][e] = xg_[gi + lsub * V + e];
                }
            }
        }
    };
    T diag_acc = T(0);
    // Stage 3: segmented reduction of a tile.
    auto compute = [&](const uint32_t (&kk0)[K], const T (&v0)[K][V], const T (&xv0)[K][XV], bool ok = true) {
        uint32_t kk[K];
        T v[K][V], xv[K][XV];
#pragma unroll
        for (int k = 0; k < K; k++) {  // selects, not a branch (see gather)
            kk[k] = ok ? kk0[k] : 0u;
#pragma unroll
            for (int e = 0; e < V; e++) v[k][e] = ok ? v0[k][e] : T(0);
#pragma unroll
            for (int e = 0; e < XV; e++) xv[k][e] = ok ? xv0[k][e] : T(0);
        }
        if constexpr (DIAG == 1) {
#pragma unroll
            for (int k = 0; k < K; k++)
#pragma unroll
                for (int e = 0; e < V; e++) diag_acc += v[k][e] * xv[k][KIND == 0 ? 0 : e] + (T)(kk[k] & 1);
            return;
        }
        // HEADs per slot and their exclusive prefix over the slots
        int pre = 0, tile_heads = 0;
        if constexpr (kDpp) {  // ballots: every column's copy of the slot flags is identical
            const uint64_t colmask = cRPI == 64 ? ~0ull : ((1ull << cRPI) - 1) << (sub * cRPI);
            const uint64_t below = colmask & ((1ull << lane) - 1);
#pragma unroll
            for (int k = 0; k < K; k++) {
                const uint64_t bal = __ballot((kk[k] >> 31) != 0);
                pre += __popcll(bal & below);
                tile_heads += __popcll(bal & (cRPI == 64 ? ~0ull : (1ull << cRPI) - 1));
            }
        } else {
            int nh = 0;
#pragma unroll
            for (int k = 0; k < K; k++) nh += (int)(kk[k] >> 31);
            pre = nh;
            for (int d = 1; d < RPI; d <<= 1) {
                const int o = __shfl(pre, (lane - d * LPR) & 63, 64);
                if (slot >= d) pre += o;
            }
            tile_heads = __shfl(pre, (RPI - 1) * LPR, 64);
            pre -= nh;
        }

        // lane-serial pass over the slot's K entries: one FMA per column into `cur`; at a HEAD the
        // running sum becomes the slot's lead (first HEAD) or a complete segment (later HEADs).
        T lead[V], cur[V];
#pragma unroll
        for (int e = 0; e < V; e++) lead[e] = cur[e] = T(0);
        int seg = seg_base + pre - 1;  // segment open at the slot's start
        bool seen = false;
#pragma unroll
        for (int k = 0; k < K; k++) {
            if (kk[k] & kHead) {
                if (seen)  // opened and closed inside this slot: owned and complete
                    emit<T, KIND, V, FASTE>(b, seg, cur, sub, LPR, SS, lane, y, alpha, beta, rd);
                else {
#pragma unroll
                    for (int e = 0; e < V; e++) lead[e] = cur[e];
                }
                seg++;
                seen = true;
#pragma unroll
                for (int e = 0; e < V; e++) cur[e] = T(0);
            }
#pragma unroll
            for (int e = 0; e < V; e++) cur[e] = fmadd(v[k][e], xv[k][KIND == 0 ? 0 : e], cur[e]);
        }
        if (!seen) {
#pragma unroll
            for (int e = 0; e < V; e++) {
                lead[e] = cur[e];
                cur[e] = T(0);
            }
        }
        // segmented inclusive scan of (seen, seen ? cur : lead) over the slots
        bool f = seen;
        T s[V];
#pragma unroll
        for (int e = 0; e < V; e++) s[e] = seen ? cur[e] : lead[e];
        bool ef;
        T es[V];
        if constexpr (kDpp) {
            const int ls = lane & (cRPI < 16 ? cRPI - 1 : 15);  // slot position inside a DPP row
            if constexpr (cRPI > 1) seg_step<0x111, 0xF>(ls >= 1, f, s);
            if constexpr (cRPI > 2) seg_step<0x112, 0xF>(ls >= 2, f, s);
            if constexpr (cRPI > 4) seg_step<0x114, 0xF>(ls >= 4, f, s);
            if constexpr (cRPI > 8) seg_step<0x118, 0xF>(ls >= 8, f, s);
            if constexpr (cRPI > 16) seg_step<0x142, 0xA>((lane & 16) != 0, f, s);
            if constexpr (cRPI > 32) seg_step<0x143, 0xC>((lane & 32) != 0, f, s);
            ef = dpp32<0x138, 0xF>((uint32_t)f) != 0;  // wave_shr:1
#pragma unroll
            for (int e = 0; e < V; e++) es[e] = dppv<0x138, 0xF>(s[e]);
        } else {
            for (int d = 1; d < RPI; d <<= 1) {
                const int src = (lane - d * LPR) & 63;
                const bool of = __shfl((int)f, src, 64) != 0;
                T os[V];
#pragma unroll
                for (int e = 0; e < V; e++) os[e] = __shfl(s[e], src, 64);
                if (slot >= d) {
                    if (!f) {
#pragma unroll
                        for (int e = 0; e < V; e++) s[e] += os[e];
                    }
                    f = f || of;
                }
            }
            // value entering each slot (exclusive scan)
            const int srcx = (lane - LPR) & 63;
            ef = __shfl((int)f, srcx, 64) != 0;
#pragma unroll
            for (int e = 0; e < V; e++) es[e] = __shfl(s[e], srcx, 64);
        }
        if (slot == 0) {
            ef = false;
#pragma unroll
            for (int e = 0; e < V; e++) es[e] = T(0);
        }
        // the segment open when entering a slot closes at the slot's first HEAD
        if (active && seen) {
            const int cseg = seg_base + pre - 1;
            const bool from_range = ef || owned;  // its HEAD lies in this range
            if (from_range || !starts_at_head) {
                T tot[V];
#pragma unroll
                for (int e = 0; e < V; e++) tot[e] = (ef ? es[e] : carry[e] + es[e]) + lead[e];
                if (from_range)
                    emit<T, KIND, V, FASTE>(b, cseg, tot, sub, LPR, SS, lane, y, alpha, beta, rd);
                else
                    hand_off<T, KIND, V>(b, r, cseg, tot, sub, LPR, SS, lane, w);
            }
        }
        // flow into the next tile
        bool lf;
        T lsv[V];
        if constexpr (kDpp) {  // last slot of each column: scalar reads
            lf = __builtin_amdgcn_readlane((int)f, cRPI - 1) != 0;
#pragma unroll
            for (int e = 0; e < V; e++) {
                lsv[e] = readlane(s[e], cRPI - 1);
#pragma unroll
                for (int j = 1; j < cLPR; j++) {
                    const T o = readlane(s[e], j * cRPI + cRPI - 1);
                    if (sub == j) lsv[e] = o;
                }
            }
        } else {
            const int last = (RPI - 1) * LPR + sub;
            lf = __shfl((int)f, last, 64) != 0;
#pragma unroll
            for (int e = 0; e < V; e++) lsv[e] = __shfl(s[e], last, 64);
        }
#pragma unroll
        for (int e = 0; e < V; e++) carry[e] = lf ? lsv[e] : carry[e] + lsv[e];
        owned = owned || lf;
        seg_base += tile_heads;
    };

    if constexpr (P == 2) {
        // Two stages, ping-pong buffers: gathers of tile t are issued before the stream loads of
        // tile t+1, so the counted vmcnt wait in compute(t) never waits on the prefetch.
        uint32_t kA[K], kB[K];
        T vA[K][V], vB[K][V], xv[K][XV];
        load_stream(t0, kA, vA);
        for (int t = t0; t < t1; t += 2) {
            const bool ok1 = t + 1 < t1;
            gather(t, kA, xv);
            load_stream(t + 1, kB, vB);
            compute(kA, vA, xv);
            gather(t + 1, kB, xv, ok1);
            load_stream(t + 2, kA, vA);
            compute(kB, vB, xv, ok1);
        }
    } else {
        // Three stages, rotating buffers: in step t the stream loads of tile t+2 and the gathers of
        // tile t+1 are in flight while tile t is reduced.
        uint32_t k0[K], k1[K], k2[K];
        T v0[K][V], v1[K][V], v2[K][V];
        T x0[K][XV], x1[K][XV], x2[K][XV];
        load_stream(t0, k0, v0);
        gather(t0, k0, x0);
        load_stream(t0 + 1, k1, v1);
        for (int t = t0; t < t1; t += 3) {
            const bool ok1 = t + 1 < t1, ok2 = t + 2 < t1, ok3 = t + 3 < t1;
            gather(t + 1, k1, x1, ok1);
            load_stream(t + 2, k2, v2);
            compute(k0, v0, x0);
            gather(t + 2, k2, x2, ok2);
            load_stream(t + 3, k0, v0);
            compute(k1, v1, x1, ok1);
            gather(t + 3, k0, x0, ok3);
            load_stream(t + 4, k1, v1);
            compute(k2, v2, x2, ok2);
        }
    }
    if constexpr (DIAG == 1) {
        if (diag_acc == T(1234.5)) y[lane] = diag_acc;  // keep the loads live
        return;
    }
    // the segment still open at the end of the range
    if (active && slot == 0) {
        const int cseg = seg_base - 1;
        if (owned)
            emit<T, KIND, V, FASTE>(b, cseg, carry, sub, LPR, SS, lane, y, alpha, beta, rd);
        else if (!starts_at_head)  // no HEAD in the whole range: all of it continues cseg
            hand_off<T, KIND, V>(b, r, cseg, carry, sub, LPR, SS, lane, w);
    }
}

#define VBC_W_CASES(KIND)                                                                          \
    case 0: run_range<T, KIND, 0, K, P, DIAG, FASTE>(b, r, lane, x, y, alpha, beta, rd); break;              \
    case 1: run_range<T, KIND, 1, K, P, DIAG, FASTE>(b, r, lane, x, y, alpha, beta, rd); break;                     \
    case 2: run_range<T, KIND, 2, K, P, DIAG, FASTE>(b, r, lane, x, y, alpha, beta, rd); break;                     \
    case 3: run_range<T, KIND, 3, K, P, DIAG, FASTE>(b, r, lane, x, y, alpha, beta, rd); break;                     \
    case 4: run_range<T, KIND, 4, K, P, DIAG, FASTE>(b, r, lane, x, y, alpha, beta, rd); break;                     \
    case 5: run_range<T, KIND, 5, K, P, DIAG, FASTE>(b, r, lane, x, y, alpha, beta, rd); break;                     \
    case 6: run_range<T, KIND, 6, K, P, DIAG, FASTE>(b, r, lane, x, y, alpha, beta, rd); break;                     \
    case 7: run_range<T, KIND, 7, K, P, DIAG, FASTE>(b, r, lane, x, y, alpha, beta, rd); break;                     \
    case 8: run_range<T, KIND, 8, K, P, DIAG, FASTE>(b, r, lane, x, y, alpha, beta, rd); break;

// One wave per range; the wave finds its bucket by a scalar scan of the (few) bins.
template <typename T, int KIND, int K, int P, int DIAG = 0, bool FASTE = false>
__global__ __launch_bounds__(kBlockThreads) void spmv_ranges(const Bin *__restrict__ bins, int nbins,
                                                             int total_ranges, const T *__restrict__ x,
                                                             T *__restrict__ y, T alpha, T beta, int rd_i)
{
    const int rg = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)));
    if (rg >= total_ranges) return;
    int bi = 0;
    while (bi + 1 < nbins && bins[bi + 1].range0 <= rg) bi++;
    const Bin b = bins[bi];
    const int r = rg - b.range0;
    const int lane = threadIdx.x & 63;
    if (lane == 0) G(b.carry_seg)[r] = -1;  // overwritten below when the range continues a segment
    const bool rd = rd_i != 0;
    switch (b.wkey) { VBC_W_CASES(KIND) default: break; }
}

// ---------------------------------------------------------------------------------------------
// Multi-RHS transposed product Y = alpha * B' X + beta * Y over the SAME tiled entry stream.
// X (m x nrhs) and Y (n x nrhs) are row-major (right-hand sides interleaved: X[i * ldx + j]), so
// the NR lanes of a slot gather one contiguous X row.  A wave handles 64/NR slots of a tile per
// pass (in the tile's logical entry order), keeps w accumulators per lane (column c, rhs j), and
// joins segments across the pass's slots with a shuffle scan; the open segment flows from pass to
// pass and tile to tile exactly as in run_range.  Continued segments go to carry_mm (w x NR per
// range) for fixup_mm.
// ---------------------------------------------------------------------------------------------
template <typename T, int W_>
__device__ __forceinline__ void load_row(gptr<const T> p, T (&r)[W_])
{
    constexpr int kVec = (W_ * (int)sizeof(T)) % 16 == 0 ? 16 / (int)sizeof(T) : 1;
    if constexpr (kVec > 1) {
        typedef T vt __attribute__((ext_vector_type(kVec)));
#pragma unroll
        for (int c = 0; c < W_; c += kVec) {
            const vt t = __builtin_nontemporal_load((gptr<const vt>)(p + c));
#pragma unroll
            for (int e = 0; e < kVec; e++) r[c + e] = t[e];
        }
    } else {
#pragma unroll
        for (int c = 0; c < W_; c++) r[c] = __builtin_nontemporal_load(p + c);
    }
}

template <typename T, int W_, int NR, int K>
__device__ __forceinline__ void run_range_mm(const Bin &b, int r, int lane, const T *__restrict__ x, int64_t ldx,
                                             T *__restrict__ y, int64_t ldy, int nrhs, T *__restrict__ carry_mm,
                                             T alpha, T beta, bool rd)
{
    constexpr int SPP = 64 / NR;  // slots per pass
    const int RPI = b.rpi;
    const int sl = lane / NR, j = lane - sl * NR;
    const bool jok = j < nrhs;
    const int t0 = r * b.tiles_per_range;
    const int t1 = min(t0 + b.tiles_per_range, b.ntiles);
    if (t0 >= t1) return;
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> xg = G(x);
    gptr<T> yg = G(y);
    const size_t tile_rows = (size_t)RPI * K;
    int seg_base = G(b.rseg)[r];
    const bool starts_at_head = (key[(size_t)t0 * tile_rows] & kHead) != 0;
    T carry[W_];
#pragma unroll
    for (int c = 0; c < W_; c++) carry[c] = T(0);
    bool owned = false;

    auto emit_mm = [&](int seg, const T (&v)[W_]) {
        if (!jok) return;
        const int o = out_of(b, seg);
#pragma unroll
        for (int c = 0; c < W_; c++) {
            if (c >= b.wst) break;
            gptr<T> yo = yg + (int64_t)(o + c) * ldy + j;
            T q = alpha * v[c];
            if (rd) q = fmadd(beta, *yo, q);
            *yo = q;
        }
    };
    auto hand_mm = [&](int seg, const T (&v)[W_]) {
        gptr<T> c0 = G(carry_mm) + ((size_t)r * W_) * NR + j;
#pragma unroll
        for (int c = 0; c < W_; c++) c0[c * NR] = v[c];
        if (j == 0) G(b.carry_seg)[r] = seg;
    };

    for (int t = t0; t < t1; t++) {
        const size_t base = (size_t)t * tile_rows;
        for (int p = 0; p < RPI; p += SPP) {
            const int s = p + sl;
            const bool sv = s < RPI;
            const int npass = min(SPP, RPI - p);  // valid slots in this pass
            uint32_t kk[K];
            T vv[K][W_], xv[K];
#pragma unroll
            for (int k = 0; k < K; k++) {
                if (sv) {
                    kk[k] = __builtin_nontemporal_load(key + key_pos(base, k, s, RPI));
                    load_row<T, W_>(val + val_pos(base, k, s, RPI, val_group((int)sizeof(T), W_)) * W_, vv[k]);
                } else {
                    kk[k] = 0u;
#pragma unroll
                    for (int c = 0; c < W_; c++) vv[k][c] = T(0);
                }
            }
#pragma unroll
            for (int k = 0; k < K; k++) xv[k] = (sv && jok) ? xg[(int64_t)(kk[k] & ~kHead) * ldx + j] : T(0);
            int nh = 0;
#pragma unroll
            for (int k = 0; k < K; k++) nh += (int)(kk[k] >> 31);
            int pre = nh;
            for (int d = 1; d < SPP; d <<= 1) {
                const int o = __shfl(pre, (lane - d * NR) & 63, 64);
                if (sl >= d) pre += o;
            }
            const int pass_heads = __shfl(pre, (npass - 1) * NR, 64);
            pre -= nh;

            T lead[W_], cur[W_];
#pragma unroll
            for (int c = 0; c < W_; c++) lead[c] = cur[c] = T(0);
            int seg = seg_base + pre - 1;
            bool seen = false;
#pragma unroll
            for (int k = 0; k < K; k++) {
                if (kk[k] & kHead) {
                    if (seen) emit_mm(seg, cur);
                    else {
#pragma unroll
                        for (int c = 0; c < W_; c++) lead[c] = cur[c];
                    }
                    seg++;
                    seen = true;
#pragma unroll
                    for (int c = 0; c < W_; c++) cur[c] = T(0);
                }
#pragma unroll
                for (int c = 0; c < W_; c++) cur[c] = fmadd(vv[k][c], xv[k], cur[c]);
            }
            if (!seen) {
#pragma unroll
                for (int c = 0; c < W_; c++) {
                    lead[c] = cur[c];
                    cur[c] = T(0);
                }
            }
            // segmented scan over the pass's slots (lane stride NR)
            bool f = seen;
            T sc[W_];
#pragma unroll
            for (int c = 0; c < W_; c++) sc[c] = seen ? cur[c] : lead[c];
            for (int d = 1; d < SPP; d <<= 1) {
                const int src = (lane - d * NR) & 63;
                const bool of = __shfl((int)f, src, 64) != 0;
                T os[W_];
#pragma unroll
                for (int c = 0; c < W_; c++) os[c] = __shfl(sc[c], src, 64);
                if (sl >= d) {
                    if (!f) {
#pragma unroll
                        for (int c = 0; c < W_; c++) sc[c] += os[c];
                    }
                    f = f || of;
                }
            }
            const int srcx = (lane - NR) & 63;
            bool ef = __shfl((int)f, srcx, 64) != 0;
            T es[W_];
#pragma unroll
            for (int c = 0; c < W_; c++) es[c] = __shfl(sc[c], srcx, 64);
            if (sl == 0) {
                ef = false;
#pragma unroll
                for (int c = 0; c < W_; c++) es[c] = T(0);
            }
            if (sv && seen) {
                const int cseg = seg_base + pre - 1;
                const bool from_range = ef || owned;
                if (from_range || !starts_at_head) {
                    T tot[W_];
#pragma unroll
                    for (int c = 0; c < W_; c++) tot[c] = (ef ? es[c] : carry[c] + es[c]) + lead[c];
                    if (from_range) emit_mm(cseg, tot);
                    else hand_mm(cseg, tot);
                }
            }
            const int last = (npass - 1) * NR + j;
            const bool lf = __shfl((int)f, last, 64) != 0;
#pragma unroll
            for (int c = 0; c < W_; c++) {
                const T ls = __shfl(sc[c], last, 64);
                carry[c] = lf ? ls : carry[c] + ls;
            }
            owned = owned || lf;
            seg_base += pass_heads;
        }
    }
    if (sl == 0) {
        const int cseg = seg_base - 1;
        if (owned) emit_mm(cseg, carry);
        else if (!starts_at_head) hand_mm(cseg, carry);
    }
}

template <typename T, int NR, int K>
__global__ __launch_bounds__(kBlockThreads) void spmm_ranges(const Bin *__restrict__ bins, int nbins, int total_ranges,
                                                             const T *__restrict__ x, int64_t ldx, T *__restrict__ y,
                                                             int64_t ldy, int nrhs, T *__restrict__ carry_mm, int64_t carry_stride,
                                                             T alpha, T beta, int rd_i)
{
    const int rg = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)));
    if (rg >= total_ranges) return;
    int bi = 0;
    while (bi + 1 < nbins && bins[bi + 1].range0 <= rg) bi++;
    const Bin b = bins[bi];
    const int r = rg - b.range0;
    const int lane = threadIdx.x & 63;
    if (lane == 0) G(b.carry_seg)[r] = -1;
    const bool rd = rd_i != 0;
    T *cm = carry_mm + (size_t)bi * carry_stride;
    switch (b.wkey) {
    case 1: run_range_mm<T, 1, NR, K>(b, r, lane, x, ldx, y, ldy, nrhs, cm, alpha, beta, rd); break;
    case 2: run_range_mm<T, 2, NR, K>(b, r, lane, x, ldx, y, ldy, nrhs, cm, alpha, beta, rd); break;
    case 3: run_range_mm<T, 3, NR, K>(b, r, lane, x, ldx, y, ldy, nrhs, cm, alpha, beta, rd); break;
    case 4: run_range_mm<T, 4, NR, K>(b, r, lane, x, ldx, y, ldy, nrhs, cm, alpha, beta, rd); break;
    case 5: run_range_mm<T, 5, NR, K>(b, r, lane, x, ldx, y, ldy, nrhs, cm, alpha, beta, rd); break;
    case 6: run_range_mm<T, 6, NR, K>(b, r, lane, x, ldx, y, ldy, nrhs, cm, alpha, beta, rd); break;
    case 7: run_range_mm<T, 7, NR, K>(b, r, lane, x, ldx, y, ldy, nrhs, cm, alpha, beta, rd); break;
    case 8: run_range_mm<T, 8, NR, K>(b, r, lane, x, ldx, y, ldy, nrhs, cm, alpha, beta, rd); break;
    default: break;
    }
}

// Fix-up of the multi-RHS product: one thread per (range, rhs); fill list rows per rhs.
template <typename T, int NR>
__global__ __launch_bounds__(kBlockThreads) void fixup_mm(const Bin *__restrict__ bins, int nbins, int total_ranges,
                                                          const int32_t *__restrict__ fill, int nfill,
                                                          T *__restrict__ y, int64_t ldy, int nrhs,
                                                          const T *__restrict__ carry_mm, int64_t carry_stride,
                                                          T alpha, T beta, int rd_i)
{
    const int i = blockIdx.x * kBlockThreads + threadIdx.x;
    const int item = i / NR, j = i % NR;
    if (j >= nrhs) return;
    if (item < total_ranges) {
        int bi = 0;
        while (bi + 1 < nbins && bins[bi + 1].range0 <= item) bi++;
        const Bin &b = bins[bi];
        const int r = item - b.range0;
        const int seg = b.carry_seg[r];
        if (seg < 0 || (r > 0 && b.carry_seg[r - 1] == seg)) return;
        const T *cm = carry_mm + (size_t)bi * carry_stride;
        const int o = out_of(b, seg);
        for (int c = 0; c < b.wst; c++) {
            T s = T(0);
            for (int q = r; q < b.nranges && b.carry_seg[q] == seg; q++) s += cm[((size_t)q * b.w + c) * NR + j];
            T *yo = y + (int64_t)(o + c) * ldy + j;
            *yo = fmadd(alpha, s, *yo);
        }
    } else if (item - total_ranges < nfill) {
        T *yo = y + (int64_t)fill[item - total_ranges] * ldy + j;
        *yo = rd_i ? beta * *yo : T(0);
    }
}

// Fix-up: add every continued-segment partial (summed in range order: deterministic) and apply
// beta to the segments that own no entry (fill list: y indices).
template <typename T, int KIND>
__global__ __launch_bounds__(kBlockThreads) void fixup(const Bin *__restrict__ bins, int nbins, int total_ranges,
                                                       const int32_t *__restrict__ fill, int nfill,
                                                       T *__restrict__ y, T alpha, T beta, int rd_i)
{
    const int i = blockIdx.x * kBlockThreads + threadIdx.x;
    if (i < total_ranges) {
        int bi = 0;
        while (bi + 1 < nbins && bins[bi + 1].range0 <= i) bi++;
        const Bin &b = bins[bi];
        const int r = i - b.range0;
        const int seg = b.carry_seg[r];
        if (seg < 0 || (r > 0 && b.carry_seg[r - 1] == seg)) return;
        const int wc = KIND == 0 ? b.w : 1;            // carry stride (layout width)
        const int wout = KIND == 0 ? b.wst : 1;        // columns written
        T *__restrict__ yo = y + out_of(b, seg);
        for (int c = 0; c < wout; c++) {
            T s = T(0);
            for (int q = r; q < b.nranges && b.carry_seg[q] == seg; q++)
                s += static_cast<const T *>(b.carry)[(size_t)q * wc + c];
            yo[c] = fmadd(alpha, s, yo[c]);
        }
    } else if (i - total_ranges < nfill) {
        T *yo = y + fill[i - total_ranges];
        *yo = rd_i ? beta * *yo : T(0);
    }
}

// y = beta * y (forward products with several width buckets accumulate bucket by bucket).
template <typename T>
__global__ __launch_bounds__(kBlockThreads) void scale(T *__restrict__ y, int64_t n, T beta, int rd_i)
{
    for (int64_t i = blockIdx.x * (int64_t)kBlockThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlockThreads)
        y[i] = rd_i ? beta * y[i] : T(0);
}

}  // namespace vbc
