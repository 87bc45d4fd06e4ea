// gfx950 slotted-segment SpMV kernel (device code, included by vbc_slots.hip only).
//
// The merge kernel of vbc_kernels.h handles any segment-length distribution, at the price of a
// segmented scan per tile.  When a width bucket's segments have near-uniform lengths (mesh operators:
// every stripe of a 2-dof 5-point stencil stores 10 rows, every row of its forward product 5 blocks)
// a *slotted* layout needs no scan at all: RPI consecutive segments form a *chunk*, segment s of the
// chunk owns slot s (LPR lanes) for the whole chunk, and the chunk's rows are stored row-major over the
// slots -- row q of the chunk is the q-th entry of every segment, RPI * w contiguous values, so each
// load instruction of a wave is one contiguous sweep exactly as in the tiled stream.  A slot folds its
// segment's entries serially in stored (reference) row order and writes the result once at the
// chunk's end.  Segments shorter than the chunk's longest are padded with PAD rows (key bit 31: x is
// taken as 0, so a padding row never meets an Inf/NaN of x); the last row of every chunk carries LAST
// (bit 30), which the wave reads from lane 0 to close the chunk.  Ranges (one wave each) are runs of
// whole chunks balanced by rows; nothing crosses a range, so there is no fix-up pass.
//   kind 0, mul!(y, B', x)  (multiply_1DVBC.jl:90-134): segment = stripe, entry = stored row;
//       slot lanes hold V columns each, y[col0 : col0+w-1] = alpha * acc (+ beta * y).
//   kind 1, mul!(y, B, x)   (multiply_1DVBC.jl:13-83): segment = output row, entry = (row, stripe)
//       block; the slot's lanes gather x[j + sub*V ...], fold per column and sum across the slot.
#pragma once
#include "vbc_kernels.h"

namespace vbc {

template <typename T, int V>
__device__ __forceinline__ T slot_reduce(const T (&v)[V], int lane, int sub, int LPR)
{
    T s = T(0);
#pragma unroll
    for (int e = 0; e < V; e++) s += v[e];
    for (int d = 1; d < LPR; d <<= 1) {
        const T t = __shfl(s, (lane + d) & 63, 64);
        if (sub + d < LPR) s += t;
    }
    return s;
}

// U rows per pipeline step; FASTE: every bin affine and beta = 0 (no loads on the write path).
// DIAG (ablation builds only): 1 = no y stores (results folded into one store per wave), 2 = no
// x gathers (x taken as 1), 3 = non-temporal y stores, 4 = y stores to one per-wave (cached) block.
// NB > 0 (FASTE launches whose bins are all `contig`): finished chunks are staged in LDS, NB at a
// time, and written as one contiguous run of y with 16-B stores -- longer write bursts, NB times
// fewer write events interleaved with the load stream.
// KC: compressed keys -- a scalar per-row base (LAST in bit 30) plus an int16 delta per slot
// (INT16_MIN marks padding): 2 index bytes per entry instead of 4.
template <typename T, int KIND, int W_, int U, bool FASTE, int DIAG = 0, int NB = 0, bool KC = false>
__device__ __forceinline__ void run_slots(const SlotBin &b, int r, int lane, const T *__restrict__ x,
                                          T *__restrict__ y, T alpha, T beta, bool rd, char *lds_wave, int *lds_out)
{
    constexpr bool kGeneric = (W_ == 0);
    constexpr int V = kGeneric ? 1 : vec_elems(sizeof(T), W_);
    const int w = kGeneric ? b.w : W_;
    const int LPR = kGeneric ? b.w : W_ / V;  // lanes per row (slot-major: lane = slot * LPR + sub)
    const int RPI = b.rpi;
    const int slot = lane / LPR, sub = lane - slot * LPR;
    const bool active = slot < RPI;
    const int R0 = G(b.rrow)[r], R1 = G(b.rrow)[r + 1];
    if (R0 >= R1) return;
    int c = G(b.rchunk)[r];
    const int lslot = active ? slot : 0, lsub = active ? sub : 0;
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const uint32_t> key = G(b.key);
    const gptr<const T> xg = G(x);
    constexpr int XV = KIND == 0 ? 1 : V;

    // Loads are unconditional (rows past the range re-read its last row and are never folded) so
    // the waitcnt pass can count them exactly through the pipeline.
    typedef __attribute__((address_space(4))) const uint32_t *cptr;  // scalar (constant) loads
    const cptr bases = (cptr)b.base;
    const cptr doffs = (cptr)b.kdoff;
    auto load = [&](int R, uint32_t (&kk)[U], uint32_t (&bs)[U], T (&v)[U][V]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int Rc = min(R + u, R1 - 1);
            const size_t p = (size_t)Rc * RPI + lslot;
            if constexpr (KC) {  // shared delta patterns: cached loads
                kk[u] = (uint32_t)(int32_t)((gptr<const int16_t>)key)[(size_t)doffs[Rc] + lslot];
                bs[u] = bases[Rc];
            } else {
                kk[u] = __builtin_nontemporal_load(key + p);
                bs[u] = 0;
            }
            ld_stream<T, V>(val + p * w + lsub * V, v[u]);
        }
    };
    constexpr uint32_t kPad16 = 0xFFFF8000u;  // INT16_MIN sign-extended
    auto gather = [&](const uint32_t (&kk)[U], const uint32_t (&bs)[U], T (&xv)[U][XV]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t gi = KC ? (bs[u] & kSlotIdx) + (kk[u] == kPad16 ? 0u : kk[u]) : kk[u] & kSlotIdx;
#pragma unroll
            for (int e = 0; e < XV; e++) xv[u][e] = DIAG == 2 ? T(1) : xg[gi + (KIND == 0 ? 0 : lsub * V + e)];
        }
    };
    T acc[V], dump[V];
#pragma unroll
    for (int e = 0; e < V; e++) acc[e] = dump[e] = T(0);
    int nbuf = 0, cfirst = c;  // staged chunks (NB > 0) and the first of them
    // Without FASTE the y offset of a segment comes from the table (sorted or non-affine segment
    // orders; bins are cut so a range holds <= kSlotOutEntries segments): the range's entries are staged
    // in LDS by the prologue, so a flush reads LDS (lgkmcnt) and never waits on the vector loads.
    const int c0 = c;
    if constexpr (!FASTE) {
        if (!b.out_affine) {
            const int n = min(kSlotOutEntries, b.nseg - c0 * RPI);
            for (int i = lane; i < n; i += 64) lds_out[i] = G(b.out)[c0 * RPI + i];
        }
    }

    // Staged chunks [cfirst, cfirst + nbuf) -> y: one contiguous run (kind 0: RPI * w values per
    // chunk, kind 1: RPI), valid segments only.
    auto write_out = [&]() {
        const int64_t segs = min((int64_t)nbuf * RPI, (int64_t)b.nseg - (int64_t)cfirst * RPI);
        const int64_t bytes = segs * (KIND == 0 ? w : 1) * (int64_t)sizeof(T);
        char *dst = reinterpret_cast<char *>(y + b.out_base + (int64_t)cfirst * RPI * b.out_stride);
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
        const int seg = c * RPI + slot;
        const bool ok = active && seg < b.nseg;
        if constexpr (NB > 0) {
            if constexpr (KIND == 0) {
                typedef T vt __attribute__((ext_vector_type(V)));
                vt t;
#pragma unroll
                for (int e = 0; e < V; e++) t[e] = alpha * acc[e];
                *reinterpret_cast<vt *>(lds_wave + ((size_t)nbuf * 64 + lane) * V * sizeof(T)) = t;
            } else {
                const T s = slot_reduce<T, V>(acc, lane, sub, LPR);
                if (sub == 0 && active) reinterpret_cast<T *>(lds_wave)[(size_t)nbuf * RPI + slot] = alpha * s;
            }
#pragma unroll
            for (int e = 0; e < V; e++) acc[e] = T(0);
            if (nbuf == 0) cfirst = c;
            c++;
            if (++nbuf == NB) write_out();
            return;
        }
        if constexpr (KIND == 0) {
            if (ok) {
                const int o = (FASTE || b.out_affine) ? b.out_base + seg * b.out_stride : lds_out[(c - c0) * RPI + slot];
                gptr<T> yo = DIAG == 4 ? G(y) + ((size_t)r * 64 + lane) * V : G(y) + o + sub * V;
                const int lim = b.wst - sub * V;  // padding columns (w > wst) are never written
                T q[V];
#pragma unroll
                for (int e = 0; e < V; e++) {
                    q[e] = alpha * acc[e];
                    if (!FASTE && rd && e < lim) q[e] = fmadd(beta, yo[e], q[e]);
                }
                if constexpr (DIAG == 1) {
#pragma unroll
                    for (int e = 0; e < V; e++) dump[e] += q[e];
                } else if (V > 1 && lim >= V) {  // the lane's whole vector: one 8- / 16-B store
                    typedef T vt __attribute__((ext_vector_type(V)));
                    vt t;
#pragma unroll
                    for (int e = 0; e < V; e++) t[e] = q[e];
                    if constexpr (DIAG == 3) __builtin_nontemporal_store(t, (gptr<vt>)yo);
                    else *(gptr<vt>)yo = t;
                } else {
#pragma unroll
                    for (int e = 0; e < V; e++)
                        if (e < lim) yo[e] = q[e];
                }
            }
        } else {
            const T s = slot_reduce<T, V>(acc, lane, sub, LPR);
            if (ok && sub == 0) {
                const int o = (FASTE || b.out_affine) ? b.out_base + seg * b.out_stride : lds_out[(c - c0) * RPI + slot];
                gptr<T> yo = G(y) + o;
                T q = alpha * s;
                if (!FASTE && rd) q = fmadd(beta, *yo, q);
                *yo = q;
            }
        }
#pragma unroll
        for (int e = 0; e < V; e++) acc[e] = T(0);
        c++;
    };
    // Rows past the range (the clamped re-reads of the last step) are folded as no-ops by a select,
    // not skipped by a branch: every loaded register is consumed on every path, so the waitcnt pass
    // never has to drain a dead load at the loop header.
    // R1 copied into a VGPR: a per-lane compare keeps `live` a select (v_cndmask) instead of a
    // scalar branch around the fold.
    int R1v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(R1v) : "s"(R1));
    auto compute = [&](int R, const uint32_t (&kk)[U], const uint32_t (&bs)[U], const T (&v)[U][V],
                       const T (&xv)[U][XV]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool live = R + u < R1v;
            const bool pad = KC ? kk[u] == kPad16 : (kk[u] & kPad) != 0;
#pragma unroll
            for (int e = 0; e < V; e++) {
                const T xe = pad ? T(0) : xv[u][KIND == 0 ? 0 : e];
                const T nv = fmadd(v[u][e], xe, acc[e]);
                acc[e] = live ? nv : acc[e];
            }
            const uint32_t lastw = KC ? bs[u] : (uint32_t)__builtin_amdgcn_readfirstlane((int)kk[u]);
            if (R + u < R1 && (lastw & kLast)) flush();
        }
    };

    // Two-stage ping-pong: the gathers of step i are issued before the stream loads of step i+1.
    // Every path to the loop header has consumed every load it issued, so the header's wait for the
    // keys of the next step is counted (vmcnt(n)), never a drain.
    uint32_t kA[U], kB[U], bA[U], bB[U];
    T vA[U][V], vB[U][V], xv[U][XV];
    load(R0, kA, bA, vA);
    __builtin_amdgcn_s_waitcnt(0);  // prologue drained: the loop header merges the back-edge state only
    for (int R = R0; R < R1; R += 2 * U) {
        gather(kA, bA, xv);
        load(R + U, kB, bB, vB);
        compute(R, kA, bA, vA, xv);
        // no early exit: a half step past the range folds nothing (live = false) and re-reads
        // cached rows, while a break here would leave loads pending on a path to the loop header
        gather(kB, bB, xv);
        load(R + 2 * U, kA, bA, vA);
        compute(R + U, kB, bB, vB, xv);
    }
    if constexpr (NB > 0) {
        if (nbuf > 0) write_out();
    }
    if constexpr (DIAG == 1) {
#pragma unroll
        for (int e = 0; e < V; e++) G(y)[(size_t)(blockIdx.x * kBlockThreads + threadIdx.x) * V + e] = dump[e];
    }
}

// Narrow rows of B'x (w * sizeof(T) < 16: CSC columns for TrSpMV!, fp32 w = 2): one lane holds SPL
// consecutive segments (slots lane*SPL .. lane*SPL+SPL-1), so each row's values are one 16-B load
// per lane and its keys one 4-16-B load; the lane folds SPL segments side by side.  Same pipeline,
// padding, LAST / PAD, staging and y-offset rules as run_slots.
template <typename T, int W_, int SPL, int U, bool FASTE, int NB, bool KC>
__device__ __forceinline__ void run_slots_narrow(const SlotBin &b, int r, int lane, const T *__restrict__ x,
                                                 T *__restrict__ y, T alpha, T beta, bool rd, char *lds_wave,
                                                 int *lds_out)
{
    constexpr int NV = SPL * W_;  // values per lane per row (16 B)
    const int RPI = b.rpi;        // = 64 * SPL
    const int R0 = G(b.rrow)[r], R1 = G(b.rrow)[r + 1];
    if (R0 >= R1) return;
    int c = G(b.rchunk)[r];
    const gptr<const T> val = G(static_cast<const T *>(b.val));
    const gptr<const T> xg = G(x);
    typedef __attribute__((address_space(4))) const uint32_t *cptr;
    const cptr bases = (cptr)b.base;
    const cptr doffs = (cptr)b.kdoff;
    typedef T vt __attribute__((ext_vector_type(NV)));
    auto load = [&](int R, uint32_t (&kk)[U][SPL], uint32_t (&bs)[U], T (&v)[U][NV]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int Rc = min(R + u, R1 - 1);
            const size_t p = (size_t)Rc * RPI + (size_t)lane * SPL;
            if constexpr (KC) {
                typedef int16_t hv __attribute__((ext_vector_type(SPL)));
                const hv d = *(gptr<const hv>)((gptr<const int16_t>)b.key + (size_t)doffs[Rc] + (size_t)lane * SPL);
#pragma unroll
                for (int k = 0; k < SPL; k++) kk[u][k] = (uint32_t)(int32_t)d[k];
                bs[u] = bases[Rc];
            } else {
                typedef uint32_t kv __attribute__((ext_vector_type(SPL)));
                const kv d = __builtin_nontemporal_load((gptr<const kv>)(G(b.key) + p));
#pragma unroll
                for (int k = 0; k < SPL; k++) kk[u][k] = d[k];
                bs[u] = 0;
            }
            const vt t = __builtin_nontemporal_load((gptr<const vt>)(val + p * W_));
#pragma unroll
            for (int e = 0; e < NV; e++) v[u][e] = t[e];
        }
    };
    constexpr uint32_t kPad16 = 0xFFFF8000u;
    auto is_pad = [&](uint32_t k) { return KC ? k == kPad16 : (k & kPad) != 0; };
    auto gather = [&](const uint32_t (&kk)[U][SPL], const uint32_t (&bs)[U], T (&xv)[U][SPL]) {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int k = 0; k < SPL; k++) {
                const uint32_t gi = KC ? (bs[u] & kSlotIdx) + (kk[u][k] == kPad16 ? 0u : kk[u][k]) : kk[u][k] & kSlotIdx;
                xv[u][k] = xg[gi];
            }
    };
    T acc[NV];
#pragma unroll
    for (int e = 0; e < NV; e++) acc[e] = T(0);
    int nbuf = 0, cfirst = c;
    const int c0 = c;
    if constexpr (!FASTE) {
        if (!b.out_affine) {
            const int n = min(kSlotOutEntries, b.nseg - c0 * RPI);
            for (int i = lane; i < n; i += 64) lds_out[i] = G(b.out)[c0 * RPI + i];
        }
    }
    auto write_out = [&]() {  // staged chunks -> one contiguous run of y (RPI * w values per chunk)
        const int64_t segs = min((int64_t)nbuf * RPI, (int64_t)b.nseg - (int64_t)cfirst * RPI);
        const int64_t bytes = segs * W_ * (int64_t)sizeof(T);
        char *dst = reinterpret_cast<char *>(y + b.out_base + (int64_t)cfirst * RPI * b.out_stride);
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
        if constexpr (NB > 0) {
            vt t;
#pragma unroll
            for (int e = 0; e < NV; e++) t[e] = alpha * acc[e];
            *reinterpret_cast<vt *>(lds_wave + ((size_t)nbuf * 64 + lane) * 16) = t;
            if (nbuf == 0) cfirst = c;
        } else {
            const int seg0 = c * RPI + lane * SPL;
            if (FASTE && b.out_stride == W_ && seg0 + SPL <= b.nseg) {  // the lane's SPL segments are adjacent in y
                vt t;
#pragma unroll
                for (int e = 0; e < NV; e++) t[e] = alpha * acc[e];
                *(gptr<vt>)(G(y) + b.out_base + (int64_t)seg0 * W_) = t;
            } else {
#pragma unroll
                for (int k = 0; k < SPL; k++) {
                    const int seg = seg0 + k;
                    if (seg < b.nseg) {
                        const int o = (FASTE || b.out_affine) ? b.out_base + seg * b.out_stride
                                                              : lds_out[(c - c0) * RPI + lane * SPL + k];
                        const int lim = b.wst;
#pragma unroll
                        for (int e = 0; e < W_; e++) {
                            if (e >= lim) break;
                            T q = alpha * acc[k * W_ + e];
                            if (!FASTE && rd) q = fmadd(beta, G(y)[o + e], q);
                            G(y)[o + e] = q;
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int e = 0; e < NV; e++) acc[e] = T(0);
        c++;
        if constexpr (NB > 0) {
            if (++nbuf == NB) write_out();
        }
    };
    int R1v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(R1v) : "s"(R1));
    auto compute = [&](int R, const uint32_t (&kk)[U][SPL], const uint32_t (&bs)[U], const T (&v)[U][NV],
                       const T (&xv)[U][SPL]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool live = R + u < R1v;
#pragma unroll
            for (int k = 0; k < SPL; k++) {
                const T xe = is_pad(kk[u][k]) ? T(0) : xv[u][k];
#pragma unroll
                for (int e = 0; e < W_; e++) {
                    const T nv = fmadd(v[u][k * W_ + e], xe, acc[k * W_ + e]);
                    acc[k * W_ + e] = live ? nv : acc[k * W_ + e];
                }
            }
            const uint32_t lastw = KC ? bs[u] : (uint32_t)__builtin_amdgcn_readfirstlane((int)kk[u][0]);
            if (R + u < R1 && (lastw & kLast)) flush();
        }
    };
    uint32_t kA[U][SPL], kB[U][SPL], bA[U], bB[U];
    T vA[U][NV], vB[U][NV], xv[U][SPL];
    load(R0, kA, bA, vA);
    __builtin_amdgcn_s_waitcnt(0);
    for (int R = R0; R < R1; R += 2 * U) {
        gather(kA, bA, xv);
        load(R + U, kB, bB, vB);
        compute(R, kA, bA, vA, xv);
        gather(kB, bB, xv);
        load(R + 2 * U, kA, bA, vA);
        compute(R + U, kB, bB, vB, xv);
    }
    if constexpr (NB > 0) {
        if (nbuf > 0) write_out();
    }
}

// Rows per step of a width: fp32 rows of 16-B lane vectors (w % 4 == 0) take half the launch's U,
// so every width keeps about the same bytes in flight and the kernel's register budget (the max over
// its width cases) stays at the FE width's.
template <typename T>
__host__ __device__ constexpr int slot_step(int w, int U)
{
    return (sizeof(T) == 4 && w > 0 && vec_elems(4, w) == 4) ? U / 2 : U;
}

// WONLY >= 0: every bin of the launch has width WONLY, so only that case is compiled -- the register
// budget is that width's (the all-width switch spilled 83 / ~600 SGPRs in fp64 / fp32, the maximum over
// cases it never runs on FE).
template <typename T, int KIND, int U, bool FASTE, int DIAG = 0, int NB = 0, bool KC = false, int WONLY = -1>
__global__ __launch_bounds__(kBlockThreads) void spmv_slots(const SlotBin *__restrict__ bins, int nbins,
                                                            int total_ranges, int xcd_chunk, const T *__restrict__ x,
                                                            T *__restrict__ y, T alpha, T beta, int rd_i)
{
    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs, so logical block
    // (xcd * xcd_chunk + i) -- a contiguous run of ranges, whose x rows overlap -- runs on one XCD
    // and shares its L2.  xcd_chunk = 0 keeps the identity mapping.
    int blk = blockIdx.x;
    if (xcd_chunk > 0) {
        const int nb = gridDim.x;
        const int xcd = blk & 7, i = blk >> 3;
        const int full = nb & ~7;  // blocks beyond the last full round keep their own index
        if (blk < full) blk = xcd * (full >> 3) + i;
    }
    const int rg = __builtin_amdgcn_readfirstlane((int)(blk * kWavesPerBlock + (threadIdx.x >> 6)));
    if (rg >= total_ranges) return;
    int bi = 0;
    while (bi + 1 < nbins && bins[bi + 1].range0 <= rg) bi++;
    const SlotBin b = bins[bi];
    const int r = rg - b.range0;
    const int lane = threadIdx.x & 63;
    const bool rd = rd_i != 0;
    __shared__ __attribute__((aligned(16))) char stage[NB > 0 ? kWavesPerBlock * NB * 1024 : 16];
    char *lds = stage + (NB > 0 ? (threadIdx.x >> 6) * NB * 1024 : 0);
    __shared__ int outs[FASTE ? 1 : kWavesPerBlock * kSlotOutEntries];
    int *lds_out = outs + (FASTE ? 0 : (threadIdx.x >> 6) * kSlotOutEntries);
    // narrow B'x rows: fp32 w = 2 only (FE fp32 124 -> 115 us); the w = 1 forms (CSC columns,
    // 2 / 4 segments per lane) measured slower than one segment per lane (C4: 90 -> 102 us)
    if constexpr (KIND == 0 && DIAG == 0 && sizeof(T) == 4 && (WONLY < 0 || WONLY == kWonlyNarrow2)) {
        if (WONLY == kWonlyNarrow2 || (b.spl == 2 && b.wkey == 2)) {
            run_slots_narrow<T, 2, 2, U / 2, FASTE, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out);
            return;
        }
    }
    if constexpr (WONLY >= 0 && WONLY != kWonlyNarrow2) {
        run_slots<T, KIND, WONLY, slot_step<T>(WONLY, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds,
                                                                              lds_out);
        return;
    }
    switch (b.wkey) {
    case 0: run_slots<T, KIND, 0, slot_step<T>(0, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out); break;
    case 1: run_slots<T, KIND, 1, slot_step<T>(1, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out); break;
    case 2: run_slots<T, KIND, 2, slot_step<T>(2, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out); break;
    case 3: run_slots<T, KIND, 3, slot_step<T>(3, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out); break;
    case 4: run_slots<T, KIND, 4, slot_step<T>(4, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out); break;
    case 5: run_slots<T, KIND, 5, slot_step<T>(5, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out); break;
    case 6: run_slots<T, KIND, 6, slot_step<T>(6, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out); break;
    case 7: run_slots<T, KIND, 7, slot_step<T>(7, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out); break;
    case 8: run_slots<T, KIND, 8, slot_step<T>(8, U), FASTE, DIAG, NB, KC>(b, r, lane, x, y, alpha, beta, rd, lds, lds_out); break;
    default: break;
    }
}

}  // namespace vbc
