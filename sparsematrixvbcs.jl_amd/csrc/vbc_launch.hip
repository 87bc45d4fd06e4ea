// libvbc kernel launches of the vector products: merge kernel (vbc_kernels.h) + slotted kernel
// (vbc_slots.hip), their fix-up passes, and the fused vector multi-RHS kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "vbc_handle.h"

namespace vbc {

// Independent launch groups of a B'x launch (each writes its own stripes of y): the swept bins, the
// slotted bins, each planar bin, and the merge kernel with its fix-up (+ the fill list).
int launch_groups(const Launch &L)
{
    int planar = L.fuse_split ? 1 : 0;  // the fused split bins: one launch
    for (const SlotBin &b : L.pbins) planar += L.fuse_split && b.fused ? 0 : 1;
    return (L.sweep_tiles > 0) + (L.slot_ranges > 0) + planar + (L.total_ranges > 0 || L.nfill > 0);
}

// The groups in order: group g of launch_groups() on stream `stream`; g < 0: every group on it.
template <typename T>
static int launch_group(const Launch &L, int kind, const void *x, void *y, double alpha, double beta, bool rd,
                        hipStream_t stream, int xcd, int slot_stage, int g)
{
    const T *xs = static_cast<const T *>(x);
    T *ys = static_cast<T *>(y);
    int gi = 0;  // index of the next group
    auto mine = [&](bool present) {
        if (!present) return false;
        return g < 0 || gi++ == g;
    };
    if (mine(L.sweep_tiles > 0)) {
        const hipError_t e = (hipError_t)launch_sweep((int)sizeof(T), kind, L.d_wbins, (int)L.wbins.size(), L.sweep_tiles,
                                                      L.sweep_tile_bytes, L.sweep_diag, x, y, alpha, beta, rd, stream);
        if (e != hipSuccess) {
            set_error("spmv_sweep launch failed: %s", hipGetErrorString(e));
            return VBC_HIP_ERROR;
        }
    }
    if (mine(L.slot_ranges > 0)) {
        bool faste = !rd, contig = true;
        for (const SlotBin &sb : L.sbins) {
            faste = faste && sb.out_affine;
            contig = contig && sb.contig;
        }
        if (ablation_knob("VBC_NO_FASTE")) faste = false;  // (the VBC_ABLATION build only)
        // auto (-1): B'x stages 8 chunks per write, Bx writes directly -- measured on FE with every
        // variant built twice (tools/ab.py --copies 2): fp64 B'x 192/177 -> 184/172 us staged,
        // fp64 Bx 186 -> 198 and fp32 Bx 142 -> 157 us staged
        int stage = slot_stage;
        if (stage < 0) stage = kind == 0 ? 8 : 0;
        if (!(faste && contig)) stage = 0;
        int wonly = L.sbins[0].wkey;  // one width in every bin: the one-width kernel
        bool narrow = kind == 0 && sizeof(T) == 4;
        for (const SlotBin &sb : L.sbins) {
            wonly = sb.wkey == wonly ? wonly : -1;
            narrow = narrow && sb.spl == 2 && sb.wkey == 2;
        }
        if (wonly == 2 && narrow) wonly = kWonlyNarrow2;
        else if (wonly == 2 && kind == 0 && sizeof(T) == 4) wonly = -1;  // mixed narrow / plain w = 2 bins
        if (L.sbins[0].nowonly) wonly = -1;  // VBC_SLOT_WONLY=0 (A/B knob)
        const hipError_t e = (hipError_t)launch_slots((int)sizeof(T), kind, L.d_sbins, (int)L.sbins.size(), L.slot_ranges,
                                                      faste, xcd, L.sbins[0].u, L.sbins[0].diag, stage, L.sbins[0].kc != 0,
                                                      wonly, x, y, alpha, beta, rd, stream);
        if (e != hipSuccess) {
            set_error("spmv_slots launch failed: %s", hipGetErrorString(e));
            return VBC_HIP_ERROR;
        }
    }
    if (L.fuse_split) {  // the fused split bins: one launch for all of them
        if (mine(true)) {
            const hipError_t e = (hipError_t)launch_split_multi((int)sizeof(T), L.multi, L.fuse_split, x, y, alpha, beta,
                                                                rd, stream);
            if (e != hipSuccess) {
                set_error("spmv_split_multi launch failed: %s", hipGetErrorString(e));
                return VBC_HIP_ERROR;
            }
        }
    }
    for (size_t i = 0; i < L.pbins.size(); i++) {  // the other planar buckets (vbc_planar.h): one launch each
        const SlotBin &pb = L.pbins[i];
        if (L.fuse_split && pb.fused) continue;
        if (!mine(true)) continue;
        const bool faste = !rd && pb.out_affine && !ablation_knob("VBC_NO_FASTE");
        const bool staged = faste && pb.contig && slot_stage != 0;
        const hipError_t e = (hipError_t)launch_planar((int)sizeof(T), pb, L.d_pbins + i, faste, staged, x, y, alpha,
                                                       beta, rd, stream);
        if (e != hipSuccess) {
            set_error("spmv_planar launch failed: %s", hipGetErrorString(e));
            return VBC_HIP_ERROR;
        }
    }
    if (!mine(L.total_ranges > 0 || L.nfill > 0)) return VBC_OK;
    if (L.total_ranges > 0) {
        const int grid = (L.total_ranges + kWavesPerBlock - 1) / kWavesPerBlock;
        const int K = L.bins.empty() ? kTileKDefault : L.bins[0].tile_k;
        // load-free owner writes when every bucket maps segments affinely and beta = 0
        bool faste = !rd;
        for (const Bin &bb : L.bins) faste = faste && bb.out_affine;
        if (ablation_knob("VBC_NO_FASTE")) faste = false;  // (the VBC_ABLATION build only)
#define VBC_LAUNCH(KIND, KK, PP)                                                                         \
    do {                                                                                                 \
        if (faste)                                                                                       \
            hipLaunchKernelGGL((spmv_ranges<T, KIND, KK, PP, 0, true>), dim3(grid), dim3(kBlockThreads), 0, stream, \
                               L.d_bins, (int)L.bins.size(), L.total_ranges, xs, ys, (T)alpha, (T)beta, (int)rd); \
        else                                                                                             \
            hipLaunchKernelGGL((spmv_ranges<T, KIND, KK, PP>), dim3(grid), dim3(kBlockThreads), 0, stream, \
                               L.d_bins, (int)L.bins.size(), L.total_ranges, xs, ys, (T)alpha, (T)beta, (int)rd); \
    } while (0)
        const int P = L.bins.empty() ? kPipeDefault : L.bins[0].pipe;
#ifdef VBC_ABLATION
        const int D = L.bins.empty() ? 0 : L.bins[0].diag;
        if constexpr (std::is_same<T, double>::value) {
            if (kind == 0 && K == 4 && P == 2 && D == 1) {
                hipLaunchKernelGGL((spmv_ranges<T, 0, 4, 2, 1>), dim3(grid), dim3(kBlockThreads), 0, stream, L.d_bins,
                                   (int)L.bins.size(), L.total_ranges, xs, ys, (T)alpha, (T)beta, (int)rd);
                return VBC_OK;
            }
            if (kind == 0 && K == 4 && P == 2 && D == 2) {
                hipLaunchKernelGGL((spmv_ranges<T, 0, 4, 2, 2>), dim3(grid), dim3(kBlockThreads), 0, stream, L.d_bins,
                                   (int)L.bins.size(), L.total_ranges, xs, ys, (T)alpha, (T)beta, (int)rd);
                return VBC_OK;
            }
        }
#endif
        if (kind == 0) {
            if (P == 2) { if (K == 4) VBC_LAUNCH(0, 4, 2); else VBC_LAUNCH(0, 8, 2); }
            else { if (K == 4) VBC_LAUNCH(0, 4, 3); else VBC_LAUNCH(0, 8, 3); }
        } else {
            if (P == 2) { if (K == 4) VBC_LAUNCH(1, 4, 2); else VBC_LAUNCH(1, 8, 2); }
            else { if (K == 4) VBC_LAUNCH(1, 4, 3); else VBC_LAUNCH(1, 8, 3); }
        }
#undef VBC_LAUNCH
        VBC_HIP(hipGetLastError());
    }
    const int work = (L.total_ranges > 1 ? L.total_ranges : 0) + L.nfill;
    if (work > 0) {
        const int nr = L.total_ranges > 1 ? L.total_ranges : 0;
        const int grid = (work + kBlockThreads - 1) / kBlockThreads;
        if (kind == 0)
            hipLaunchKernelGGL((fixup<T, 0>), dim3(grid), dim3(kBlockThreads), 0, stream, L.d_bins,
                               (int)L.bins.size(), nr, L.d_fill, L.nfill, ys, (T)alpha, (T)beta, (int)rd);
        else
            hipLaunchKernelGGL((fixup<T, 1>), dim3(grid), dim3(kBlockThreads), 0, stream, L.d_bins,
                               (int)L.bins.size(), nr, L.d_fill, L.nfill, ys, (T)alpha, (T)beta, (int)rd);
        VBC_HIP(hipGetLastError());
    }
    return VBC_OK;
}

template <typename T>
static int launch(const vbc_handle *h, const Launch &L, int kind, const void *x, void *y, double alpha, double beta,
                  bool rd, hipStream_t stream)
{
    const int G = launch_groups(L);
    const int nside = (int)L.fork_streams.size();
    if (kind != 0 || G < 2 || nside == 0)
        return launch_group<T>(L, kind, x, y, alpha, beta, rd, stream, h->xcd, h->slot_stage, -1);
    // fork: the side streams wait for the caller's stream; group 0 stays on it, group g >= 1 goes to
    // side stream (g - 1) % nside; every side stream that ran a group is joined back.  The event
    // sequence is serialised per handle (products on several caller streams at once).
    std::lock_guard<std::mutex> lk(const_cast<vbc_handle *>(h)->fork_mu);
    const int used = std::min(nside, G - 1);
    // A fork pulls the side streams into the caller's graph capture until that capture ends.  A product
    // whose caller stream is in another capture state than a side stream (an eager product while a
    // capture on another stream holds them, or a capture of a second graph) must not queue work there:
    // it runs its groups one after another on its own stream instead (same results, no fork).
    {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        unsigned long long cid = 0;
        bool same = hipStreamGetCaptureInfo(stream, &cs, &cid) == hipSuccess &&
                    cs != hipStreamCaptureStatusInvalidated;
        for (int i = 0; i < used && same; i++) {
            hipStreamCaptureStatus ss = hipStreamCaptureStatusNone;
            unsigned long long sid = 0;
            same = hipStreamGetCaptureInfo(L.fork_streams[i], &ss, &sid) == hipSuccess &&
                   (ss == hipStreamCaptureStatusNone || (ss == hipStreamCaptureStatusActive &&
                                                         cs == hipStreamCaptureStatusActive && sid == cid));
        }
        if (!same) {
            (void)hipGetLastError();  // a refused query leaves no sticky error behind
            return launch_group<T>(L, kind, x, y, alpha, beta, rd, stream, h->xcd, h->slot_stage, -1);
        }
    }
    VBC_HIP(hipEventRecord(L.fork_events[0], stream));
    for (int i = 0; i < used; i++) VBC_HIP(hipStreamWaitEvent(L.fork_streams[i], L.fork_events[0], 0));
    // the heaviest group goes last, on the caller's stream: submitted first, it would fill every CU and
    // the small groups would wait for its tail (the ldoor stand-in's 'min memory': 3-wide bucket + one
    // 32-stripe chunk of 6-wide stripes)
    int gh = 0;
    if ((int)L.gwork.size() == G)
        for (int g = 1; g < G; g++)
            if (L.gwork[g] > L.gwork[gh]) gh = g;
    int st = VBC_OK, si = 0;
    for (int g = 0; g < G && st == VBC_OK; g++)
        if (g != gh)
            st = launch_group<T>(L, kind, x, y, alpha, beta, rd, L.fork_streams[si++ % nside], h->xcd, h->slot_stage, g);
    if (st == VBC_OK) st = launch_group<T>(L, kind, x, y, alpha, beta, rd, stream, h->xcd, h->slot_stage, gh);
    for (int i = 0; i < used; i++) {  // joined even after a failed launch: no side stream is left dangling
        if (hipEventRecord(L.fork_events[1 + i], L.fork_streams[i]) != hipSuccess ||
            hipStreamWaitEvent(stream, L.fork_events[1 + i], 0) != hipSuccess) {
            if (st == VBC_OK) st = fail(VBC_HIP_ERROR, "fork join failed");
        }
    }
    return st;
}

template <typename T>
static int mul_device(const vbc_handle *h, int trans, const void *x, void *y, double alpha, double beta,
                      hipStream_t stream)
{
    if (trans) {
        if (h->n == 0) return VBC_OK;
        return launch<T>(h, h->lt, 0, x, y, alpha, beta, beta != 0.0, stream);
    }
    if (h->m == 0) return VBC_OK;
    if (h->has_ft) return launch<T>(h, h->lft, 0, x, y, alpha, beta, beta != 0.0, stream);  // on C = Bᵀ
    if (h->f_scale) {
        hipLaunchKernelGGL((scale<T>), dim3(std::min<int64_t>((h->m + kBlockThreads - 1) / kBlockThreads, 4096)),
                           dim3(kBlockThreads), 0, stream, static_cast<T *>(y), h->m, (T)beta, (int)(beta != 0.0));
        VBC_HIP(hipGetLastError());
    }
    for (size_t b = 0; b < h->lf.size(); b++) {
        const bool own_beta = !h->f_scale;
        if (int st = launch<T>(h, h->lf[b], 1, x, y, alpha, own_beta ? beta : 1.0, own_beta ? beta != 0.0 : true,
                               stream))
            return st;
    }
    return VBC_OK;
}

int mul_dispatch(const vbc_handle *h, int trans, const void *x, void *y, double alpha, double beta,
                 hipStream_t stream)
{
    if (h->dtype == VBC_I64) return mul_int(h, trans, x, y, alpha, beta, stream);
    return h->dtype == VBC_F64 ? mul_device<double>(h, trans, x, y, alpha, beta, stream)
                               : mul_device<float>(h, trans, x, y, alpha, beta, stream);
}

// Multi-RHS transposed product on the tiled stream (row-major X / Y), in chunks of <= 64 columns.
template <typename T>
static int mulmat_t_rowmajor(vbc_handle *h, int64_t nrhs, const char *X, int64_t ldx, char *Y, int64_t ldy,
                             double alpha, double beta, hipStream_t s)
{
    const Launch &L = h->lt;
    const int NRmax = 64;
    int64_t stride = 1;
    for (const Bin &b : L.bins) stride = std::max<int64_t>(stride, (int64_t)b.nranges * b.w * NRmax);
    const size_t need = (size_t)std::max<size_t>(L.bins.size(), 1) * stride * sizeof(T);
    if (h->carry_mm_bytes < need) {
        if (h->d_carry_mm) (void)hipFree(h->d_carry_mm);
        h->d_carry_mm = nullptr;
        h->carry_mm_bytes = 0;
        VBC_HIP(hipMalloc(&h->d_carry_mm, need));
        h->carry_mm_bytes = need;
    }
    T *cm = static_cast<T *>(h->d_carry_mm);
    const bool rd = beta != 0.0;
    for (int64_t c0 = 0; c0 < nrhs; c0 += NRmax) {
        const int nr = (int)std::min<int64_t>(NRmax, nrhs - c0);
        const T *xs = reinterpret_cast<const T *>(X) + c0;
        T *ys = reinterpret_cast<T *>(Y) + c0;
        const int NR = nr <= 16 ? 16 : 64;
        const int64_t cs = nr <= 16 ? stride / 4 : stride;  // carry slots are sized per NR
        if (L.total_ranges > 0) {
            const int grid = (L.total_ranges + kWavesPerBlock - 1) / kWavesPerBlock;
            const int K = L.bins[0].tile_k;
#define VBC_MM(NRR, KK)                                                                                  \
    hipLaunchKernelGGL((spmm_ranges<T, NRR, KK>), dim3(grid), dim3(kBlockThreads), 0, s, L.d_bins,       \
                       (int)L.bins.size(), L.total_ranges, xs, ldx, ys, ldy, nr, cm, cs, (T)alpha, (T)beta, (int)rd)
            if (NR == 16) { if (K == 4) VBC_MM(16, 4); else VBC_MM(16, 8); }
            else { if (K == 4) VBC_MM(64, 4); else VBC_MM(64, 8); }
#undef VBC_MM
            VBC_HIP(hipGetLastError());
        }
        const int nrng = L.total_ranges > 1 ? L.total_ranges : 0;
        const int64_t work = (int64_t)(nrng + L.nfill) * NR;
        if (work > 0) {
            const int grid = (int)((work + kBlockThreads - 1) / kBlockThreads);
            if (NR == 16)
                hipLaunchKernelGGL((fixup_mm<T, 16>), dim3(grid), dim3(kBlockThreads), 0, s, L.d_bins, (int)L.bins.size(),
                                   nrng, L.d_fill, L.nfill, ys, ldy, nr, cm, cs, (T)alpha, (T)beta, (int)rd);
            else
                hipLaunchKernelGGL((fixup_mm<T, 64>), dim3(grid), dim3(kBlockThreads), 0, s, L.d_bins, (int)L.bins.size(),
                                   nrng, L.d_fill, L.nfill, ys, ldy, nr, cm, cs, (T)alpha, (T)beta, (int)rd);
            VBC_HIP(hipGetLastError());
        }
    }
    return VBC_OK;
}

int mulmat_rowmajor(vbc_handle *h, int64_t nrhs, const char *X, int64_t ldx, char *Y, int64_t ldy, double alpha,
                    double beta, hipStream_t s)
{
    return h->dtype == VBC_F64 ? mulmat_t_rowmajor<double>(h, nrhs, X, ldx, Y, ldy, alpha, beta, s)
                               : mulmat_t_rowmajor<float>(h, nrhs, X, ldx, Y, ldy, alpha, beta, s);
}

void occupancy_ranges(int esz, int K, int P, int occ[2])
{
#define VBC_OCC(TT, KK, PP)                                                                           \
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[0], spmv_ranges<TT, 0, KK, PP>, kBlockThreads, 0); \
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[1], spmv_ranges<TT, 1, KK, PP>, kBlockThreads, 0)
    if (esz == 8) {
        if (K == 4) { if (P == 2) { VBC_OCC(double, 4, 2); } else { VBC_OCC(double, 4, 3); } }
        else { if (P == 2) { VBC_OCC(double, 8, 2); } else { VBC_OCC(double, 8, 3); } }
    } else {
        if (K == 4) { if (P == 2) { VBC_OCC(float, 4, 2); } else { VBC_OCC(float, 4, 3); } }
        else { if (P == 2) { VBC_OCC(float, 8, 2); } else { VBC_OCC(float, 8, 3); } }
    }
#undef VBC_OCC
}

}  // namespace vbc
