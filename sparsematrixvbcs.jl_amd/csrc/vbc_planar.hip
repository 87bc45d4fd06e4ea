// Launchers of the planar slotted kernel (vbc_planar.h): one launch per planar bucket, one kernel
// instantiation per (value type, width 3..8, write path, key form, row run 1..3).
#include <hip/hip_runtime.h>

#include "vbc_planar.h"

namespace vbc {

template <typename T, int W_, bool KC, int RUN>
static void launch_w(const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                     double alpha, double beta, bool rd, hipStream_t s)
{
    const int grid = (hb.nranges + kWavesPerBlock - 1) / kWavesPerBlock;
    const T *xs = static_cast<const T *>(x);
    T *ys = static_cast<T *>(y);
    constexpr int NB = planar_nb<T, W_>();
    if (hb.mask)  // chunk-local length order: a y-offset table, never the affine write path
        hipLaunchKernelGGL((spmv_planar<T, W_, false, 0, KC, RUN, true>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs,
                           ys, (T)alpha, (T)beta, (int)rd);
    else if (faste && staged)
        hipLaunchKernelGGL((spmv_planar<T, W_, true, NB, KC, RUN>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs, ys,
                           (T)alpha, (T)beta, (int)rd);
    else if (faste)
        hipLaunchKernelGGL((spmv_planar<T, W_, true, 0, KC, RUN>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs, ys,
                           (T)alpha, (T)beta, (int)rd);
    else
        hipLaunchKernelGGL((spmv_planar<T, W_, false, 0, KC, RUN>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs, ys,
                           (T)alpha, (T)beta, (int)rd);
}

template <typename T, int W_, bool KC, int RUN>
static void launch_split(const SlotBin &hb, const SlotBin *d_b, const void *x, void *y, double alpha, double beta,
                         bool rd, hipStream_t s)
{
    const T *xs = static_cast<const T *>(x);
    T *ys = static_cast<T *>(y);
    const dim3 grid(hb.nranges);
#ifdef VBC_ABLATION
    if constexpr (W_ == 3 && RUN == 3 && !KC) {  // ablations (the VBC_ABLATION build only, VBC_DIAG=1..4)
        if (hb.diag >= 1 && hb.diag <= 4) {
#define VBC_SPLIT_DIAG(D)                                                                                                     \
    if (hb.diag == D) {                                                                                                       \
        if (hb.split == 2) hipLaunchKernelGGL((spmv_planar_split<T, 3, false, 3, 2, D>), grid, dim3(128), 0, s, hb, xs, ys, (T)alpha, (T)beta, (int)rd); \
        else if (hb.split == 4) hipLaunchKernelGGL((spmv_planar_split<T, 3, false, 3, 4, D>), grid, dim3(256), 0, s, hb, xs, ys, (T)alpha, (T)beta, (int)rd); \
        else hipLaunchKernelGGL((spmv_planar_split<T, 3, false, 3, 8, D>), grid, dim3(512), 0, s, hb, xs, ys, (T)alpha, (T)beta, (int)rd); \
        return;                                                                                                               \
    }
            VBC_SPLIT_DIAG(1) VBC_SPLIT_DIAG(2) VBC_SPLIT_DIAG(3) VBC_SPLIT_DIAG(4)
#undef VBC_SPLIT_DIAG
        }
    }
#endif
    switch (hb.split) {
    case 2: hipLaunchKernelGGL((spmv_planar_split<T, W_, KC, RUN, 2>), grid, dim3(128), 0, s, hb, xs, ys, (T)alpha, (T)beta, (int)rd); break;
    case 4: hipLaunchKernelGGL((spmv_planar_split<T, W_, KC, RUN, 4>), grid, dim3(256), 0, s, hb, xs, ys, (T)alpha, (T)beta, (int)rd); break;
    default: hipLaunchKernelGGL((spmv_planar_split<T, W_, KC, RUN, 8>), grid, dim3(512), 0, s, hb, xs, ys, (T)alpha, (T)beta, (int)rd); break;
    }
}

template <typename T, bool KC, int RUN>
static int launch_r(const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                    double alpha, double beta, bool rd, hipStream_t s)
{
    if (hb.split > 1) {
        switch (hb.wkey) {
        case 1: launch_split<T, 1, KC, RUN>(hb, d_b, x, y, alpha, beta, rd, s); break;
        case 2: launch_split<T, 2, KC, RUN>(hb, d_b, x, y, alpha, beta, rd, s); break;
        case 3: launch_split<T, 3, KC, RUN>(hb, d_b, x, y, alpha, beta, rd, s); break;
        case 4: launch_split<T, 4, KC, RUN>(hb, d_b, x, y, alpha, beta, rd, s); break;
        case 5: launch_split<T, 5, KC, RUN>(hb, d_b, x, y, alpha, beta, rd, s); break;
        case 6: launch_split<T, 6, KC, RUN>(hb, d_b, x, y, alpha, beta, rd, s); break;
        case 7: launch_split<T, 7, KC, RUN>(hb, d_b, x, y, alpha, beta, rd, s); break;
        case 8: launch_split<T, 8, KC, RUN>(hb, d_b, x, y, alpha, beta, rd, s); break;
        default: return (int)hipErrorInvalidValue;
        }
        return (int)hipGetLastError();
    }
    switch (hb.wkey) {
    case 3: launch_w<T, 3, KC, RUN>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 4: launch_w<T, 4, KC, RUN>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 5: launch_w<T, 5, KC, RUN>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 6: launch_w<T, 6, KC, RUN>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 7: launch_w<T, 7, KC, RUN>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 8: launch_w<T, 8, KC, RUN>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// row runs (SlotBin::run): 1 (none), 2 or 3 consecutive x rows per gather
template <typename T, bool KC>
static int launch_t(const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                    double alpha, double beta, bool rd, hipStream_t s)
{
    switch (hb.run) {
    case 1: return launch_r<T, KC, 1>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
    case 2: return launch_r<T, KC, 2>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
    case 3: return launch_r<T, KC, 3>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
    default: return (int)hipErrorInvalidValue;
    }
}

template <bool KC, bool DOT>
static int launch_pair(const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                       double alpha, double beta, bool rd, hipStream_t s)
{
    const int grid = (hb.nranges + kWavesPerBlock - 1) / kWavesPerBlock;
    const double *xs = static_cast<const double *>(x);
    double *ys = static_cast<double *>(y);
    if (hb.mask)
        hipLaunchKernelGGL((spmv_planar_pair<false, 0, KC, true, DOT>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs, ys,
                           alpha, beta, (int)rd);
    else if (faste && staged)
        hipLaunchKernelGGL((spmv_planar_pair<true, 8, KC, false, DOT>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs, ys,
                           alpha, beta, (int)rd);
    else if (faste)
        hipLaunchKernelGGL((spmv_planar_pair<true, 0, KC, false, DOT>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs, ys,
                           alpha, beta, (int)rd);
    else
        hipLaunchKernelGGL((spmv_planar_pair<false, 0, KC, false, DOT>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs,
                           ys, alpha, beta, (int)rd);
    return (int)hipGetLastError();
}

template <typename T, int W_, int R, bool KC>
static void launch_fwd_wr(const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                          double alpha, double beta, bool rd, hipStream_t s)
{
    const int grid = (hb.nranges + kWavesPerBlock - 1) / kWavesPerBlock;
    const T *xs = static_cast<const T *>(x);
    T *ys = static_cast<T *>(y);
    if constexpr (!KC) {
        if (hb.split > 1) {  // few chunks: P waves per chunk (spmv_planar_fwd_split)
            const dim3 g(hb.nranges);
            if (hb.split == 2) hipLaunchKernelGGL((spmv_planar_fwd_split<T, W_, R, 2>), g, dim3(128), 0, s, hb, xs, ys, (T)alpha, (T)beta, (int)rd);
            else if (hb.split == 4) hipLaunchKernelGGL((spmv_planar_fwd_split<T, W_, R, 4>), g, dim3(256), 0, s, hb, xs, ys, (T)alpha, (T)beta, (int)rd);
            else hipLaunchKernelGGL((spmv_planar_fwd_split<T, W_, R, 8>), g, dim3(512), 0, s, hb, xs, ys, (T)alpha, (T)beta, (int)rd);
            return;
        }
    }
    constexpr int NB = (8192 / (64 * R * (int)sizeof(T))) > 8 ? 8 : (8192 / (64 * R * (int)sizeof(T)));
    if (hb.mask)
        hipLaunchKernelGGL((spmv_planar_fwd<T, W_, R, false, 0, KC, true>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs,
                           ys, (T)alpha, (T)beta, (int)rd);
    else if (faste && staged)
        hipLaunchKernelGGL((spmv_planar_fwd<T, W_, R, true, NB, KC>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs, ys,
                           (T)alpha, (T)beta, (int)rd);
    else if (faste)
        hipLaunchKernelGGL((spmv_planar_fwd<T, W_, R, true, 0, KC>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs, ys,
                           (T)alpha, (T)beta, (int)rd);
    else
        hipLaunchKernelGGL((spmv_planar_fwd<T, W_, R, false, 0, KC>), dim3(grid), dim3(kBlockThreads), 0, s, hb, xs, ys,
                           (T)alpha, (T)beta, (int)rd);
}

// forward row runs: w in {2, 3, 4}, R in {2, 3}
template <typename T, bool KC>
static int launch_fwd(const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                      double alpha, double beta, bool rd, hipStream_t s)
{
#define VBC_FWD(W, RR)                                                                                      if (hb.wkey == W && hb.run == RR) {                                                                         launch_fwd_wr<T, W, RR, KC>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);                          return (int)hipGetLastError();                                                                      }
    VBC_FWD(2, 2) VBC_FWD(2, 3) VBC_FWD(3, 2) VBC_FWD(3, 3) VBC_FWD(4, 2) VBC_FWD(4, 3)
#undef VBC_FWD
    return (int)hipErrorInvalidValue;
}

// per-lane compacted streams (vbc_planar.h run_planar_lanes): w in 3..8, runs of 1..3
template <typename T, int W_, int RUN>
static void launch_lanes_w(const SlotBin &hb, const SlotBin *d_b, const T *xs, T *ys, double alpha, double beta,
                           bool rd, hipStream_t s)
{
    const dim3 grid((hb.nranges + kWavesPerBlock - 1) / kWavesPerBlock), blk(kBlockThreads);
#ifdef VBC_ABLATION
    if constexpr (W_ == 3 && RUN == 3) {  // ablations (the VBC_ABLATION build only, VBC_DIAG=1..3)
        if (hb.diag == 1) { hipLaunchKernelGGL((spmv_planar_lanes<T, W_, RUN, false, false, 1>), grid, blk, 0, s, hb, xs, ys, (T)alpha, (T)beta); return; }
        if (hb.diag == 2) { hipLaunchKernelGGL((spmv_planar_lanes<T, W_, RUN, false, false, 2>), grid, blk, 0, s, hb, xs, ys, (T)alpha, (T)beta); return; }
        if (hb.diag == 3) { hipLaunchKernelGGL((spmv_planar_lanes<T, W_, RUN, false, false, 3>), grid, blk, 0, s, hb, xs, ys, (T)alpha, (T)beta); return; }
    }
#endif
    if (rd) hipLaunchKernelGGL((spmv_planar_lanes<T, W_, RUN, false, true>), grid, blk, 0, s, hb, xs, ys, (T)alpha, (T)beta);
    else if (hb.deep) hipLaunchKernelGGL((spmv_planar_lanes<T, W_, RUN, true, false>), grid, blk, 0, s, hb, xs, ys, (T)alpha, (T)beta);
    else hipLaunchKernelGGL((spmv_planar_lanes<T, W_, RUN, false, false>), grid, blk, 0, s, hb, xs, ys, (T)alpha, (T)beta);
}

template <typename T, int RUN>
static int launch_lanes_r(const SlotBin &hb, const SlotBin *d_b, const void *x, void *y, double alpha, double beta,
                          bool rd, hipStream_t s)
{
    const T *xs = static_cast<const T *>(x);
    T *ys = static_cast<T *>(y);
    switch (hb.wkey) {
    case 3: launch_lanes_w<T, 3, RUN>(hb, d_b, xs, ys, alpha, beta, rd, s); break;
    case 4: launch_lanes_w<T, 4, RUN>(hb, d_b, xs, ys, alpha, beta, rd, s); break;
    case 5: launch_lanes_w<T, 5, RUN>(hb, d_b, xs, ys, alpha, beta, rd, s); break;
    case 6: launch_lanes_w<T, 6, RUN>(hb, d_b, xs, ys, alpha, beta, rd, s); break;
    case 7: launch_lanes_w<T, 7, RUN>(hb, d_b, xs, ys, alpha, beta, rd, s); break;
    case 8: launch_lanes_w<T, 8, RUN>(hb, d_b, xs, ys, alpha, beta, rd, s); break;
    default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

template <typename T>
static int launch_lanes(const SlotBin &hb, const SlotBin *d_b, const void *x, void *y, double alpha, double beta,
                        bool rd, hipStream_t s)
{
    switch (hb.run) {
    case 1: return launch_lanes_r<T, 1>(hb, d_b, x, y, alpha, beta, rd, s);
    case 2: return launch_lanes_r<T, 2>(hb, d_b, x, y, alpha, beta, rd, s);
    case 3: return launch_lanes_r<T, 3>(hb, d_b, x, y, alpha, beta, rd, s);
    default: return (int)hipErrorInvalidValue;
    }
}

int occupancy_lanes(int esz)
{
    int occ = 0;
    if (esz == 8) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_planar_lanes<double, 3, 3, false, false>, kBlockThreads, 0);
    else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_planar_lanes<float, 3, 3, false, false>, kBlockThreads, 0);
    return occ;
}

int launch_planar(int esz, const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                  double alpha, double beta, bool rd, hipStream_t s)
{
    if (hb.nranges <= 0) return (int)hipSuccess;
    if (hb.lanes && hb.pair) {  // lane-pair streams (B'x, fp64, w = 3, runs of 3)
        if (hb.kind != 0 || esz != 8 || hb.wkey != 3 || hb.run != 3) return (int)hipErrorInvalidValue;
        const dim3 grid((hb.nranges + kWavesPerBlock - 1) / kWavesPerBlock), blk(kBlockThreads);
        const double *xs = static_cast<const double *>(x);
        double *ys = static_cast<double *>(y);
        if (rd) hipLaunchKernelGGL((spmv_pair_lanes<true>), grid, blk, 0, s, hb, xs, ys, alpha, beta);
        else hipLaunchKernelGGL((spmv_pair_lanes<false>), grid, blk, 0, s, hb, xs, ys, alpha, beta);
        return (int)hipGetLastError();
    }
    if (hb.lanes) {  // per-lane compacted streams (B'x)
        if (hb.kind != 0) return (int)hipErrorInvalidValue;
        return esz == 8 ? launch_lanes<double>(hb, d_b, x, y, alpha, beta, rd, s)
                        : launch_lanes<float>(hb, d_b, x, y, alpha, beta, rd, s);
    }
    if (hb.kind == 1) {  // forward with row runs (vbc_planar.h run_planar_fwd)
        if (esz == 8)
            return hb.kc ? launch_fwd<double, true>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s)
                         : launch_fwd<double, false>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
        return hb.kc ? launch_fwd<float, true>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s)
                     : launch_fwd<float, false>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
    }
    if (hb.pair) {  // fp64, w = 3, runs of 3: lane pairs (vbc_planar.h run_pair)
        if (esz != 8 || hb.wkey != 3 || hb.run != 3) return (int)hipErrorInvalidValue;
        if (hb.dot)  // the forward product of 3 x 3 node blocks (SlotBin::dot)
            return hb.kc ? launch_pair<true, true>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s)
                         : launch_pair<false, true>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
        return hb.kc ? launch_pair<true, false>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s)
                     : launch_pair<false, false>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
    }
    if (esz == 8)
        return hb.kc ? launch_t<double, true>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s)
                     : launch_t<double, false>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
    return hb.kc ? launch_t<float, true>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s)
                 : launch_t<float, false>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
}

template <typename T>
static int launch_split_multi_t(const SplitMulti &M, int P, const void *x, void *y, double alpha, double beta, bool rd,
                                hipStream_t s)
{
    const T *xs = static_cast<const T *>(x);
    T *ys = static_cast<T *>(y);
    const dim3 grid(M.nchunks);
    const int mode = M.pad0;  // SplitMulti::pad0: slice loop 0 plain, 1 pipelined, 2 batched, 3 batched non-temporal
#define VBC_MULTI(PP)                                                                                                   \
    if (mode == 3) hipLaunchKernelGGL((spmv_split_multi<T, PP, 3>), grid, dim3(64 * PP), 0, s, M, xs, ys, (T)alpha, (T)beta, (int)rd); \
    else if (mode == 2) hipLaunchKernelGGL((spmv_split_multi<T, PP, 2>), grid, dim3(64 * PP), 0, s, M, xs, ys, (T)alpha, (T)beta, (int)rd); \
    else if (mode == 1) hipLaunchKernelGGL((spmv_split_multi<T, PP, 1>), grid, dim3(64 * PP), 0, s, M, xs, ys, (T)alpha, (T)beta, (int)rd); \
    else hipLaunchKernelGGL((spmv_split_multi<T, PP, 0>), grid, dim3(64 * PP), 0, s, M, xs, ys, (T)alpha, (T)beta, (int)rd);
    switch (P) {
    case 2: VBC_MULTI(2) break;
    case 4: VBC_MULTI(4) break;
    case 8: VBC_MULTI(8) break;
    default: return (int)hipErrorInvalidValue;
    }
#undef VBC_MULTI
    return (int)hipGetLastError();
}

int launch_split_multi(int esz, const SplitMulti &M, int P, const void *x, void *y, double alpha, double beta, bool rd,
                       hipStream_t s)
{
    if (M.nchunks <= 0) return (int)hipSuccess;
    return esz == 8 ? launch_split_multi_t<double>(M, P, x, y, alpha, beta, rd, s)
                    : launch_split_multi_t<float>(M, P, x, y, alpha, beta, rd, s);
}

// Resident waves per CU of the fused split launch (batched slice loop) with P waves per workgroup.
int occupancy_split_multi(int esz, int P)
{
    int nb = 0;
#define VBC_OCC_MULTI(TT, PP) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, spmv_split_multi<TT, PP, 2>, 64 * PP, 0)
    if (esz == 8) {
        if (P == 2) VBC_OCC_MULTI(double, 2); else if (P == 4) VBC_OCC_MULTI(double, 4); else VBC_OCC_MULTI(double, 8);
    } else {
        if (P == 2) VBC_OCC_MULTI(float, 2); else if (P == 4) VBC_OCC_MULTI(float, 4); else VBC_OCC_MULTI(float, 8);
    }
#undef VBC_OCC_MULTI
    return nb * P;
}

int occupancy_planar(int esz)
{
    int occ = 0;
    if (esz == 8) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_planar<double, 3, true, 0, true, 1>, kBlockThreads, 0);
    else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_planar<float, 3, true, 0, true, 1>, kBlockThreads, 0);
    return occ;
}

}  // namespace vbc
