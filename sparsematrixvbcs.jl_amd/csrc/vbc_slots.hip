// Launchers of the slotted-segment kernel (vbc_slots.h), compiled in their own translation unit.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "vbc_slots.h"

namespace vbc {

template <typename T, int U, bool KC>
static void launch_t(int kind, const SlotBin *d_bins, int nbins, int total_ranges, bool faste, int xcd, int diag, int stage,
                     const void *x, void *y, double alpha, double beta, bool rd, hipStream_t s)
{
    const int grid = (total_ranges + kWavesPerBlock - 1) / kWavesPerBlock;
    const int xcd_chunk = (xcd && grid >= 16) ? 1 : 0;
    const T *xs = static_cast<const T *>(x);
    T *ys = static_cast<T *>(y);
#define VBC_SLOTS(KIND, F)                                                                               \
    hipLaunchKernelGGL((spmv_slots<T, KIND, U, F, 0, 0, KC>), dim3(grid), dim3(kBlockThreads), 0, s, d_bins, nbins, \
                       total_ranges, xcd_chunk, xs, ys, (T)alpha, (T)beta, (int)rd)
    if constexpr (sizeof(T) == 8 && U == 8 && !KC) {  // ablations (tools/ab.py only)
        if (kind == 0 && faste && diag == 1) {
            hipLaunchKernelGGL((spmv_slots<T, 0, U, true, 1>), dim3(grid), dim3(kBlockThreads), 0, s, d_bins, nbins,
                               total_ranges, xcd_chunk, xs, ys, (T)alpha, (T)beta, (int)rd);
            return;
        }
        if (kind == 0 && faste && diag == 2) {
            hipLaunchKernelGGL((spmv_slots<T, 0, U, true, 2>), dim3(grid), dim3(kBlockThreads), 0, s, d_bins, nbins,
                               total_ranges, xcd_chunk, xs, ys, (T)alpha, (T)beta, (int)rd);
            return;
        }
        if (kind == 0 && faste && diag == 4) {
            hipLaunchKernelGGL((spmv_slots<T, 0, U, true, 4>), dim3(grid), dim3(kBlockThreads), 0, s, d_bins, nbins,
                               total_ranges, xcd_chunk, xs, ys, (T)alpha, (T)beta, (int)rd);
            return;
        }
        if (kind == 0 && faste && diag == 3) {
            hipLaunchKernelGGL((spmv_slots<T, 0, U, true, 3>), dim3(grid), dim3(kBlockThreads), 0, s, d_bins, nbins,
                               total_ranges, xcd_chunk, xs, ys, (T)alpha, (T)beta, (int)rd);
            return;
        }
    }
#define VBC_STAGED(KIND, NB)                                                                             \
    hipLaunchKernelGGL((spmv_slots<T, KIND, U, true, 0, NB, KC>), dim3(grid), dim3(kBlockThreads), 0, s, d_bins, nbins, \
                       total_ranges, xcd_chunk, xs, ys, (T)alpha, (T)beta, (int)rd)
    if (faste && stage == 8) { if (kind == 0) VBC_STAGED(0, 8); else VBC_STAGED(1, 8); return; }
#undef VBC_STAGED
    if (kind == 0) { if (faste) VBC_SLOTS(0, true); else VBC_SLOTS(0, false); }
    else { if (faste) VBC_SLOTS(1, true); else VBC_SLOTS(1, false); }
#undef VBC_SLOTS
}

// u: rows per pipeline step (4 or 8 for fp64, 8 or 16 for fp32).
int launch_slots(int esz, int kind, const SlotBin *d_bins, int nbins, int total_ranges, bool faste, int xcd, int u, int diag, int stage, bool kc,
                 const void *x, void *y, double alpha, double beta, bool rd, hipStream_t stream)
{
    if (total_ranges <= 0) return hipSuccess;
#define VBC_LT(TT, UU, KK) launch_t<TT, UU, KK>(kind, d_bins, nbins, total_ranges, faste, xcd, diag, stage, x, y, alpha, beta, rd, stream)
    if (esz == 8) {
        if (kc) VBC_LT(double, 8, true);
        else if (u == 4) VBC_LT(double, 4, false);
        else VBC_LT(double, 8, false);
    } else {
        if (kc) VBC_LT(float, 16, true);
        else if (u == 8) VBC_LT(float, 8, false);
        else VBC_LT(float, 16, false);
    }
#undef VBC_LT
    return hipGetLastError();
}

int occupancy_slots(int esz, int kind)
{
    int occ = 0;
    if (esz == 8) {
        if (kind == 0) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_slots<double, 0, 8, true>, kBlockThreads, 0);
        else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_slots<double, 1, 8, true>, kBlockThreads, 0);
    } else {
        if (kind == 0) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_slots<float, 0, 16, true>, kBlockThreads, 0);
        else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_slots<float, 1, 16, true>, kBlockThreads, 0);
    }
    return occ;
}

}  // namespace vbc
