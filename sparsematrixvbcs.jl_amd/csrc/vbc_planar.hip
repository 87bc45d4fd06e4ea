// Launchers of the planar slotted kernel (vbc_planar.h): one launch per planar bucket, one kernel
// instantiation per (value type, width 3..8, write path, key form).
#include <hip/hip_runtime.h>

#include "vbc_planar.h"

namespace vbc {

template <typename T, int W_, bool KC>
static void launch_w(const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                     double alpha, double beta, bool rd, hipStream_t s)
{
    const int grid = (hb.nranges + kWavesPerBlock - 1) / kWavesPerBlock;
    const T *xs = static_cast<const T *>(x);
    T *ys = static_cast<T *>(y);
    constexpr int NB = planar_nb<T, W_>();
    if (faste && staged)
        hipLaunchKernelGGL((spmv_planar<T, W_, true, NB, KC>), dim3(grid), dim3(kBlockThreads), 0, s, d_b, xs, ys,
                           (T)alpha, (T)beta, (int)rd);
    else if (faste)
        hipLaunchKernelGGL((spmv_planar<T, W_, true, 0, KC>), dim3(grid), dim3(kBlockThreads), 0, s, d_b, xs, ys,
                           (T)alpha, (T)beta, (int)rd);
    else
        hipLaunchKernelGGL((spmv_planar<T, W_, false, 0, KC>), dim3(grid), dim3(kBlockThreads), 0, s, d_b, xs, ys,
                           (T)alpha, (T)beta, (int)rd);
}

template <typename T, bool KC>
static int launch_t(const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                    double alpha, double beta, bool rd, hipStream_t s)
{
    switch (hb.wkey) {
    case 3: launch_w<T, 3, KC>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 4: launch_w<T, 4, KC>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 5: launch_w<T, 5, KC>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 6: launch_w<T, 6, KC>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 7: launch_w<T, 7, KC>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    case 8: launch_w<T, 8, KC>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s); break;
    default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int launch_planar(int esz, const SlotBin &hb, const SlotBin *d_b, bool faste, bool staged, const void *x, void *y,
                  double alpha, double beta, bool rd, hipStream_t s)
{
    if (hb.nranges <= 0) return (int)hipSuccess;
    if (esz == 8)
        return hb.kc ? launch_t<double, true>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s)
                     : launch_t<double, false>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
    return hb.kc ? launch_t<float, true>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s)
                 : launch_t<float, false>(hb, d_b, faste, staged, x, y, alpha, beta, rd, s);
}

int occupancy_planar(int esz)
{
    int occ = 0;
    if (esz == 8) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_planar<double, 3, true, 0, true>, kBlockThreads, 0);
    else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_planar<float, 3, true, 0, true>, kBlockThreads, 0);
    return occ;
}

}  // namespace vbc
