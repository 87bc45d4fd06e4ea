// Dispatch of the slotted-kernel launchers by value type (the kernels live in vbc_slots_f64.hip and
// vbc_slots_f32.hip, one translation unit each).
#include <hip/hip_runtime.h>

#include "vbc_kernels.h"

namespace vbc {

int launch_slots_f64(int kind, const SlotBin *d_bins, int nbins, int total_ranges, bool faste, int xcd, int diag,
                     int stage, bool kc, int wonly, const void *x, void *y, double alpha, double beta, bool rd,
                     hipStream_t stream);
int launch_slots_f32(int kind, const SlotBin *d_bins, int nbins, int total_ranges, bool faste, int xcd, int diag,
                     int stage, bool kc, int wonly, const void *x, void *y, double alpha, double beta, bool rd,
                     hipStream_t stream);
int occupancy_slots_f64(int kind);
int occupancy_slots_f32(int kind);

int launch_slots(int esz, int kind, const SlotBin *d_bins, int nbins, int total_ranges, bool faste, int xcd, int u,
                 int diag, int stage, bool kc, int wonly, const void *x, void *y, double alpha, double beta, bool rd,
                 hipStream_t stream)
{
    (void)u;  // one step depth per type (vbc_slots_f64.hip / vbc_slots_f32.hip)
    if (total_ranges <= 0) return hipSuccess;
    return esz == 8 ? launch_slots_f64(kind, d_bins, nbins, total_ranges, faste, xcd, diag, stage, kc, wonly, x, y, alpha, beta, rd, stream)
                    : launch_slots_f32(kind, d_bins, nbins, total_ranges, faste, xcd, diag, stage, kc, wonly, x, y, alpha, beta, rd, stream);
}

int occupancy_slots(int esz, int kind) { return esz == 8 ? occupancy_slots_f64(kind) : occupancy_slots_f32(kind); }

}  // namespace vbc
