// libvbc kernel launches of the matrix-core multi-RHS product (vbc_panel.h).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "vbc_handle.h"

namespace vbc {

// Multi-RHS transposed product on the panel layout (MFMA), X / Y addressed by (row, column) strides,
// in chunks of <= 64 right-hand sides (four 16-column accumulators).
// trans = 1: Y = αB'X + βY on the panel layout of B (lm); trans = 0: Y = αBX + βY on the panel layout
// of Bᵀ (lmf, VBC_CREATE_MULTI_FORWARD) -- the same kernel with x and y extents exchanged.
template <typename T>
static int mulmat_panel(const vbc_handle *h, int trans, int64_t nrhs, const char *X, int64_t sxr, int64_t sxc,
                        char *Y, int64_t syr, int64_t syc, double alpha, double beta, hipStream_t s)
{
    const PanelLaunch &L = trans ? h->lm : h->lmf;
    const int64_t xrows = trans ? h->m : h->n, yrows = trans ? h->n : h->m;
    const bool rd = beta != 0.0;
    // small-tile buckets (vbc_tiles.h): their own launches, disjoint columns of Y
    if (int st = mulmat_tiles_any(h, trans, nrhs, X, sxr, sxc, Y, syr, syc, alpha, beta, s)) return st;
    for (int64_t c0 = 0; c0 < nrhs; c0 += 64) {
        const int nr = (int)std::min<int64_t>(64, nrhs - c0);
        const T *xs = reinterpret_cast<const T *>(X) + c0 * sxc;
        T *ys = reinterpret_cast<T *>(Y) + c0 * syc;
        if (L.total_ranges > 0) {
            const int grid = (L.total_ranges + kWavesPerBlock - 1) / kWavesPerBlock;
            // byte extents of X and Y as addressed by this chunk (rows 0..m-1 / 0..n-1, columns 0..nr-1)
            const int64_t span = ((xrows - 1) * sxr + (int64_t)(nr - 1) * sxc + 1) * (int64_t)sizeof(T);
            const int64_t yspan = ((yrows - 1) * syr + (int64_t)(nr - 1) * syc + 1) * (int64_t)sizeof(T);
            const int64_t lim = int64_t(1) << 31;
            const bool buf = span + 64 * sxc * (int64_t)sizeof(T) < lim && h->panel_val_bytes < lim && !h->panel_nobuf;
            bool affine = true;
            for (const PanelBin &pb : L.bins) affine = affine && pb.out_affine;
            const bool fast = buf && affine && !rd && yspan < lim;
            const uint32_t xb = (uint32_t)span, yb = (uint32_t)std::min<int64_t>(yspan, lim - 1);
#define VBC_PANEL(NB, BUF, FAST)                                                                              \
    hipLaunchKernelGGL((spmm_panel<T, NB, BUF, FAST>), dim3(grid), dim3(kBlockThreads), 0, s, L.d_bins,        \
                       (int)L.bins.size(), L.total_ranges, xs, sxr, sxc, xb, ys, syr, syc, yb, nr, (T)alpha, (T)beta, \
                       (int)rd, h->panel_valu)
#define VBC_PANEL_NB(BUF, FAST)                                                                               \
    do {                                                                                                      \
        if (nr <= 16) VBC_PANEL(1, BUF, FAST);                                                                \
        else if (nr <= 32) VBC_PANEL(2, BUF, FAST);                                                           \
        else VBC_PANEL(4, BUF, FAST);                                                                         \
    } while (0)
            if (fast) VBC_PANEL_NB(true, true);
            else if (buf) VBC_PANEL_NB(true, false);
            else VBC_PANEL_NB(false, false);
#undef VBC_PANEL_NB
#undef VBC_PANEL
            VBC_HIP(hipGetLastError());
        }
        if (L.nfill > 0) {
            const int64_t work = (int64_t)L.nfill * nr;
            hipLaunchKernelGGL((fill_rows_mm<T>), dim3((int)((work + kBlockThreads - 1) / kBlockThreads)), dim3(kBlockThreads),
                               0, s, L.d_fill, L.nfill, ys, syr, syc, nr, (T)beta, (int)rd);
            VBC_HIP(hipGetLastError());
        }
    }
    return VBC_OK;
}

int mulmat_panel_any(const vbc_handle *h, int trans, int64_t nrhs, const char *X, int64_t sxr, int64_t sxc, char *Y,
                     int64_t syr, int64_t syc, double alpha, double beta, hipStream_t s)
{
    return h->dtype == VBC_F64 ? mulmat_panel<double>(h, trans, nrhs, X, sxr, sxc, Y, syr, syc, alpha, beta, s)
                               : mulmat_panel<float>(h, trans, nrhs, X, sxr, sxc, Y, syr, syc, alpha, beta, s);
}

int occupancy_panel(int esz)
{
    int om = 0;
    if (esz == 8) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&om, spmm_panel<double, 1, true, true>, kBlockThreads, 0);
    else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&om, spmm_panel<float, 1, true, true>, kBlockThreads, 0);
    return om;
}

}  // namespace vbc
