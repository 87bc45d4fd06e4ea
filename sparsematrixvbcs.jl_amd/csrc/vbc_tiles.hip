// libvbc kernel launches of the tile-granular multi-RHS product (vbc_tiles.h): small u x w tiles
// (u, w <= 4) of the panel layout's buckets, 16 right-hand sides per launch.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "vbc_handle.h"
#include "vbc_tiles.h"

namespace vbc {

template <typename T, int UB, int W, int NBT, int D>
static void launch_tiles_uwn(const TileBin &tb, int grid, hipStream_t s, const T *xs, int64_t sxr, int64_t sxc,
                             uint32_t xb, bool buf, T *ys, int64_t syr, int64_t syc, int nr, T alpha, T beta, int rd,
                             int fast)
{
#define VBC_TILES(MASKU, BUF)                                                                                      \
    hipLaunchKernelGGL((spmm_tiles<T, UB, W, NBT, MASKU, BUF, D>), dim3(grid), dim3(kBlockThreads),                 \
                       (size_t)tb.stage_bytes * kWavesPerBlock, s, tb, xs, sxr,                                  \
                       sxc, xb, ys, syr, syc, nr, alpha, beta, rd, fast)
    if (tb.masku) {
        if (buf) VBC_TILES(true, true);
        else VBC_TILES(true, false);
    } else {
        if (buf) VBC_TILES(false, true);
        else VBC_TILES(false, false);
    }
#undef VBC_TILES
}

template <typename T, int UB, int W>
static void launch_tiles_uw(const TileBin &tb, int grid, hipStream_t s, const T *xs, int64_t sxr, int64_t sxc,
                            uint32_t xb, bool buf, T *ys, int64_t syr, int64_t syc, int nr, T alpha, T beta, int rd,
                            int fast)
{
#ifdef VBC_ABLATION
    if (tb.depth == 3) {
        if (tb.nbt == 8) launch_tiles_uwn<T, UB, W, 8, 3>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast);
        else launch_tiles_uwn<T, UB, W, 4, 3>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast);
        return;
    }
#endif
    if (tb.nbt == 8) launch_tiles_uwn<T, UB, W, 8, 2>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast);
    else launch_tiles_uwn<T, UB, W, 4, 2>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast);
}

template <typename T, int UB>
static void launch_tiles_u(const TileBin &tb, int grid, hipStream_t s, const T *xs, int64_t sxr, int64_t sxc,
                           uint32_t xb, bool buf, T *ys, int64_t syr, int64_t syc, int nr, T alpha, T beta, int rd,
                           int fast)
{
    switch (tb.w) {
    case 1: launch_tiles_uw<T, UB, 1>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast); break;
    case 2: launch_tiles_uw<T, UB, 2>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast); break;
    case 3: launch_tiles_uw<T, UB, 3>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast); break;
    default: launch_tiles_uw<T, UB, 4>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast); break;
    }
}

// Y = alpha op(B) X + beta Y for the tile buckets of L (the other buckets are the panel kernel's): per
// 16 right-hand sides one launch per bucket.  xrows: rows of X (m for B'X, n for B·X on Bᵀ's layout).
template <typename T>
static int mulmat_tiles(const vbc_handle *h, const PanelLaunch &L, int64_t nrhs, int64_t xrows, const char *X,
                        int64_t sxr, int64_t sxc, char *Y, int64_t syr, int64_t syc, double alpha, double beta,
                        hipStream_t s)
{
    const bool rd = beta != 0.0;
    for (int64_t c0 = 0; c0 < nrhs; c0 += 16) {
        const int nr = (int)std::min<int64_t>(16, nrhs - c0);
        const T *xs = reinterpret_cast<const T *>(X) + c0 * sxc;
        T *ys = reinterpret_cast<T *>(Y) + c0 * syc;
        const int64_t lim = int64_t(1) << 31;
        // bytes of X as this chunk addresses it, plus the over-read of a tile slot's rows past the last
        // row (the slot rows a tile does not store: masked, but still loaded)
        const int64_t span = ((xrows - 1) * sxr + (int64_t)(nr - 1) * sxc + 1) * (int64_t)sizeof(T);
        // the mul24 buffer path: an invalid key's all-ones 24-bit row times the row stride must land past X
        // without wrapping 32 bits (vbc_tiles.h load_x)
        const int64_t sxr_b = sxr * (int64_t)sizeof(T);
        const bool buf = span + 4 * sxr_b < lim && sxr_b > 0 && sxr_b <= 255 && (int64_t)kTileRow * sxr_b >= span &&
                         !h->panel_nobuf;
        const uint32_t xb = (uint32_t)std::min<int64_t>(span, lim - 1);
        for (const TileBin &tb : L.tbins) {
            if (tb.nranges == 0) continue;
            // one contiguous run of Y per range: affine map of stride w, 16 contiguous right-hand sides
            const bool rows16 = nr == 16 && syc == 1 && syr == 16 && reinterpret_cast<uintptr_t>(ys) % 16 == 0;
            int fast = tb.out_affine && tb.out_stride == tb.w && rows16 ? 1 : 0;
            // (the dword form: stripes in another order still store 16-B pieces of each stripe's block)
            const int fast_dw = fast ? 1 : (rows16 ? 2 : 0);
            const int grid = (tb.nranges + kWavesPerBlock - 1) / kWavesPerBlock;
            switch (tb.ub) {
            case 1: launch_tiles_u<T, 1>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, (T)alpha, (T)beta, rd, fast_dw); break;
            case 2: launch_tiles_u<T, 2>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, (T)alpha, (T)beta, rd, fast_dw); break;
            case 3: launch_tiles_u<T, 3>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, (T)alpha, (T)beta, rd, fast_dw); break;
            default: launch_tiles_u<T, 4>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, (T)alpha, (T)beta, rd, fast_dw); break;
            }
            VBC_HIP(hipGetLastError());
        }
    }
    return VBC_OK;
}

int mulmat_tiles_any(const vbc_handle *h, int trans, int64_t nrhs, const char *X, int64_t sxr, int64_t sxc, char *Y,
                     int64_t syr, int64_t syc, double alpha, double beta, hipStream_t s)
{
    const PanelLaunch &L = trans ? h->lm : h->lmf;
    if (L.tbins.empty()) return VBC_OK;
    const int64_t xrows = trans ? h->m : h->n;
    return h->dtype == VBC_F64 ? mulmat_tiles<double>(h, L, nrhs, xrows, X, sxr, sxc, Y, syr, syc, alpha, beta, s)
                               : mulmat_tiles<float>(h, L, nrhs, xrows, X, sxr, sxc, Y, syr, syc, alpha, beta, s);
}

// resident waves per CU of the tile kernel (3 x 3 tiles: the layout's ranges are sized for it)
int occupancy_tiles(int esz)
{
    int ob = 0;
    if (esz == 8)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&ob, spmm_tiles<double, 3, 3, kTileBatch, false, true>,
                                                           kBlockThreads, kWavesPerBlock * kTileStripes * 3 * 16 * 8);
    else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&ob, spmm_tiles<float, 3, 3, kTileBatch, false, true>,
                                                           kBlockThreads, kWavesPerBlock * kTileStripes * 3 * 16 * 4);
    return std::max(1, ob) * kWavesPerBlock;
}

}  // namespace vbc
