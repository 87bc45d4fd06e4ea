// libvbc kernel launches of the tile-granular multi-RHS product (vbc_tiles.h): small u x w tiles
// (u, w <= 4) of the panel layout's buckets, 16 right-hand sides per launch.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "vbc_handle.h"
#include "vbc_tiles.h"

namespace vbc {

template <typename T, int UB, int W, int NBT>
static void launch_tiles_uwn(const TileBin &tb, int grid, hipStream_t s, const T *xs, int64_t sxr, int64_t sxc,
                             uint32_t xb, bool buf, T *ys, int64_t syr, int64_t syc, int nr, T alpha, T beta, int rd,
                             int fast)
{
#define VBC_TILES(MASKU, BUF)                                                                                      \
    hipLaunchKernelGGL((spmm_tiles<T, UB, W, NBT, MASKU, BUF>), dim3(grid), dim3(kBlockThreads),                 \
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
    if (tb.nbt == 8) launch_tiles_uwn<T, UB, W, 8>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast);
    else launch_tiles_uwn<T, UB, W, 4>(tb, grid, s, xs, sxr, sxc, xb, buf, ys, syr, syc, nr, alpha, beta, rd, fast);
}

// the 16-B form (vbc_tiles.h spmm_tiles4): fp32, 16 contiguous right-hand sides
template <int UB, int W>
static void launch_tiles4_uw(const TileBin &tb, int grid, hipStream_t s, const float *xs, int64_t sxr, uint32_t xb,
                             float *ys, int64_t syr, int64_t syc, float alpha, float beta, int rd, int fast)
{
    const size_t lds = (size_t)tb.stage_bytes * kWavesPerBlock;
#define VBC_TILES4(NBT, MASKU)                                                                                      \
    hipLaunchKernelGGL((spmm_tiles4<UB, W, NBT, MASKU>), dim3(grid), dim3(kBlockThreads), lds, s, tb, xs, sxr, xb, ys, \
                       syr, syc, alpha, beta, rd, fast)
    if (tb.nbt == 8) {
        if (tb.masku) VBC_TILES4(8, true);
        else VBC_TILES4(8, false);
    } else {
        if (tb.masku) VBC_TILES4(4, true);
        else VBC_TILES4(4, false);
    }
#undef VBC_TILES4
}
template <int UB>
static void launch_tiles4_u(const TileBin &tb, int grid, hipStream_t s, const float *xs, int64_t sxr, uint32_t xb,
                            float *ys, int64_t syr, int64_t syc, float alpha, float beta, int rd, int fast)
{
    switch (tb.w) {
    case 1: launch_tiles4_uw<UB, 1>(tb, grid, s, xs, sxr, xb, ys, syr, syc, alpha, beta, rd, fast); break;
    case 2: launch_tiles4_uw<UB, 2>(tb, grid, s, xs, sxr, xb, ys, syr, syc, alpha, beta, rd, fast); break;
    case 3: launch_tiles4_uw<UB, 3>(tb, grid, s, xs, sxr, xb, ys, syr, syc, alpha, beta, rd, fast); break;
    default: launch_tiles4_uw<UB, 4>(tb, grid, s, xs, sxr, xb, ys, syr, syc, alpha, beta, rd, fast); break;
    }
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

// the persistent staged-X form (spmm_tiles_xp): nwg workgroups of 6 waves, both LDS stages double-buffered
static size_t tiles_xp_lds(const TileBin &tb)
{
    return 2 * (size_t)tb.xslots * tb.ub * 16 * sizeof(float) + 2 * (size_t)tb.stage_bytes + 2 * kTileXStreams * sizeof(int);
}
template <int UB, int W>
static void launch_tiles_xp_uw(const TileBin &tb, hipStream_t s, const float *xs, int64_t sxr, int64_t xrows, float *ys,
                               float alpha, float beta, int rd)
{
    const size_t lds = tiles_xp_lds(tb);
    static bool attr[2] = {false, false};  // dynamic LDS above 64 KB: raised once per instantiation
    if (!attr[tb.masku ? 1 : 0]) {
        if (tb.masku) (void)hipFuncSetAttribute(reinterpret_cast<const void *>(spmm_tiles_xp<UB, W, true>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTileXPLds);
        else (void)hipFuncSetAttribute(reinterpret_cast<const void *>(spmm_tiles_xp<UB, W, false>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTileXPLds);
        attr[tb.masku ? 1 : 0] = true;
    }
    if (tb.masku)
        hipLaunchKernelGGL((spmm_tiles_xp<UB, W, true>), dim3(tb.nwg), dim3(kTileXPThreads), lds, s, tb, xs, sxr, xrows, ys,
                           alpha, beta, rd);
    else
        hipLaunchKernelGGL((spmm_tiles_xp<UB, W, false>), dim3(tb.nwg), dim3(kTileXPThreads), lds, s, tb, xs, sxr, xrows, ys,
                           alpha, beta, rd);
}
template <int UB>
static void launch_tiles_xp_u(const TileBin &tb, hipStream_t s, const float *xs, int64_t sxr, int64_t xrows, float *ys,
                              float alpha, float beta, int rd)
{
    switch (tb.w) {
    case 1: launch_tiles_xp_uw<UB, 1>(tb, s, xs, sxr, xrows, ys, alpha, beta, rd); break;
    case 2: launch_tiles_xp_uw<UB, 2>(tb, s, xs, sxr, xrows, ys, alpha, beta, rd); break;
    case 3: launch_tiles_xp_uw<UB, 3>(tb, s, xs, sxr, xrows, ys, alpha, beta, rd); break;
    default: launch_tiles_xp_uw<UB, 4>(tb, s, xs, sxr, xrows, ys, alpha, beta, rd); break;
    }
}

// the staged-X form (spmm_tiles_x): one workgroup per cluster, LDS = X stage + output stage
template <typename T, int UB, int W, bool MASKU, bool X4, int NW>
static void launch_tiles_x_k(const TileBin &tb, hipStream_t s, const T *xs, int64_t sxr, int64_t sxc, int64_t xrows,
                             T *ys, int64_t syr, int64_t syc, int nr, T alpha, T beta, int rd, int fast)
{
    const size_t lds = (size_t)tb.xslots * UB * 16 * sizeof(T) + (size_t)tb.stage_bytes;
    if (lds > 65536) {  // (above the default dynamic LDS limit: raised once per instantiation)
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(spmm_tiles_x<T, UB, W, MASKU, X4, NW>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTileXLds8);
            attr = true;
        }
    }
    hipLaunchKernelGGL((spmm_tiles_x<T, UB, W, MASKU, X4, NW>), dim3(tb.nranges), dim3(NW * 64), lds, s, tb, xs, sxr, sxc,
                       xrows, ys, syr, syc, nr, alpha, beta, rd, fast);
}
template <typename T, int UB, int W>
static void launch_tiles_x_uw(const TileBin &tb, hipStream_t s, const T *xs, int64_t sxr, int64_t sxc, int64_t xrows,
                              bool x4, T *ys, int64_t syr, int64_t syc, int nr, T alpha, T beta, int rd, int fast)
{
#define VBC_TILESX(MASKU, X4)                                                                                          \
    do {                                                                                                               \
        if constexpr (sizeof(T) == 4) {                                                                                \
            if (tb.nwaves == 8) {                                                                                      \
                launch_tiles_x_k<T, UB, W, MASKU, X4, 8>(tb, s, xs, sxr, sxc, xrows, ys, syr, syc, nr, alpha, beta, rd, fast); \
                break;                                                                                                 \
            }                                                                                                          \
        }                                                                                                              \
        launch_tiles_x_k<T, UB, W, MASKU, X4, 4>(tb, s, xs, sxr, sxc, xrows, ys, syr, syc, nr, alpha, beta, rd, fast); \
    } while (0)
    if (tb.masku) {
        if (x4) VBC_TILESX(true, true);
        else VBC_TILESX(true, false);
    } else {
        if (x4) VBC_TILESX(false, true);
        else VBC_TILESX(false, false);
    }
#undef VBC_TILESX
}
template <typename T, int UB>
static void launch_tiles_x_u(const TileBin &tb, hipStream_t s, const T *xs, int64_t sxr, int64_t sxc, int64_t xrows,
                             bool x4, T *ys, int64_t syr, int64_t syc, int nr, T alpha, T beta, int rd, int fast)
{
    switch (tb.w) {
    case 1: launch_tiles_x_uw<T, UB, 1>(tb, s, xs, sxr, sxc, xrows, x4, ys, syr, syc, nr, alpha, beta, rd, fast); break;
    case 2: launch_tiles_x_uw<T, UB, 2>(tb, s, xs, sxr, sxc, xrows, x4, ys, syr, syc, nr, alpha, beta, rd, fast); break;
    case 3: launch_tiles_x_uw<T, UB, 3>(tb, s, xs, sxr, sxc, xrows, x4, ys, syr, syc, nr, alpha, beta, rd, fast); break;
    default: launch_tiles_x_uw<T, UB, 4>(tb, s, xs, sxr, sxc, xrows, x4, ys, syr, syc, nr, alpha, beta, rd, fast); break;
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
            if (tb.staged) {
                const bool x4 = nr == 16 && sxc == 1 && (sxr * (int64_t)sizeof(T)) % 16 == 0 &&
                                reinterpret_cast<uintptr_t>(xs) % 16 == 0;
                const int fastx = nr == 16 && syc == 1 && syr == 16 && reinterpret_cast<uintptr_t>(ys) % 16 == 0;
                if constexpr (sizeof(T) == 4) {
                    if (h->tile_persist && x4 && fastx && tb.nwg > 0 && tiles_xp_lds(tb) <= (size_t)kTileXPLds) {
                        const float *xf = reinterpret_cast<const float *>(xs);
                        float *yf = reinterpret_cast<float *>(ys);
                        switch (tb.ub) {
                        case 1: launch_tiles_xp_u<1>(tb, s, xf, sxr, xrows, yf, (float)alpha, (float)beta, rd); break;
                        case 2: launch_tiles_xp_u<2>(tb, s, xf, sxr, xrows, yf, (float)alpha, (float)beta, rd); break;
                        case 3: launch_tiles_xp_u<3>(tb, s, xf, sxr, xrows, yf, (float)alpha, (float)beta, rd); break;
                        default: launch_tiles_xp_u<4>(tb, s, xf, sxr, xrows, yf, (float)alpha, (float)beta, rd); break;
                        }
                        VBC_HIP(hipGetLastError());
                        continue;
                    }
                }
                switch (tb.ub) {
                case 1: launch_tiles_x_u<T, 1>(tb, s, xs, sxr, sxc, xrows, x4, ys, syr, syc, nr, (T)alpha, (T)beta, rd, fastx); break;
                case 2: launch_tiles_x_u<T, 2>(tb, s, xs, sxr, sxc, xrows, x4, ys, syr, syc, nr, (T)alpha, (T)beta, rd, fastx); break;
                case 3: launch_tiles_x_u<T, 3>(tb, s, xs, sxr, sxc, xrows, x4, ys, syr, syc, nr, (T)alpha, (T)beta, rd, fastx); break;
                default: launch_tiles_x_u<T, 4>(tb, s, xs, sxr, sxc, xrows, x4, ys, syr, syc, nr, (T)alpha, (T)beta, rd, fastx); break;
                }
                VBC_HIP(hipGetLastError());
                continue;
            }
            // one contiguous run of Y per range: affine map of stride w, 16 contiguous right-hand sides
            const bool rows16 = nr == 16 && syc == 1 && syr == 16 && reinterpret_cast<uintptr_t>(ys) % 16 == 0;
            int fast = tb.out_affine && tb.out_stride == tb.w && rows16 ? 1 : 0;
            // (the dword form: stripes in another order still store 16-B pieces of each stripe's block)
            const int fast_dw = fast ? 1 : (rows16 ? 2 : 0);
            const int grid = (tb.nranges + kWavesPerBlock - 1) / kWavesPerBlock;
            // the 16-B form: fp32, 16 contiguous right-hand sides in 16-B aligned rows (one dwordx4 per tile row)
            if constexpr (sizeof(T) == 4) {
                const bool x4 = h->tile_x4 && buf && nr == 16 && sxc == 1 && (sxr * 4) % 16 == 0 &&
                                reinterpret_cast<uintptr_t>(xs) % 16 == 0;
                if (x4) {
                    const float *xf = reinterpret_cast<const float *>(xs);
                    float *yf = reinterpret_cast<float *>(ys);
                    switch (tb.ub) {
                    case 1: launch_tiles4_u<1>(tb, grid, s, xf, sxr, xb, yf, syr, syc, (float)alpha, (float)beta, rd, fast); break;
                    case 2: launch_tiles4_u<2>(tb, grid, s, xf, sxr, xb, yf, syr, syc, (float)alpha, (float)beta, rd, fast); break;
                    case 3: launch_tiles4_u<3>(tb, grid, s, xf, sxr, xb, yf, syr, syc, (float)alpha, (float)beta, rd, fast); break;
                    default: launch_tiles4_u<4>(tb, grid, s, xf, sxr, xb, yf, syr, syc, (float)alpha, (float)beta, rd, fast); break;
                    }
                    VBC_HIP(hipGetLastError());
                    continue;
                }
            }
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
