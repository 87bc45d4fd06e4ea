// Host-side handle and launch descriptors shared by libvbc's translation units (vbc_device.hip:
// creation and the C ABI; vbc_launch.hip / vbc_panel_launch.hip: the kernel launches).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <vector>

#include "vbc_internal.h"
#include "vbc_kernels.h"
#include "vbc_panel.h"
#include "vbc_tiles.h"

namespace vbc {

#define VBC_HIP(call)                                                                             \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            set_error("%s failed: %s", #call, hipGetErrorString(e_));                             \
            return VBC_HIP_ERROR;                                                                 \
        }                                                                                         \
    } while (0)

// One fused launch of spmv_ranges (+ its fix-up pass).
struct Launch {
    std::vector<Bin> bins;
    Bin *d_bins = nullptr;
    int total_ranges = 0;
    int nfill = 0;
    size_t o_fill = 0;             // arena offset of the fill list (y indices)
    const int32_t *d_fill = nullptr;
    std::vector<SlotBin> sbins;    // slotted buckets (vbc_slots.h), launched before the merge kernel
    SlotBin *d_sbins = nullptr;
    int slot_ranges = 0;
    std::vector<SlotBin> pbins;    // planar slotted buckets (vbc_planar.h), one launch each
    SlotBin *d_pbins = nullptr;
    std::vector<SweepBin> wbins;   // row-swept buckets (vbc_sweep.hip, B'x only), launched first
    SweepBin *d_wbins = nullptr;
    int sweep_tiles = 0;
    int sweep_tile_bytes = 0;      // LDS accumulator bytes per wave the layout was cut for
    int sweep_diag = 0;            // VBC_SWEEP_DIAG ablation (tools/ab.py only)
    // B'x with several independent launch groups (swept, slotted, each planar bucket, merge + fix-up:
    // disjoint stripes of y): the groups after the first run on side streams forked from the caller's
    // stream by an event and joined back, so small buckets overlap instead of queueing one after the
    // other (graph capture records them as parallel branches).  Empty when one group or VBC_FORK=0.
    // small mixed-width B'x (vbc_device.hip build_transposed): every planar split bin in ONE launch of
    // spmv_split_multi with fuse_split waves per chunk (0: one launch per planar bin)
    int fuse_split = 0;
    int fuse_p = 0;  // the fused split's P as build_transposed chose it (finalize_launch builds `multi`)
    SplitMulti multi{};
    std::vector<double> gwork;  // matrix bytes of each launch group (launch_groups order): the heaviest is
                                // submitted last, so the small groups are already dispatched when it fills the chip
    std::vector<hipStream_t> fork_streams;
    std::vector<hipEvent_t> fork_events;  // [0]: the fork, [1 + i]: side stream i done
};

// The panel layout of the MFMA multi-RHS transposed product (vbc_panel.h): one launch.
struct PanelLaunch {
    std::vector<PanelBin> bins;
    PanelBin *d_bins = nullptr;
    std::vector<TileBin> tbins;  // small-tile buckets (vbc_tiles.h, u, w <= 4): one launch each
    int total_ranges = 0;
    int nfill = 0;
    size_t o_fill = 0;
    const int32_t *d_fill = nullptr;
};

// Integer-eltype layout (vbc_generic.hip): the reference layout itself, 0-based, on the device.
struct IntLayout {
    int64_t L = 0, nrows = 0;
    const int32_t *col0 = nullptr, *w = nullptr, *rows = nullptr;  // per stripe / per stored row
    const int32_t *col2stripe = nullptr;  // per column j: its stripe
    const int32_t *row2stripe = nullptr;  // per stored row: its stripe
    const int64_t *rbeg = nullptr;        // L+1 prefix into rows
    const int64_t *voff = nullptr;        // per stripe: first value
    const int64_t *val = nullptr;         // values as Int64
};

// Host description of the input stripes, common to 1D, 2D (expanded) and CSC inputs.
struct Stripes {
    int64_t m = 0, n = 0, L = 0;
    std::vector<int64_t> col0;  // 0-based first column of stripe l
    std::vector<int32_t> w;     // width
    std::vector<int64_t> rbeg;  // L+1 prefix into rows
    std::vector<int32_t> rows;  // 0-based x row of each stored w-wide row
    std::vector<int64_t> voff;  // element offset of the stripe's first value in the input val
    std::vector<int32_t> vst;   // per stripe: elements between its stored rows' values (empty: the width;
                                // a column piece keeps its source stripe's stride)
    int64_t vstride(int64_t l) const { return vst.empty() ? w[l] : vst[l]; }
    std::vector<int64_t> grp;   // 2D input: Π's block-row starts (K + 1, 0-based); empty for 1D / CSC
};

}  // namespace vbc

struct vbc_handle {
    int64_t m = 0, n = 0, L = 0, K = 0, nblocks = 0, nrows = 0, nval = 0, nnz = 0;
    int dtype = 0, esz = 8, device = 0;
    void *d_arena = nullptr;
    size_t arena_bytes = 0;
    bool has_t = false, has_f = false, has_m = false;
    vbc::PanelLaunch lm;          // multi-RHS transposed product on matrix cores (VBC_CREATE_MULTI)
    int64_t bytes_m = 0;          // matrix bytes one panel product streams
    vbc::PanelLaunch lmf;         // multi-RHS forward product on matrix cores (VBC_CREATE_MULTI_FORWARD): the
                                  // panel layout of Bᵀ (output row groups as stripes, tile columns as rows)
    bool has_mf = false;
    int64_t bytes_mf = 0;         // matrix bytes one forward panel product streams
    int32_t mf_group = 0;         // forward panel: widest output row group
    int target_ranges_m = 4096;
    int panel_valu = 0;           // ablation bits of the panel kernel (VBC_PANEL_VALU / VBC_PANEL_DIAG, the VBC_ABLATION
                                  // build only; 0 in the product library)
    int panel_nobuf = 0;          // VBC_PANEL_NOBUF=1: 64-bit addressing variant (tests / A/B)
    int panel_tiles = -1;         // VBC_PANEL_TILES: small-tile buckets tile-granular (vbc_tiles.h): -1 auto, 0 never,
                                  // 1 whenever representable (any fill)
    int occ_tiles = 24;           // resident waves per CU of the tile kernel (the layout's range count)
    int tile_nbt = vbc::kTileBatch;  // VBC_TILE_NBT: tiles per stream per pipeline stage of the tile kernel (4 / 8)
    int tile_depth = 2;  // VBC_TILE_DEPTH (VBC_ABLATION build): register sets of the tile kernel's pipeline (2 / 3)
    int tile_cluster = 1;             // VBC_TILE_CLUSTER=0: tile ranges launched in natural stripe order (no X-locality balls);
                                      // 2: balls at any range count (tests)
    int tile_spr = vbc::kTileStripes;  // VBC_TILE_SPR: stripes per range (wave) of the tile layout
    int64_t panel_val_bytes = 0;  // largest bin val array of the panel layout
    vbc::IntLayout li;            // integer eltypes (dtype VBC_I64): exact wrapping products
    vbc::Launch lt;               // transposed product: all buckets in one launch
    vbc::Launch lft;              // forward product as the transposed product of C = Bᵀ (small mixed widths)
    bool has_ft = false;
    int fwd_t = 1;                // VBC_FWD_T: 0 never build the forward product on C = Bᵀ, 2 always
    std::vector<vbc::Launch> lf;  // forward product: one launch per width bucket
    bool f_scale = false;         // forward with several buckets: scale y by beta first
    int64_t bytes_t = 0, bytes_f = 0;
    void *d_carry_mm = nullptr;   // multi-RHS carry slots (allocated on first use)
    size_t carry_mm_bytes = 0;
    int target_ranges_k[2] = {4096, 4096};  // resident waves of the B'x / Bx kernels (one range each)
    int tile_k = vbc::kTileKDefault;  // entries per slot per tile
    int lanes_rdiv = 2;               // VBC_LANES_RDIV: lane-stream tiles sized for target_ranges_l / this many ranges
    int pipe = vbc::kPipeDefault;     // software-pipeline depth (2 or 3 tiles)
    int diag = 0;                     // ablation variant (VBC_DIAG; tools/ab.py only)
    int target_ranges_s[2] = {4096, 4096};  // resident waves of the slotted kernels
    int slots_mode = -1;              // VBC_SLOTS: -1 auto, 0 never, 1 always (when representable)
    double slots_pad = 1.10;          // auto: largest padded/real row ratio of a slotted bucket
    int slot_narrow = 1;              // VBC_SLOT_NARROW=0: one segment per lane slot for narrow B'x rows too
    int slots_sort = 1;               // VBC_SLOTS_SORT: 0 natural order only, 1 sort when needed, 2 always sort
    int xcd = 1;                      // VBC_XCD=0: identity block order in the slotted kernel (XCD-contiguous ranges:
                                      // FE 170.3 -> 169.2 us, its 1/8 stripe shard 28.1 -> 26.0 us)
    int64_t range_bytes = 192 << 10;  // VBC_RANGE_KB: a slotted bucket with fewer layout bytes per range at full
                                      // occupancy runs half the waves per SIMD (longer ranges)
    int xcd_p = 1;                    // VBC_XCD_P=0: identity workgroup order in the planar kernels (XCD-contiguous:
                                      // ldoor stand-in fp64 76.8 -> 70.2 us, fp32 44.6 -> 39.8, TrSpMV! 44.6 -> 39.3)
    int occ_s[2] = {4, 4};            // workgroups per CU of the slotted kernels (occupancy)
    int64_t slot_rows_padded = 0, slot_rows_real = 0;  // entries of slotted buckets (with / without padding)
    int64_t slot_rows_padded_last = 0;
    int slot_u = 0;                   // rows per step of the slotted kernel (VBC_SLOT_U)
    bool slot_dedup = true;           // VBC_SLOT_DEDUP=0: one stored delta pattern per compressed row
    int slot_keys16 = 1;              // VBC_SLOT_KEYS16: 0 keep 32-bit keys, 1 auto, 2 compress whenever possible
    int fork = 1;                     // VBC_FORK=0: B'x launch groups queue on the caller's stream (Launch::fork_*)
    int slot_stage = -1;              // VBC_SLOT_STAGE = 0 / 4 / 8: chunks staged in LDS per y write (-1 auto)
    int slot_planar = -1;             // VBC_SLOT_PLANAR: -1 auto (B'x, w = 3..8 wider than a lane vector), 0 never, 1 w >= 3
    int slot_runs = 1;                // VBC_SLOT_RUNS=0: no row-run gathers in planar buckets
    int planar_pair = 1;              // VBC_PLANAR_PAIR: 0 never, 1 auto (>= 8 runs per stripe), 2 always (fp64 w = 3 runs)
    int planar_mask = 1;              // VBC_PLANAR_MASK: planar B'x buckets whose natural order pads > slots_pad: 1 masked
                                      // chunk-local length order (SlotBin::mask), 0 length-sorted windows of 32 chunks
    int planar_mask_pair = 1;         // VBC_PLANAR_MASK_PAIR=0: the lane-pair kernel folds its padding rows (no nlive)
    int mask_window = 2;              // VBC_MASK_WINDOW: chunks per length-sort window of the masked order (a prefix
                                      // of live lanes holds in every chunk of a window sorted by decreasing length;
                                      // fe3d fp64 1 / 2 / 4 / 8: 284 / 276 / 284 / 287 us, fp32 145 / 145 / 152 / 159,
                                      // ldoor fp32 37.2 / 37.1 / 36.5 / 36.3)
    int planar_split = -1;            // VBC_PLANAR_SPLIT: -1 auto (few chunks), 0 never, 2 / 4 / 8 waves per chunk
    int target_ranges_p = 4096;       // resident waves of the planar kernel
    int target_ranges_l = 4096;       // resident waves of the lane-stream planar kernel
    int slot_wonly = 1;               // VBC_SLOT_WONLY=0: the all-width slotted kernel even for one-width launches
    int split_kc = 0;                 // VBC_SPLIT_KC=1: compressed keys for split planar bins too
    int small_split = 0;              // > 1: this B'x layout is the fused small-matrix split with P waves per chunk
    uint32_t fuse_w = 0;              // bit w: the width-w bucket belongs to the fused split (all, or the side buckets)
    int small_fuse = 1;               // VBC_SMALL_FUSE: 0 = never fuse the buckets of a small matrix
    int side_fuse = -1;               // VBC_SIDE_FUSE: the dominant bucket outside the fused split (-1 auto, 0 never,
                                      // 1 whenever one width holds >= 80 % of the chunks)
    int colsplit = 1;                 // VBC_COLSPLIT=0: no column pieces (side stripes of a multiple of the
                                      // dominant width run as that many dominant-width stripes)
    double fork_side_bytes = 1 << 20; // VBC_FORK_SIDE_KB: beside a group with >= 90 % of the bytes, the others fork only
                                      // while they hold at most this many bytes
    int fuse_pmax = 8;                // VBC_FUSE_PMAX: most waves per chunk of the fused split launch (2 / 4 / 8; P = 16,
                                      // 1024-thread workgroups, measured 1.4-1.9x slower: profiles/r04_ab20_*.log)
    int colsplit_w = 0;               // VBC_COLSPLIT_W=c: every stripe wider than c as c-wide pieces (A/B)
    int64_t split_nt_bytes = 0;       // VBC_SPLIT_NT_MB: value bytes above which split bins stream nt (0: never)
    int small_rows = 8;               // VBC_SMALL_ROWS: fewest chunk rows per wave (fp64) of the fused small split
    int cus = 256;                    // compute units of the device
    int occ_multi[4] = {0, 0, 0, 0};  // resident waves per CU of the fused split launch, P = 2 / 4 / 8 (index log2 P)
    double ksplit = 1.0;              // VBC_KSPLIT: fused split stripes above this x the mean chunk work are cut
                                      // into 2 / 4 lane parts (SlotBin::ks; 0: never)
    int split_pipe = -1;              // VBC_SPLIT_PIPE: split bins' pipelined slice loop (-1 auto, 0 off, 1 on)
    double split_deep = 2.0;          // VBC_SPLIT_DEEP: auto slice loop batched above this many steps per wave
    int split_rows = 12;              // VBC_SPLIT_ROWS: fewest chunk rows per wave of an automatic split
    int fwd_min_rows = 16;            // VBC_FWD_MIN_ROWS: fewest chunk rows per range of the forward run layout
    int planar_wps = 2;               // VBC_PLANAR_WPS: most resident waves per SIMD of a plain planar bin (0: occupancy)
    int planar_wps_pair = 1;          // VBC_PLANAR_WPS_PAIR: the same for the fp64 lane-pair layout
    int lanes_pair = 0;               // VBC_LANES_PAIR=1: a lane pair per stream in the lane-stream layout (fp64 w = 3,
                                      // runs of 3; one 16-B x gather per lane per run).  FE-3D measured 217 -> 223 us
                                      // with pairs (profiles/r03_ab_pairlanes_fe3d.log), so off by default
    int lanes_deep = 0;               // VBC_LANES_DEEP=1: the lanes kernel's deeper pipeline (gathers a step ahead)
    int planar_lanes = -1;            // VBC_PLANAR_LANES: -1 auto, 0 never, 1 always (planar B'x buckets with
                                      // natural contiguous outputs): per-lane compacted streams (run_planar_lanes)
    int occ_p = 4;                    // workgroups per CU of the planar kernel
    int sweep_mode = -1;              // VBC_SWEEP: -1 auto (no x locality), 0 never, 1 always (w <= 8)
    int sweep_tile = vbc::kSweepTileBytes;  // VBC_SWEEP_TILE=16: 16 KB of LDS accumulators per wave
    int sweep_pack = 1;               // VBC_SWEEP_PACK=0/1: swept keys as gather index + 16-bit segment (6 B per
                                      // entry, two loads) or one packed 32-bit key per entry (default: fp64)

    // Mutable per-handle state, guarded by `mu` (the layout itself is immutable after create):
    //  * host-pointer staging buffers, grown on demand and reused across calls (VBC_MEM_HOST);
    //  * the product order of handles whose layout has shared scratch (the merge layout's carry
    //    slots and the fused multi-RHS carries): a product enqueued on a different stream than the
    //    previous one first waits for that one's completion event, so concurrent products on
    //    distinct streams stay correct.  Slotted / swept / panel layouts hold no scratch and skip it.
    std::mutex mu;
    std::mutex fork_mu;               // the fork / join event sequence of a forked B'x launch (Launch::fork_*)
    void *d_stage[4] = {nullptr, nullptr, nullptr, nullptr};  // x / X, y / Y staging; 2, 3: column temporaries
    size_t stage_bytes[4] = {0, 0, 0, 0};
    bool has_scratch = false;         // set at create: some launch of this handle uses carry slots
    hipEvent_t order_ev = nullptr;    // recorded after each product with scratch
    hipStream_t order_stream = nullptr;
    bool order_valid = false;
};


namespace vbc {

// vbc_launch.hip
int launch_groups(const Launch &L);  // independent launch groups of a B'x launch (vbc_launch.hip)
int mul_dispatch(const vbc_handle *h, int trans, const void *x, void *y, double alpha, double beta,
                 hipStream_t stream);
int mulmat_rowmajor(vbc_handle *h, int64_t nrhs, const char *X, int64_t ldx, char *Y, int64_t ldy, double alpha,
                    double beta, hipStream_t s);
void occupancy_ranges(int esz, int K, int P, int occ[2]);
// vbc_generic.hip
int mul_int(const vbc_handle *h, int trans, const void *x, void *y, double alpha, double beta, hipStream_t s);
int convert_gather(const void *src, int src_dtype, int64_t inc, void *dst, int dst_dtype, int64_t n, hipStream_t s);
int convert_scatter(const void *src, int src_dtype, void *dst, int dst_dtype, int64_t inc, int64_t n, hipStream_t s);
// vbc_panel_launch.hip
int mulmat_panel_any(const vbc_handle *h, int trans, int64_t nrhs, const char *X, int64_t sxr, int64_t sxc, char *Y,
                     int64_t syr, int64_t syc, double alpha, double beta, hipStream_t s);
int occupancy_panel(int esz);
// vbc_tiles.hip
int mulmat_tiles_any(const vbc_handle *h, int trans, int64_t nrhs, const char *X, int64_t sxr, int64_t sxc, char *Y,
                     int64_t syr, int64_t syc, double alpha, double beta, hipStream_t s);
int occupancy_tiles(int esz);

}  // namespace vbc
