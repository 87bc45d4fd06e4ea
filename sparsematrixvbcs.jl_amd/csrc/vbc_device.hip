// libvbc device side: handle creation (reference layout -> tiled HBM entry streams), product launches
// and the C ABI of include/vbc.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstring>
#include <cmath>
#include <map>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "vbc_handle.h"
#include "vbc_planar.h"

namespace vbc {

static thread_local std::string g_err;

void set_error(const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

// Restores the caller's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Arena builder: reserves aligned regions, fills a host image, uploads once.
struct Arena {
    std::vector<char> host;
    size_t reserve(size_t bytes)
    {
        size_t off = (host.size() + 255) & ~size_t(255);
        host.resize(off + std::max<size_t>(bytes, 1));
        return off;
    }
    template <typename U>
    U *at(size_t off) { return reinterpret_cast<U *>(host.data() + off); }
};

struct PendingBin {
    Bin b;
    size_t o_key, o_val, o_rseg, o_out, o_carry, o_cseg;
    double work = 0;  // matrix bytes the bin streams (launch-group ordering)
};

static int check_limits(const Stripes &s)
{
    if (s.m >= (int64_t(1) << 31) || s.n >= (int64_t(1) << 31))
        return fail(VBC_INVALID_ARG, "m and n must be < 2^31 on the GPU path");
    for (int32_t w : s.w)
        if (w > 64) return fail(VBC_UNSUPPORTED_DTYPE, "stripe width > 64 is not supported on the GPU path");
    return VBC_OK;
}

// A logical entry of a bucket's stream: gather index + where its w values come from.
struct Entry {
    uint32_t key;   // gather index | HEAD
    int64_t voff;   // element offset into the input val
};

// Lay out one bucket's entry stream (segment-ordered) as tiles, ranges and fix-up slots.
static int build_bucket(vbc_handle *h, int kind, int w, const std::vector<Entry> &ents,
                        const std::vector<int32_t> &out, int64_t total_entries, const char *val,
                        Arena &ar, int &range0, PendingBin &pb, int wsrc = 0)
{
    // wsrc < w: the entries carry wsrc values each, stored w wide with zero padding columns
    if (wsrc <= 0) wsrc = w;
    const int esz = h->esz;
    const int V = w <= 8 ? vec_elems(esz, w) : 1;
    const int LPR = w / V;
    const int RPI = 64 / LPR;
    const int K = h->tile_k;
    const int64_t tile_rows = (int64_t)RPI * K;
    const int64_t R = (int64_t)ents.size();
    const int64_t ntiles = (R + tile_rows - 1) / tile_rows;
    if (ntiles >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "bucket too large");
    if ((int64_t)out.size() >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "too many segments");
    // ranges: one wave each, about target_ranges over the whole launch, >= 2 tiles per range
    int64_t nr = (int64_t)std::llround((double)h->target_ranges_k[kind] * (double)R / (double)std::max<int64_t>(total_entries, 1));
    nr = std::max<int64_t>(1, std::min<int64_t>(nr, (ntiles + 1) / 2));
    const int64_t tpr = ntiles > 0 ? (ntiles + nr - 1) / nr : 1;
    nr = ntiles > 0 ? (ntiles + tpr - 1) / tpr : 0;
    pb = PendingBin{};
    pb.b.kind = kind;
    pb.b.wkey = w <= 8 ? w : 0;
    pb.b.w = w;
    pb.b.wst = wsrc;
    pb.b.rpi = RPI;
    pb.b.range0 = range0;
    pb.b.nranges = (int32_t)nr;
    pb.b.tiles_per_range = (int32_t)tpr;
    pb.b.ntiles = (int32_t)ntiles;
    pb.b.tile_k = K;
    pb.b.pipe = h->pipe;
    pb.b.diag = h->diag;
    pb.b.out_affine = 1;
    pb.b.out_base = out.empty() ? 0 : out[0];
    pb.b.out_stride = out.size() > 1 ? out[1] - out[0] : 0;
    for (size_t q = 1; q < out.size() && pb.b.out_affine; q++)
        pb.b.out_affine = (int64_t)out[q] == (int64_t)out[0] + (int64_t)q * pb.b.out_stride;
    if (ablation_knob("VBC_NO_AFFINE")) pb.b.out_affine = 0;  // (the VBC_ABLATION build only)
    range0 += (int)nr;
    const int64_t Rp = ntiles * tile_rows;
    pb.o_key = ar.reserve(Rp * 4);
    pb.o_val = ar.reserve(Rp * w * esz);
    pb.o_rseg = ar.reserve(std::max<int64_t>(nr, 1) * 4);
    pb.o_out = ar.reserve(std::max<size_t>(out.size(), 1) * 4);
    pb.o_carry = ar.reserve(std::max<int64_t>(nr, 1) * (kind == 0 ? w : 1) * esz);
    pb.o_cseg = ar.reserve(std::max<int64_t>(nr, 1) * 4);
    uint32_t *key = ar.at<uint32_t>(pb.o_key);
    char *vv = ar.at<char>(pb.o_val);
    int32_t *rseg = ar.at<int32_t>(pb.o_rseg);
    std::memcpy(ar.at<int32_t>(pb.o_out), out.data(), out.size() * 4);
    int64_t heads = 0;
    const int GV = val_group(esz, w);  // grouped tile layout (vbc_kernels.h key_pos / val_pos)
    for (int64_t t = 0; t < Rp; t++) {
        const int64_t tile = t / tile_rows, within = t - tile * tile_rows;
        const int slot = (int)(within / K), k = (int)(within - (int64_t)slot * K);
        const size_t pk = key_pos((size_t)(tile * tile_rows), k, slot, RPI);
        const size_t pv = val_pos((size_t)(tile * tile_rows), k, slot, RPI, GV);
        if (within == 0 && tile % tpr == 0) rseg[tile / tpr] = (int32_t)heads;
        if (t < R) {
            key[pk] = ents[t].key;
            heads += (ents[t].key >> 31);
            std::memcpy(vv + pv * w * esz, val + ents[t].voff * esz, (size_t)wsrc * esz);
            if (wsrc < w) std::memset(vv + (pv * w + wsrc) * esz, 0, (size_t)(w - wsrc) * esz);
        } else {
            key[pk] = 0;  // padding extends the last segment by zeros
            std::memset(vv + pv * w * esz, 0, (size_t)w * esz);
        }
    }
    return VBC_OK;
}

// ---- slotted layout (vbc_slots.h) ----------------------------------------------------------------

struct PendingSlot {
    SlotBin b;
    size_t o_key, o_val, o_out, o_rrow, o_rchunk, o_base = 0, o_doff = 0, o_nlive = 0;
    size_t o_trow = 0, o_tseg = 0, o_lseg = 0;  // lanes layout (build_lanes)
    bool lanes_done = false;                    // keys already stored (build_lanes: 32-bit keys per run)
    int64_t key_bytes = 0;       // index bytes as stored (keys, deltas, bases, delta offsets)
    std::vector<uint32_t> keys;  // full keys until commit_slot_keys picks the stored form
    int64_t rows = 0;
    int64_t real = 0;            // entries without padding
    bool kc_ok = false;          // every row's keys fit base + int16 deltas
};

// Per-row base of the compressed form: the first non-padding key of the row (0 if none).
static bool slot_keys_compressible(const std::vector<uint32_t> &keys, int64_t rows, int RPI)
{
    for (int64_t r = 0; r < rows; r++) {
        const uint32_t *k = keys.data() + r * RPI;
        int64_t base = -1;
        for (int s = 0; s < RPI; s++) {
            if (k[s] & kPad) continue;
            const int64_t g = k[s] & kSlotIdx;
            if (base < 0) base = g;
            if (g - base < -32767 || g - base > 32767) return false;
        }
    }
    return true;
}

// Store a slotted bin's keys: full 32-bit keys, or (kc) per-row bases + int16 deltas.  Compressed rows
// with identical delta patterns are stored once (a mesh operator's interior chunks all share one --
// FE: [0, 2, 4, ...] -- so its delta stream collapses to a few KB that stay in L2); each row carries
// the offset of its pattern.  VBC_SLOT_DEDUP=0 keeps one pattern per row (A/B).
static void commit_slot_keys(PendingSlot &ps, bool kc, Arena &ar, bool dedup)
{
    const int RPI = ps.b.rpi;
    const int64_t E = ps.rows * RPI;
    ps.b.kc = kc ? 1 : 0;
    if (!kc) {
        ps.o_key = ar.reserve(E * 4);
        std::memcpy(ar.at<uint32_t>(ps.o_key), ps.keys.data(), E * 4);
        ps.key_bytes = E * 4;
    } else {
        std::vector<int16_t> d(E);
        std::vector<uint32_t> bs(ps.rows), doff(ps.rows);
        for (int64_t r = 0; r < ps.rows; r++) {
            const uint32_t *k = ps.keys.data() + r * RPI;
            uint32_t base = 0;
            for (int s = 0; s < RPI; s++)
                if (!(k[s] & kPad)) { base = k[s] & kSlotIdx; break; }
            bs[r] = base | (k[0] & kLast);
            for (int s = 0; s < RPI; s++)
                d[r * RPI + s] = (k[s] & kPad) ? INT16_MIN : (int16_t)((int64_t)(k[s] & kSlotIdx) - (int64_t)base);
        }
        std::unordered_map<std::string, uint32_t> seen;
        int64_t stored = 0;  // distinct patterns, in rows
        for (int64_t r = 0; r < ps.rows; r++) {
            const int16_t *row = d.data() + r * RPI;
            if (dedup) {
                std::string kbytes(reinterpret_cast<const char *>(row), (size_t)RPI * 2);
                auto it = seen.find(kbytes);
                if (it != seen.end()) { doff[r] = it->second; continue; }
                seen.emplace(std::move(kbytes), (uint32_t)(stored * RPI));
            }
            if (stored != r) std::memmove(d.data() + stored * RPI, row, (size_t)RPI * 2);
            doff[r] = (uint32_t)(stored * RPI);
            stored++;
        }
        ps.o_key = ar.reserve(stored * RPI * 2);
        ps.o_base = ar.reserve(ps.rows * 4);
        ps.o_doff = ar.reserve(ps.rows * 4);
        std::memcpy(ar.at<int16_t>(ps.o_key), d.data(), (size_t)stored * RPI * 2);
        std::memcpy(ar.at<uint32_t>(ps.o_base), bs.data(), (size_t)ps.rows * 4);
        std::memcpy(ar.at<uint32_t>(ps.o_doff), doff.data(), (size_t)ps.rows * 4);
        ps.key_bytes = stored * RPI * 2 + ps.rows * 8;
    }
    std::vector<uint32_t>().swap(ps.keys);
}

// Segments per lane of a B'x bucket whose rows are narrower than a 16-B lane vector: fp32 w = 2 folds
// two segments side by side (run_slots_narrow); w = 1 (CSC) keeps one segment per lane (faster).
static int slot_spl(const vbc_handle *h, int kind, int w)
{
    if (kind != 0 || !h->slot_narrow) return 1;
    return (h->esz == 4 && w == 2) ? 2 : 1;  // the only narrow form that measured faster (vbc_slots.h)
}

// Planar chunk rows (vbc_planar.h) for a B'x bucket of width w: one stripe per lane whenever a row
// is wider than one 16-B lane vector would hold with a single lane (fp64 w >= 3, fp32 w >= 5) and for
// fp32 w = 3 (12-B rows, no padding to 4).
static bool slot_planar(const vbc_handle *h, int kind, int w)
{
    if (kind == 0 && h->small_split > 1 && w >= 1 && w <= 8 && ((h->fuse_w >> w) & 1)) return true;  // fused split (below)
    if (kind != 0 || h->slot_planar == 0 || w < 3 || w > 8) return false;
    return h->esz == 8 || w != 4;
}

// Slots per chunk of a bucket stored w wide (lane-vector width as in the kernel).
static int slot_rpi(const vbc_handle *h, int kind, int w)
{
    if (slot_planar(h, kind, w)) return 64;
    const int spl = slot_spl(h, kind, w);
    if (spl > 1) return 64 * spl;
    const int V = w <= 8 ? vec_elems(h->esz, w) : 1;
    return 64 / (w / V);
}

// Rows of each chunk: the longest segment of its RPI (>= 1, so every chunk closes).
static std::vector<int32_t> chunk_rows(const std::vector<int64_t> &sbeg, int RPI)
{
    const int64_t nseg = (int64_t)sbeg.size() - 1;
    std::vector<int32_t> cr((nseg + RPI - 1) / RPI, 1);
    for (int64_t q = 0; q < nseg; q++)
        cr[q / RPI] = (int32_t)std::max<int64_t>(cr[q / RPI], sbeg[q + 1] - sbeg[q]);
    return cr;
}

// Segment order of a sorted slotted bucket: by decreasing length inside windows of kSortWindow
// chunks (neighbouring segments stay near each other, so x locality survives the sort).
constexpr int kSortWindow = 32;
static std::vector<int64_t> sorted_order(const std::vector<int64_t> &sbeg, int RPI)
{
    const int64_t nseg = (int64_t)sbeg.size() - 1, win = (int64_t)kSortWindow * RPI;
    std::vector<int64_t> ord(nseg);
    for (int64_t i = 0; i < nseg; i++) ord[i] = i;
    for (int64_t a = 0; a < nseg; a += win) {
        const int64_t e = std::min(nseg, a + win);
        std::stable_sort(ord.begin() + a, ord.begin() + e, [&](int64_t p, int64_t q) {
            return sbeg[p + 1] - sbeg[p] > sbeg[q + 1] - sbeg[q];
        });
    }
    return ord;
}

static std::vector<int64_t> permuted_sbeg(const std::vector<int64_t> &sbeg, const std::vector<int64_t> &ord)
{
    std::vector<int64_t> p(sbeg.size());
    p[0] = 0;
    for (size_t i = 0; i < ord.size(); i++) p[i + 1] = p[i] + sbeg[ord[i] + 1] - sbeg[ord[i]];
    return p;
}

// Whether a bucket (segments sbeg over `real` entries) runs slotted: auto mode asks for a padded row
// count within slots_pad of the real one and chunks short enough to balance over the ranges, first
// in the natural segment order (affine y map), then sorted by length (y offsets from the table).
// Returns 0 (merge layout), 1 (slotted, natural order) or 2 (slotted, `order`).
// Chunk-local length order (SlotBin::mask): the segments of each window of `win` consecutive natural
// segments (mask_window chunks) by decreasing length -- the window keeps its segments (most of the
// x locality of the natural order: the sort over windows of 32 chunks lost it, FE-3D's x is fetched
// ~10x), and every chunk row's live lanes are a prefix, so the kernel points the dead lanes at lane
// 0's lines.
static std::vector<int64_t> chunk_sorted_order(const std::vector<int64_t> &sbeg, int win)
{
    const int64_t nseg = (int64_t)sbeg.size() - 1;
    std::vector<int64_t> ord(nseg);
    for (int64_t i = 0; i < nseg; i++) ord[i] = i;
    for (int64_t a = 0; a < nseg; a += win)
        std::stable_sort(ord.begin() + a, ord.begin() + std::min(nseg, a + win), [&](int64_t p, int64_t q) {
            return sbeg[p + 1] - sbeg[p] > sbeg[q + 1] - sbeg[q];
        });
    return ord;
}

// Padded / real rows a masked planar bucket may carry: padding costs instructions, not lines.
constexpr double kMaskPad = 3.0;
// Padded / real rows a bucket of the fused small-matrix split may carry in length-sorted order: a chunk
// costs its longest stripe's rows / P whatever its padding, and the padding rows read cached zeros.
constexpr double kSmallPad = 4.0;

static int want_slots(const vbc_handle *h, int kind, int w, const std::vector<int64_t> &sbeg,
                      int64_t total_entries, int64_t gather_limit, std::vector<int64_t> &order,
                      bool *mask = nullptr, int wsrc = -1)
{
    const bool fused = kind == 0 && h->small_split > 1 && wsrc >= 1 && wsrc <= 8 && ((h->fuse_w >> wsrc) & 1);
    if (mask) *mask = false;
    const int64_t nseg = (int64_t)sbeg.size() - 1;
    const int64_t real = nseg > 0 ? sbeg[nseg] - sbeg[0] : 0;
    order.clear();
    if (h->slots_mode == 0 || real == 0 || gather_limit >= (int64_t)kSlotIdxLimit) return 0;
    if (nseg >= (int64_t(1) << 31)) return 0;
    const int RPI = slot_rpi(h, kind, w);
    double pad_limit = 0;
    // (not for buckets small enough for the split product, which folds every padding row: build_slots)
    const double share_p = (double)h->target_ranges_p * (double)real / (double)std::max<int64_t>(total_entries, 1);
    // (P >= 4; a masked bucket skips P = 2: ldoor's 1/8 stripe shard, 615 chunks, masked lane pairs
    // 15.3 us vs split P = 2 16.3 us; the ct20stif stand-in, 273 chunks, keeps P = 4: 10.9 vs 12.8 us)
    const bool split_likely = h->planar_split != 0 && (double)((nseg + RPI - 1) / RPI) * 8 <= share_p;
    auto fits = [&](const std::vector<int64_t> &sb, bool force) {
        const std::vector<int32_t> cr = chunk_rows(sb, RPI);
        int64_t rows = 0, longest = 0;
        for (int32_t c : cr) { rows += c; longest = std::max<int64_t>(longest, c); }
        if (rows * RPI >= (int64_t(1) << 31)) return false;
        if (force) return true;
        const double ratio = (double)(rows * RPI) / (double)real;
        const double share = (double)h->target_ranges_s[kind] * (double)real / (double)std::max<int64_t>(total_entries, 1);
        const double rows_per_range = (double)rows / std::max(1.0, share);
        // (chunks are atomic: a planar w = 6 bucket of the ldoor stand-in with chunks up to 2x the rows
        // per range ran 193 us against the merge kernel's 171 us, profiles/r03_fork_ab2.log)
        return ratio <= (pad_limit > 0 ? pad_limit : h->slots_pad) && (double)longest <= std::max(64.0, 0.5 * rows_per_range);
    };
    if (fused && h->slots_mode != 0) {
        // fused small-matrix split (build_transposed): P waves fold every chunk, so a chunk longer than
        // the rows of a range does not unbalance anything; padding rows cost instructions and a few
        // cached lines of a matrix that stays in L2, so a sorted order may pad up to kSmallPad
        auto pad = [&](const std::vector<int64_t> &sb) {  // rows the chunks' lanes that hold a segment step through
            const std::vector<int32_t> cr = chunk_rows(sb, RPI);
            int64_t padded = 0;
            for (size_t c = 0; c < cr.size(); c++)
                padded += (int64_t)cr[c] * std::min<int64_t>(RPI, nseg - (int64_t)c * RPI);
            return (double)padded / (double)real;
        };
        // a bucket's padding counts against the whole launch: a few-chunk bucket (one chunk of 5 stripes,
        // one of them long) may pad far beyond kSmallPad and still add only a few workgroups' rows
        auto ok = [&](double p) { return p <= kSmallPad || (p - 1.0) * (double)real <= 0.05 * (double)total_entries; };
        if (h->slots_sort != 2 && (pad(sbeg) <= h->slots_pad || (h->slots_sort == 0 && ok(pad(sbeg))))) return 1;
        if (h->slots_sort == 0) return 0;
        order = sorted_order(sbeg, RPI);
        if (ok(pad(permuted_sbeg(sbeg, order)))) return 2;
        order.clear();
        return 0;
    }
    if (h->slots_sort != 2 && fits(sbeg, h->slots_mode == 1)) return 1;
    if (h->slots_sort == 0) return 0;
    if (mask && kind == 0 && h->planar_mask != 0 && slot_planar(h, 0, w) && !split_likely) {
        order = chunk_sorted_order(sbeg, RPI * h->mask_window);
        pad_limit = kMaskPad;
        if (fits(permuted_sbeg(sbeg, order), h->slots_mode == 1)) {
            *mask = true;
            return 2;
        }
        pad_limit = 0;
    }
    order = sorted_order(sbeg, RPI);
    if (fits(permuted_sbeg(sbeg, order), h->slots_mode == 1)) return 2;
    order.clear();
    return 0;
}

// Row runs of a planar bucket (SlotBin::run): the largest R in {3, 2} such that every segment's rows
// come in aligned runs of R consecutive x rows -- the dof rows of a node in a stiffness operator
// stored by node stripes (fe3d, the ldoor / ct20stif stand-ins).  The kernel then reads one key per
// run and gathers the run's R x values at once.  VBC_SLOT_RUNS=0 disables it (A/B, tests).
static int slot_runs(const vbc_handle *h, const std::vector<Entry> &ents, const std::vector<int64_t> &sbeg)
{
    if (h->slot_runs == 0) return 1;
    const int64_t nseg = (int64_t)sbeg.size() - 1;
    for (int R = 3; R >= 2; R--) {
        bool ok = sbeg[nseg] > sbeg[0];
        for (int64_t q = 0; q < nseg && ok; q++) {
            const int64_t b = sbeg[q], len = sbeg[q + 1] - b;
            if (len % R) { ok = false; break; }
            for (int64_t t = 0; t < len && ok; t += R)
                for (int d = 1; d < R; d++)
                    if (ents[b + t + d].key != ents[b + t].key + (uint32_t)d) { ok = false; break; }
        }
        if (ok) return R;
    }
    return 1;
}

// Lay out a slotted bucket: chunk rows row-major over the slots, PAD / LAST keys, ranges of whole
// chunks balanced by rows.  ents[sbeg[q] ...] are segment q's entries (keys = gather index only).
// pair_only: build nothing and return kBuildDeclined unless the bucket takes the lane-pair layout.
constexpr int kBuildDeclined = -1;
static int build_slots(vbc_handle *h, int kind, int w, int wsrc, const std::vector<Entry> &ents,
                       const std::vector<int64_t> &sbeg0, const std::vector<int32_t> &out0, int64_t total_entries,
                       const char *val, Arena &ar, int &range0, PendingSlot &ps,
                       const std::vector<int64_t> &order = {}, bool mask = false, int ks = 1, bool pair_only = false)
{
    const int esz = h->esz;
    // segment q of the layout is input segment order[q] (natural order when `order` is empty)
    const std::vector<int64_t> sbeg = order.empty() ? sbeg0 : permuted_sbeg(sbeg0, order);
    std::vector<int64_t> pstart(sbeg.size() - 1);
    std::vector<int32_t> out(out0.size());
    for (size_t q = 0; q < pstart.size(); q++) {
        const int64_t o = order.empty() ? (int64_t)q : order[q];
        pstart[q] = sbeg0[o];
        out[q] = out0[o];
    }
    const int64_t nseg = (int64_t)sbeg.size() - 1;
    int64_t nstripes = nseg;
    if (ks > 1) {  // stripes cut into ks parts (build_ksplit): out / nseg per stripe, lanes 0 .. 64/ks - 1
        const int m = 64 / ks;
        std::vector<int32_t> os;
        for (int64_t q = 0; q < nseg; q++)
            if (q % 64 < m && out[q] >= 0) os.push_back(out[q]);
        nstripes = (int64_t)os.size();
        out.swap(os);
    }
    const int64_t real = sbeg[nseg] - sbeg[0];
    const bool planar = slot_planar(h, kind, w);
    const int run = planar ? slot_runs(h, ents, sbeg0) : 1;  // sbeg0: the input order ents is in
    // runs with holes (build_transposed, hole_runs): absent rows are entries with voff < 0
    bool holes = false;
    for (const Entry &en : ents) holes = holes || en.voff < 0;
    if (holes && !(planar && run > 1 && kind == 0)) return fail(VBC_INVALID_ARG, "internal: runs with holes outside a planar B'x bin");
    // pair layout (vbc_planar.h run_pair): fp64 3-wide stripes with runs of 3, a lane pair per stripe
    // (for long segments: FE-3D's ~3 runs per stripe measured slower with 32-stripe chunks, 304 -> 315
    // us, ldoor's ~15 faster, 92 -> 81 us)
    bool pair = planar && run == 3 && esz == 8 && w == 3 && wsrc == 3 && h->planar_pair != 0 &&
                (h->planar_pair == 2 || real >= 3 * 8 * std::max<int64_t>(nseg, 1));
    int RPI = 0, split = 1;
    std::vector<int32_t> cr;
    int64_t nch = 0, rows = 0;
    const double target = planar ? (double)h->target_ranges_p : (double)h->target_ranges_s[kind];
    const double share = target * (double)real / (double)std::max<int64_t>(total_entries, 1);
    for (int attempt = 0; attempt < 2; attempt++) {
        RPI = pair ? 32 : slot_rpi(h, kind, w);
        cr = chunk_rows(sbeg, RPI);
        for (int32_t &c : cr) {
            c = (c + run - 1) / run * run;  // whole runs (an empty chunk: one padding run)
            if (pair) c /= 3;               // pair layout: rows are run-rows
        }
        nch = (int64_t)cr.size();
        rows = 0;
        for (int32_t c : cr) rows += c;
        // planar buckets with fewer chunks than wave slots: one chunk per workgroup of `split` waves
        split = 1;
        if (planar && kind == 0 && h->small_split > 1 && wsrc <= 8 && ((h->fuse_w >> wsrc) & 1)) {
            split = h->small_split;  // fused small-matrix split: one P for every bucket of the launch
        } else if (planar && h->planar_split != 0) {
            if (h->planar_split > 1) split = h->planar_split;
            else if ((double)nch / (pair ? 2 : 1) * 2 <= share) {  // in 64-stripe chunks
                // few chunks (at most half the wave slots): P waves per chunk while the grid stays within
                // twice the slots and every wave keeps >= 12 (fp64) / 6 (fp32) rows of its chunk.  Graph-
                // timed (profiles/r03_splitu_*.log, r03_split3_*.log): ct20stif stand-in fp64 (56 rows per
                // chunk) P = 2 6.5 us, 4 5.9, 8 6.2; fp32 5.1 / 4.3 / 4.2; ldoor's 1/8 shard fp64 11.5 /
                // 11.0 / 11.8, fp32 8.5 / 7.5 / 7.3; 1/4 shard fp64: lane pairs 22.3, P = 4 20.6; the 1/2
                // shard (2500 chunks) and the whole ldoor keep the lane pairs (37.6 vs P = 2 40.6; 67 vs 87)
                const double avg = (double)rows * (pair ? 3 : 1) / (double)std::max<int64_t>(nch, 1);  // x rows
                const double minrows = (double)h->split_rows * esz / 8.0;
                // (round 5: the doubled grid stays within ONE round of wave slots -- ldoor's 1/4 stripe shard,
                // 1249 chunks: P = 2 19.7 us, P = 4 20.5; the 1/8 shard keeps P = 4, 11.0 us against P = 2 11.8,
                // profiles/r05_shards_ab.log)
                while (split < 8 && (double)nch / (pair ? 2 : 1) * split * 2 <= share && avg / (split * 2) >= minrows)
                    split *= 2;
            }
        }
        // the split product runs the plain planar layout; so does a pair layout that would fill fewer than
        // half the wave slots, when the split product may be chosen instead (ldoor's 1/8 shard: 1250 pair
        // chunks 21.8 us, planar split 16.3 us)
        const bool drop = pair && (split > 1 || (!mask && h->planar_pair != 2 && h->planar_split != 0 && 2.0 * (double)nch < share));
        if (!drop) break;
        pair = false;
    }
    if (pair_only && !pair) return kBuildDeclined;  // (nothing reserved yet)
    int64_t nr = (int64_t)std::llround(share);
    // one wave per SIMD of the chip for this bucket (the target is CUs x occupancy x waves per workgroup)
    const double quantum = share / std::max(1, planar ? h->occ_p : h->occ_s[kind]);
    if (!planar && h->range_bytes > 0 && share >= 2 * quantum) {
        // small slotted buckets: half the waves per SIMD, each with a longer range (FE's stripe shards:
        // 1/2 89.7 -> 87.4 us, 1/4 49.0 -> 43.3 us, 1/8 28.1 -> 24.4 us; the full matrix keeps all)
        const double bytes = (double)rows * RPI * (w * esz + 4);
        if (bytes / share < (double)h->range_bytes) nr = (int64_t)std::llround(share / 2);
    }
    // plain planar bins: at most planar_wps waves per SIMD (fewer, longer ranges keep the resident
    // waves' x window in L2: ldoor fp64 lane pairs 3 -> 2 waves per SIMD 67.8 -> 65.4 us, fp32 4 -> 2
    // 36.5 -> 34.7 us, the C4 CSC product 36.7 -> 34.6 us; 1.5 or 2.5 per SIMD are slower,
    // profiles/r03_bxranges2_*.log, r03_wps_*.log)
    // (round 5: the fp64 lane-pair layout takes one wave per SIMD -- ldoor 64.4 -> 63.2 us, its 1/2 stripe
    // shard 36.5 -> 34.7 us; fp32 planar keeps two: ldoor fp32 34.9 vs 36.9, profiles/r05_shards_ab.log)
    const int wps = (pair && h->planar_wps_pair > 0) ? h->planar_wps_pair : h->planar_wps;
    if (planar && split == 1 && wps > 0) nr = std::min<int64_t>(nr, std::max<int64_t>(1, std::llround(quantum * wps)));
    nr = std::max<int64_t>(1, std::min<int64_t>(nr, nch));
    // fewer chunks than wave slots: whole waves per SIMD (ldoor's 1/4 shard: 2500 pair chunks as 2500
    // ranges 33.0 us, as 2048 ranges 27.7 us)
    const int64_t qi = (int64_t)quantum;
    if (split == 1 && qi >= 1 && nr < (int64_t)std::llround(share) && nr > qi) nr = nr / qi * qi;
    if (split > 1) nr = nch;
    bool affine = true;
    for (size_t q = 1; q < out.size() && affine; q++)
        affine = (int64_t)out[q] == (int64_t)out[0] + (int64_t)q * (out[1] - out[0]);
    std::vector<int32_t> rrow{0}, rchunk{0};
    int64_t acc = 0;
    for (int64_t c = 0; c < nch; c++) {
        acc += cr[c];
        // a table-mapped bin keeps <= kSlotOutEntries segments per range (their y offsets sit in LDS)
        const bool full = split > 1 || (!affine && (int64_t)(c + 2 - rchunk.back()) * RPI > kSlotOutEntries);
        if (c + 1 < nch && (full || ((int64_t)rrow.size() < nr && acc * nr >= (int64_t)rrow.size() * rows))) {
            rrow.push_back((int32_t)acc);
            rchunk.push_back((int32_t)(c + 1));
        }
    }
    rrow.push_back((int32_t)rows);
    nr = (int64_t)rchunk.size();
    if (layout_knob("VBC_VERBOSE"))
        fprintf(stderr, "[vbc] slot bin kind %d w %d planar %d pair %d run %d split %d chunks %lld rows %lld ranges %lld "
                "(target share %.0f)\n", kind, w, (int)planar, (int)pair, run, split, (long long)nch, (long long)rows,
                (long long)nr, share);
    ps = PendingSlot{};
    SlotBin &b = ps.b;
    b.kind = kind;
    b.wkey = w <= 8 ? w : 0;
    b.w = w;
    b.wst = wsrc;
    b.rpi = RPI;
    b.range0 = range0;
    b.nranges = (int32_t)nr;
    b.nseg = (int32_t)nstripes;
    b.ks = ks;
    b.fused = (planar && kind == 0 && split > 1 && h->small_split > 1 && wsrc <= 8 && ((h->fuse_w >> wsrc) & 1)) ? 1 : 0;
    b.u = h->slot_u;
    b.diag = h->diag;
    b.xcd = (planar && split == 1) ? h->xcd_p : 0;  // split grids are small (one chunk per workgroup)
    b.nowonly = h->slot_wonly ? 0 : 1;
    b.spl = slot_spl(h, kind, w);
    b.planar = planar ? 1 : 0;
    b.run = run;
    b.split = split;
    b.pair = pair ? 1 : 0;
    b.mask = (mask && planar && split == 1 && (!pair || h->planar_mask_pair)) ? 1 : 0;
    b.holes = holes ? 1 : 0;
    if (holes && (split == 1 || pair)) return fail(VBC_INVALID_ARG, "internal: runs with holes need the split product");
    if (planar && split > 1) {
        // split bins' slice loop (vbc_planar.h split_chunk): 0 one step at a time, 1 pipelined, 2 batched;
        // auto: the plain loop when a wave's slice is at most two steps of ~VBC_SPLIT_VALS values, else
        // batched (VBC_SPLIT_PIPE=0 / 1 / 2 forces one)
        const double rows_per_wave = (double)rows / (double)std::max<int64_t>(nch, 1) / split;
        const int u0 = (9 / w) / run * run;  // planar_split_step (vbc_planar.h, VBC_SPLIT_VALS = 9)
        const double step_rows = (double)std::min(8 * run, std::max(run, u0));
        // (fused bins only: a single-bucket split bin keeps the plain loop -- ldoor's 1/8 stripe shard 12.4 us
        // batched, 11.1 us plain, profiles/r04_ab22_*.log)
        b.deep = h->split_pipe >= 0 ? h->split_pipe : (b.fused && rows_per_wave > h->split_deep * step_rows ? 2 : 0);
        // VBC_SPLIT_NT_MB: above that many value bytes the batched loop reads keys and values non-temporally
        // (mode 3).  Off by default: slower on every table partition, the 300 MB ldoor 'min blocks' too
        // (68.3 -> 77.7 us; ct20stif strict 8.9 -> 12.3 us; profiles/r04_ab4_*.log)
        if (b.deep == 2 && h->split_nt_bytes > 0 && (double)h->nval * h->esz > (double)h->split_nt_bytes) b.deep = 3;
    }
    b.out_affine = 1;
    b.out_base = out.empty() ? 0 : out[0];
    b.out_stride = out.size() > 1 ? out[1] - out[0] : 0;
    for (size_t q = 1; q < out.size() && b.out_affine; q++)
        b.out_affine = (int64_t)out[q] == (int64_t)out[0] + (int64_t)q * b.out_stride;
    if (ablation_knob("VBC_NO_AFFINE")) b.out_affine = 0;  // (the VBC_ABLATION build only)
    {
        const int V = w <= 8 ? vec_elems(esz, w) : 1;
        const bool full = b.spl > 1 || planar || (RPI * (w / V) == 64 && V * esz <= 16);
        b.contig = b.out_affine && (kind == 0 ? (full && wsrc == w && (nseg <= 1 || b.out_stride == w))
                                              : (nseg <= 1 || b.out_stride == 1));
    }
    if (planar) b.range0 = 0;  // its own launch
    else range0 += (int)nr;
    const int64_t E = rows * RPI;
    ps.rows = rows;
    ps.real = real;
    ps.keys.resize(E);
    ps.o_val = ar.reserve(E * w * esz * (pair ? 3 : 1));
    ps.o_out = ar.reserve(std::max<size_t>(out.size(), 1) * 4);
    ps.o_rrow = ar.reserve(rrow.size() * 4);
    ps.o_rchunk = ar.reserve(rchunk.size() * 4);
    if (b.mask) ps.o_nlive = ar.reserve((size_t)rows * 4);
    std::memcpy(ar.at<int32_t>(ps.o_out), out.data(), out.size() * 4);
    std::memcpy(ar.at<int32_t>(ps.o_rrow), rrow.data(), rrow.size() * 4);
    std::memcpy(ar.at<int32_t>(ps.o_rchunk), rchunk.data(), rchunk.size() * 4);
    uint32_t *key = ps.keys.data();
    char *vv = ar.at<char>(ps.o_val);
    int64_t row = 0;
    if (pair) {  // run-rows of 32 stripes: segments A (64 lanes x 16 B), B, C, D (vbc_planar.h run_pair)
        double *dv = reinterpret_cast<double *>(vv);
        for (int64_t c = 0; c < nch; c++) {
            for (int32_t qr = 0; qr < cr[c]; qr++, row++) {
                const uint32_t last = qr + 1 == cr[c] ? kLast : 0u;
                double *blk = dv + row * 288;
                if (b.mask) {  // live stripe slots of this run-row: a prefix in chunk-local length order
                    uint32_t nl = 0;
                    for (int sl = 0; sl < 32; sl++) {
                        const int64_t seg = c * 32 + sl;
                        if (seg < nseg && sbeg[seg] + 3 * qr < sbeg[seg + 1]) {
                            if (nl != (uint32_t)sl) return fail(VBC_INVALID_ARG, "masked pair chunk: live slots not a prefix");
                            nl++;
                        }
                    }
                    ar.at<uint32_t>(ps.o_nlive)[row] = nl;
                }
                for (int sl = 0; sl < 32; sl++) {
                    const int64_t seg = c * 32 + sl, e = row * 32 + sl;
                    const bool real_run = seg < nseg && sbeg[seg] + 3 * qr < sbeg[seg + 1];
                    double v[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
                    if (real_run) {
                        for (int d = 0; d < 3; d++)
                            std::memcpy(v[d], val + ents[pstart[seg] + 3 * qr + d].voff * esz, 3 * sizeof(double));
                        key[e] = ents[pstart[seg] + 3 * qr].key | last;
                    } else {
                        key[e] = kPad | last;
                    }
                    blk[4 * sl + 0] = v[0][0];
                    blk[4 * sl + 1] = v[0][1];
                    blk[4 * sl + 2] = v[0][2];
                    blk[4 * sl + 3] = v[1][2];
                    blk[128 + 2 * sl + 0] = v[1][0];
                    blk[128 + 2 * sl + 1] = v[1][1];
                    blk[192 + sl] = v[2][2];
                    blk[224 + 2 * sl + 0] = v[2][0];
                    blk[224 + 2 * sl + 1] = v[2][1];
                }
            }
        }
    }
    for (int64_t c = 0; c < (pair ? 0 : nch); c++) {
        for (int32_t qr = 0; qr < cr[c]; qr++, row++) {
            const uint32_t last = qr + run == cr[c] ? kLast : 0u;  // on the last run's first row
            if (b.mask) {  // live lanes of this chunk row: a prefix in chunk-local length order
                uint32_t nl = 0;
                for (int sl = 0; sl < RPI; sl++) {
                    const int64_t seg = c * RPI + sl;
                    if (seg < nseg && sbeg[seg] + qr < sbeg[seg + 1]) {
                        if (nl != (uint32_t)sl) return fail(VBC_INVALID_ARG, "masked planar chunk: live lanes not a prefix");
                        nl++;
                    }
                }
                ar.at<uint32_t>(ps.o_nlive)[row] = nl;
            }
            for (int sl = 0; sl < RPI; sl++) {
                const int64_t seg = c * RPI + sl, e = row * RPI + sl;
                const bool real_row = seg < nseg && sbeg[seg] + qr < sbeg[seg + 1];
                const Entry *en = real_row ? &ents[pstart[seg] + qr] : nullptr;
                // padding rows gather x[0] (m >= 1: the bucket has entries), taken as 0
                key[e] = real_row ? (en->key | last) : (kPad | last);
                if (holes && real_row && qr % run == 0) {  // a run's first key: which of its rows are stored
                    uint32_t mk = 0;
                    for (int d = 0; d < run; d++) mk |= (en[d].voff >= 0 ? 1u : 0u) << (kHoleShift + d);
                    key[e] |= mk;
                }
                if (planar) {  // column-group-major chunk row (vbc_planar.h)
                    char *rowp = vv + row * RPI * w * esz;
                    for (int cc = 0; cc < w; cc++) {
                        char *dst = rowp + planar_off(esz, w, sl, cc) * esz;
                        if (real_row && cc < wsrc && en->voff >= 0) std::memcpy(dst, val + (en->voff + cc) * esz, (size_t)esz);
                        else std::memset(dst, 0, (size_t)esz);
                    }
                } else if (real_row) {
                    std::memcpy(vv + e * w * esz, val + en->voff * esz, (size_t)wsrc * esz);
                    if (wsrc < w) std::memset(vv + (e * w + wsrc) * esz, 0, (size_t)(w - wsrc) * esz);
                } else {
                    std::memset(vv + e * w * esz, 0, (size_t)w * esz);
                }
            }
        }
    }
    // compressed keys: measured faster on FE except the fp32 forward product (145 -> 158 us)
    const bool kc_wanted = h->slot_keys16 == 1 ? !(kind == 1 && esz == 4) : h->slot_keys16 == 2;
    // split bins (small matrices, latency-bound): 32-bit keys unless VBC_SPLIT_KC=1 -- a compressed key
    // costs a dependent scalar load (its row's pattern offset) before the key itself
    const bool split_kc = split == 1 || h->split_kc;
    ps.kc_ok = kc_wanted && split_kc && slot_keys_compressible(ps.keys, rows, RPI);
    h->slot_rows_padded += E;
    h->slot_rows_real += real;
    h->slot_rows_padded_last = E;
    return VBC_OK;
}

// Per-lane compacted streams (SlotBin::lanes, vbc_planar.h run_planar_lanes) for a planar B'x bucket in
// natural order with contiguous outputs (out[q] = out[0] + q * w, wsrc == w).  Tiles of S consecutive
// stripes (S a multiple of 4, at most one LDS tile buffer: 512 fp64 / 1024 fp32 3-wide stripes), k
// tiles per range, the ranges ~ the kernel's resident waves; inside a tile the stripes are cut into 64
// contiguous sub-blocks minimising the longest stream (binary search on the step count), and the
// sub-blocks go to the lanes by decreasing length, so the live lanes of every step are a prefix.
// An empty stripe is one zero run with PAD | LAST.  ents[sbeg[q] ..] are stripe q's rows (gather index
// keys), rows in runs of `run`.
// Whether a planar B'x bucket runs the lane-stream layout: VBC_PLANAR_LANES=1 forces it (where
// representable), 0 never; auto: a bucket the masked order would take (natural order pads beyond
// slots_pad) with natural contiguous outputs, few empty stripes, and >= 256 stripes per resident wave
// (sub-blocks of ~4 stripes per lane balance the streams).
static bool want_lanes(const vbc_handle *h, int wps, int w, const std::vector<int64_t> &sbeg,
                       const std::vector<int32_t> &out, int64_t total_entries, bool mask)
{
    if (h->planar_lanes == 0 || !slot_planar(h, 0, w) || wps != w) return false;
    const int64_t nseg = (int64_t)sbeg.size() - 1;
    if (nseg < 64 || nseg >= (int64_t(1) << 31)) return false;
    for (size_t q = 1; q < out.size(); q++)
        if ((int64_t)out[q] != (int64_t)out[0] + (int64_t)q * w) return false;
    int64_t empty = 0;
    for (int64_t q = 0; q < nseg; q++) empty += sbeg[q + 1] == sbeg[q];
    if (h->planar_lanes == 1) return true;
    if (!mask || empty * 100 > nseg) return false;
    const int64_t real = sbeg[nseg] - sbeg[0];
    const double share = (double)h->target_ranges_l * (double)real / (double)std::max<int64_t>(total_entries, 1);
    return (double)nseg >= 256.0 * std::max(1.0, share);
}

static int build_lanes(vbc_handle *h, int w, const std::vector<Entry> &ents, const std::vector<int64_t> &sbeg,
                       const std::vector<int32_t> &out, int run, int64_t total_entries, const char *val, Arena &ar,
                       PendingSlot &ps)
{
    const int esz = h->esz;
    // lane pairs (spmv_pair_lanes): fp64 3-wide stripes in runs of 3 -- one 16-B x gather per lane per run
    const bool pair = h->lanes_pair && esz == 8 && w == 3 && run == 3;
    const int NS = pair ? 32 : 64;  // streams per tile
    const int64_t nseg = (int64_t)sbeg.size() - 1;
    const int64_t real = sbeg[nseg] - sbeg[0];
    std::vector<int32_t> len(nseg);  // runs per stripe (an empty stripe: one zero run)
    for (int64_t q = 0; q < nseg; q++) len[q] = (int32_t)std::max<int64_t>(1, (sbeg[q + 1] - sbeg[q]) / run);
    // (sized for half the resident waves -- round 5: fewer, longer tiles near the LDS cap; FE-3D 12,255 tiles of
    // 272 stripes 218.2 us, 10,163 of 328 213.8 us, profiles/r05zh_lanes_ab.log -- the selection rule above
    // keeps the full count)
    const double share = (double)h->target_ranges_l / std::max(1, h->lanes_rdiv) * (double)real /
                         (double)std::max<int64_t>(total_entries, 1);
    const int64_t nr_target = std::max<int64_t>(1, std::llround(share));
    // one tile per range (a wave) of at most one LDS tile buffer of outputs; S a multiple of 4 stripes,
    // the ranges a whole number of rounds of the target
    const int64_t smax = (kLaneTileBytes / (w * esz)) & ~3;
    const int64_t rounds = std::max<int64_t>(1, (nseg + nr_target * smax - 1) / (nr_target * smax));
    int64_t S = (nseg + rounds * nr_target - 1) / (rounds * nr_target);
    S = std::min<int64_t>(smax, std::max<int64_t>(4, (S + 3) / 4 * 4));
    const int64_t ntiles = (nseg + S - 1) / S, nr = ntiles;
    // per tile: NS contiguous streams (first stripe of each), their lengths in runs, the steps
    std::vector<int32_t> trow{0}, tseg;
    std::vector<int16_t> lseg((size_t)ntiles * 64);
    std::vector<std::vector<int32_t>> parts((size_t)ntiles);  // per tile: stream -> {first, end, runs}
    const int rows_per_step = pair ? 1 : run;  // a pair layout row is a run-row
    int64_t rows = 0;
    for (int64_t t = 0; t < ntiles; t++) {
        const int64_t a = t * S, e = std::min(nseg, a + S);
        tseg.push_back((int32_t)a);
        int64_t lo = 0, hi = 0;
        for (int64_t q = a; q < e; q++) {
            lo = std::max<int64_t>(lo, len[q]);
            hi += len[q];
        }
        auto nparts = [&](int64_t cap) {
            int64_t p = 1, cur = 0;
            for (int64_t q = a; q < e; q++) {
                if (cur + len[q] > cap) { p++; cur = len[q]; }
                else cur += len[q];
            }
            return p;
        };
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if (nparts(mid) <= NS) hi = mid;
            else lo = mid + 1;
        }
        const int64_t T = lo;
        std::vector<std::array<int64_t, 3>> pv;  // {length, first stripe, end}
        int64_t cur = 0, first = a;
        for (int64_t q = a; q < e; q++) {
            if (cur + len[q] > T) { pv.push_back({cur, first, q}); first = q; cur = 0; }
            cur += len[q];
        }
        pv.push_back({cur, first, e});
        std::stable_sort(pv.begin(), pv.end(), [](const std::array<int64_t, 3> &p, const std::array<int64_t, 3> &q) {
            return p[0] > q[0];
        });
        std::vector<int32_t> &pt = parts[t];
        for (int l = 0; l < 64; l++) {
            const bool has = l < NS && l < (int)pv.size();
            lseg[(size_t)t * 64 + l] = (int16_t)(has ? pv[l][1] - a : e - a);
            pt.push_back(has ? (int32_t)pv[l][1] : (int32_t)e);
            pt.push_back(has ? (int32_t)pv[l][2] : (int32_t)e);
            pt.push_back(has ? (int32_t)pv[l][0] : 0);  // the stream's length (runs)
        }
        rows += T * rows_per_step;
        trow.push_back((int32_t)rows);
    }
    tseg.push_back((int32_t)nseg);
    if (rows * 64 >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "lane-stream layout too large");
    const std::vector<int32_t> &rrow = trow;  // one tile per range
    std::vector<int32_t> rchunk(nr + 1);
    for (int64_t r = 0; r <= nr; r++) rchunk[r] = (int32_t)r;
    if (layout_knob("VBC_VERBOSE"))
        fprintf(stderr, "[vbc] lanes bin w %d run %d pair %d stripes %lld ranges %lld x %lld stripes (target %d), rows "
                "%lld (live %.3f)\n", w, run, (int)pair, (long long)nseg, (long long)nr, (long long)S, h->target_ranges_l,
                (long long)rows, (double)real / (double)std::max<int64_t>(1, rows * NS * (run / rows_per_step)));
    ps = PendingSlot{};
    SlotBin &b = ps.b;
    b.kind = 0;
    b.wkey = w;
    b.w = w;
    b.wst = w;
    b.rpi = NS;
    b.nranges = (int32_t)nr;
    b.nseg = (int32_t)nseg;
    b.u = h->slot_u;
    b.diag = h->diag;
    b.xcd = h->xcd_p;
    b.spl = 1;
    b.planar = 1;
    b.run = run;
    b.split = 1;
    b.pair = pair ? 1 : 0;
    b.mask = 1;
    b.lanes = 1;
    b.deep = h->lanes_deep;
    b.ntiles = (int32_t)ntiles;
    b.out_affine = 1;
    b.out_base = out.empty() ? 0 : out[0];
    b.out_stride = w;
    b.contig = 1;
    ps.rows = rows;
    ps.real = real;
    const int64_t vals_per_row = pair ? 288 : (int64_t)64 * w;
    const int64_t keys_per_row = NS;
    ps.o_val = ar.reserve((size_t)rows * vals_per_row * esz);
    ps.o_out = ar.reserve(4);
    ps.o_rrow = ar.reserve(rrow.size() * 4);
    ps.o_rchunk = ar.reserve(rchunk.size() * 4);
    ps.o_nlive = ar.reserve((size_t)rows * 4);
    ps.o_trow = ar.reserve(trow.size() * 4);
    ps.o_tseg = ar.reserve(tseg.size() * 4);
    ps.o_lseg = ar.reserve(lseg.size() * 2);
    ps.o_key = ar.reserve((size_t)rows * keys_per_row * 4);
    ps.key_bytes = (int64_t)(real / run) * 4;  // one key per run is read
    ps.lanes_done = true;
    std::memcpy(ar.at<int32_t>(ps.o_rrow), rrow.data(), rrow.size() * 4);
    std::memcpy(ar.at<int32_t>(ps.o_rchunk), rchunk.data(), rchunk.size() * 4);
    std::memcpy(ar.at<int32_t>(ps.o_trow), trow.data(), trow.size() * 4);
    std::memcpy(ar.at<int32_t>(ps.o_tseg), tseg.data(), tseg.size() * 4);
    std::memcpy(ar.at<int16_t>(ps.o_lseg), lseg.data(), lseg.size() * 2);
    *ar.at<int32_t>(ps.o_out) = b.out_base;
    uint32_t *key = ar.at<uint32_t>(ps.o_key);
    uint32_t *nlv = ar.at<uint32_t>(ps.o_nlive);
    char *vv = ar.at<char>(ps.o_val);
    std::memset(vv, 0, (size_t)rows * vals_per_row * esz);
    std::memset(key, 0, (size_t)rows * keys_per_row * 4);
    for (int64_t t = 0; t < ntiles; t++) {
        const int64_t R0 = trow[t], T = (trow[t + 1] - R0) / rows_per_step;
        for (int64_t st = 0; st < T; st++) {
            uint32_t nl = 0;  // streams are in decreasing length: the live ones are a prefix
            while ((int)nl < NS && parts[t][3 * nl + 2] > st) nl++;
            for (int d = 0; d < rows_per_step; d++) nlv[R0 + st * rows_per_step + d] = nl;
        }
        for (int l = 0; l < NS; l++) {
            int64_t st = 0;
            for (int32_t q = parts[t][3 * l]; q < parts[t][3 * l + 1]; q++) {
                const int64_t nrun = (sbeg[q + 1] - sbeg[q]) / run;
                if (nrun == 0) {  // empty stripe: one zero run, PAD | LAST (writes its zeros)
                    key[(R0 + st * rows_per_step) * keys_per_row + l] = kPad | kLast;
                    st++;
                    continue;
                }
                for (int64_t u = 0; u < nrun; u++, st++) {
                    const int64_t row0 = R0 + st * rows_per_step;
                    key[row0 * keys_per_row + l] = ents[sbeg[q] + u * run].key | (u + 1 == nrun ? kLast : 0u);
                    if (pair) {  // the run's 3 x 3 values in the pair run-row form (run_pair)
                        double v[3][3];
                        for (int d = 0; d < 3; d++)
                            std::memcpy(v[d], val + ents[sbeg[q] + u * 3 + d].voff * esz, 3 * sizeof(double));
                        double *blk = reinterpret_cast<double *>(vv) + row0 * 288;
                        blk[4 * l + 0] = v[0][0];
                        blk[4 * l + 1] = v[0][1];
                        blk[4 * l + 2] = v[0][2];
                        blk[4 * l + 3] = v[1][2];
                        blk[128 + 2 * l + 0] = v[1][0];
                        blk[128 + 2 * l + 1] = v[1][1];
                        blk[192 + l] = v[2][2];
                        blk[224 + 2 * l + 0] = v[2][0];
                        blk[224 + 2 * l + 1] = v[2][1];
                        continue;
                    }
                    for (int d = 0; d < run; d++) {
                        const Entry &en = ents[sbeg[q] + u * run + d];
                        char *rowp = vv + (row0 + d) * 64 * w * esz;
                        for (int cc = 0; cc < w; cc++)
                            std::memcpy(rowp + planar_off(esz, w, l, cc) * esz, val + (en.voff + cc) * esz, (size_t)esz);
                    }
                }
            }
        }
    }
    h->slot_rows_padded += rows * NS * (run / rows_per_step);
    h->slot_rows_real += real;
    h->slot_rows_padded_last = rows * NS * (run / rows_per_step);
    return VBC_OK;
}

// One launch's slotted bins share one key form (the kernel is specialised on it).
static void commit_launch_keys(const vbc_handle *h, std::vector<PendingSlot> &pss, Arena &ar)
{
    bool kc = false;
    for (const PendingSlot &ps : pss) {
        if (ps.lanes_done) continue;  // the lanes layout stores its own keys (its own launch)
        kc = true;
    }
    for (const PendingSlot &ps : pss) kc = kc && (ps.lanes_done || ps.kc_ok);
    for (PendingSlot &ps : pss)
        if (!ps.lanes_done) commit_slot_keys(ps, kc, ar, h->slot_dedup);
}

// ---- row-swept layout (vbc_sweep.hip) ------------------------------------------------------------

struct PendingSweep {
    SweepBin b;
    size_t o_tstep, o_key, o_loc, o_val, o_out, o_sbase;
    double work = 0;  // matrix bytes the bin streams (launch-group ordering)
};

// Whether a bucket lacks x locality: the gathers of windows of 64 consecutive segments (the segments
// one slotted chunk folds together) span most of an x (length nx) too large for L2.  Mesh operators
// span a few bandwidths (FE: ~10^4 rows of 10^7); the costs.jl:63-83 generator spans all of x.
// Segment q's entries are ents[sbeg[q] .. sbeg[q+1]), keys = gather index.
static bool sweep_possible(const vbc_handle *h, int w, int64_t nx)
{
    return h->sweep_mode != 0 && w <= 8 && nx < kSlotIdxLimit && (h->sweep_mode == 1 || (double)nx * h->esz >= 16e6);
}

static bool want_sweep(const vbc_handle *h, int w, int64_t nx, const std::vector<int64_t> &sbeg,
                       const std::vector<Entry> &ents)
{
    const int64_t nseg = (int64_t)sbeg.size() - 1;
    if (h->sweep_mode == 0 || w > 8 || nx >= kSlotIdxLimit || nseg <= 0 || nseg >= (int64_t(1) << 31)) return false;
    if (h->sweep_mode == 1) return true;
    const double xbytes = (double)nx * h->esz;
    if (xbytes < 16e6) return false;  // x stays in L2 / MALL anyway
    std::vector<double> span;
    for (int64_t a = 0; a < nseg; a += 64) {
        int64_t lo = INT64_MAX, hi = -1;
        for (int64_t e = sbeg[a]; e < sbeg[std::min(nseg, a + 64)]; e++) {
            lo = std::min<int64_t>(lo, ents[e].key);
            hi = std::max<int64_t>(hi, ents[e].key);
        }
        if (hi >= 0) span.push_back((double)(hi - lo + 1) * h->esz);
    }
    if (span.empty()) return false;
    std::nth_element(span.begin(), span.begin() + span.size() / 2, span.end());
    return span[span.size() / 2] >= 0.25 * xbytes;
}

// Segments per tile: as many as the wave's LDS tile holds (kind 0: w accumulators per stripe, kind 1:
// one per output row).  Capping narrow buckets so that every tile costs the same measured slower on
// the mixed-width NS workload (379 -> 395 us).
static int sweep_segments(const vbc_handle *h, int kind, int w)
{
    return (int)std::max(1, std::min(65535, h->sweep_tile / ((kind == 0 ? w : 1) * h->esz)));
}

// Lay out a swept bucket: tiles of S segments; each tile's entries in 64-lane steps, taken in
// ascending gather order by a min-heap over the segments' next entries (a segment enters a step at
// most once, and its entries keep their stored order).  out[q] = y offset of segment q.
static int build_sweep(vbc_handle *h, int kind, int w, const std::vector<int64_t> &sbeg,
                       const std::vector<Entry> &ents, const std::vector<int32_t> &out, const char *val, Arena &ar,
                       int &tile0, PendingSweep &pw)
{
    const int esz = h->esz;
    const int64_t nseg = (int64_t)sbeg.size() - 1;
    const int S = sweep_segments(h, kind, w);
    const int64_t ntiles = (nseg + S - 1) / S;
    if (tile0 + ntiles >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "bucket too large");
    std::vector<int32_t> tstep{0};
    std::vector<uint32_t> keys;
    std::vector<uint16_t> locs;
    std::vector<int64_t> voffs;  // value offset of each lane slot, -1 = padding
    keys.reserve(ents.size() + 64 * ntiles);
    locs.reserve(ents.size() + 64 * ntiles);
    voffs.reserve(ents.size() + 64 * ntiles);
    typedef std::pair<uint32_t, int32_t> Head;  // (gather index, segment within tile)
    std::vector<Head> heap, picks;
    std::vector<int64_t> cur(S);
    for (int64_t t = 0; t < ntiles; t++) {
        const int64_t s0 = t * S;
        const int ns = (int)std::min<int64_t>(S, nseg - s0);
        heap.clear();
        for (int q = 0; q < ns; q++) {
            cur[q] = sbeg[s0 + q];
            if (cur[q] < sbeg[s0 + q + 1]) heap.push_back({ents[cur[q]].key, q});
        }
        std::make_heap(heap.begin(), heap.end(), std::greater<Head>());
        while (!heap.empty()) {
            picks.clear();
            while (!heap.empty() && picks.size() < 64) {
                std::pop_heap(heap.begin(), heap.end(), std::greater<Head>());
                picks.push_back(heap.back());
                heap.pop_back();
            }
            for (const Head &p : picks) {
                keys.push_back(p.first);
                locs.push_back((uint16_t)p.second);
                voffs.push_back(ents[cur[p.second]].voff);
            }
            for (size_t k = picks.size(); k < 64; k++) {
                keys.push_back(kPad);
                locs.push_back(0);
                voffs.push_back(-1);
            }
            for (const Head &p : picks)
                if (++cur[p.second] < sbeg[s0 + p.second + 1]) {
                    heap.push_back({ents[cur[p.second]].key, p.second});
                    std::push_heap(heap.begin(), heap.end(), std::greater<Head>());
                }
        }
        if ((int64_t)keys.size() / 64 >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "bucket too large");
        tstep.push_back((int32_t)(keys.size() / 64));
    }
    // Packed keys: a step's 64 entries are consecutive picks of the ascending heap, so their gather
    // indices lie within a narrow window above the first lane's: key = PAD | segment << lbits | delta,
    // one 32-bit load per lane instead of the 32-bit index plus the 16-bit segment (6 -> 4 B per entry
    // and one load instruction less per step), the base read once per step through the scalar cache.
    const int64_t nsteps = (int64_t)keys.size() / 64;
    int sbits = 1;
    while ((1 << sbits) < S) sbits++;
    const int lbits = 31 - sbits;
    bool packed = h->sweep_pack != 0 && lbits >= 8;
    std::vector<uint32_t> sbase;
    if (packed) {
        sbase.resize((size_t)nsteps);
        for (int64_t st = 0; st < nsteps && packed; st++) {
            const uint32_t b0 = keys[st * 64];  // the smallest pick: never padding
            sbase[st] = b0 & kSlotIdx;
            for (int l = 0; l < 64; l++) {
                const uint32_t k = keys[st * 64 + l];
                if (k & kPad) continue;
                if (k < b0 || ((k - b0) >> lbits) != 0) { packed = false; break; }
            }
        }
    }
    if (packed)
        for (int64_t e = 0; e < (int64_t)keys.size(); e++) {
            const uint32_t k = keys[e];
            keys[e] = (k & kPad) ? kPad : ((uint32_t)locs[e] << lbits) | (k - sbase[e / 64]);
        }
    pw = PendingSweep{};
    SweepBin &b = pw.b;
    b.kind = kind;
    b.packed = packed ? 1 : 0;
    b.lbits = packed ? lbits : 0;
    b.w = w;
    b.tile0 = tile0;
    b.ntiles = (int32_t)ntiles;
    b.S = S;
    b.nseg = (int32_t)nseg;
    b.out_affine = 1;
    b.out_base = out.empty() ? 0 : out[0];
    b.out_stride = out.size() > 1 ? out[1] - out[0] : 0;
    for (size_t q = 1; q < out.size() && b.out_affine; q++)
        b.out_affine = (int64_t)out[q] == (int64_t)out[0] + (int64_t)q * b.out_stride;
    tile0 += (int)ntiles;
    const int64_t E = (int64_t)keys.size();
    pw.o_tstep = ar.reserve(tstep.size() * 4);
    pw.o_key = ar.reserve(E * 4);
    pw.o_loc = ar.reserve(packed ? 4 : E * 2);
    pw.o_sbase = ar.reserve(packed ? (size_t)nsteps * 4 : 4);
    pw.o_val = ar.reserve(E * w * esz);
    pw.o_out = ar.reserve(out.size() * 4);
    std::memcpy(ar.at<int32_t>(pw.o_tstep), tstep.data(), tstep.size() * 4);
    std::memcpy(ar.at<uint32_t>(pw.o_key), keys.data(), E * 4);
    if (packed) std::memcpy(ar.at<uint32_t>(pw.o_sbase), sbase.data(), (size_t)nsteps * 4);
    else std::memcpy(ar.at<uint16_t>(pw.o_loc), locs.data(), E * 2);
    std::memcpy(ar.at<int32_t>(pw.o_out), out.data(), out.size() * 4);
    char *vv = ar.at<char>(pw.o_val);
    for (int64_t e = 0; e < E; e++) {
        if (voffs[e] >= 0) std::memcpy(vv + e * w * esz, val + voffs[e] * esz, (size_t)w * esz);
        else std::memset(vv + e * w * esz, 0, (size_t)w * esz);
    }
    (kind == 0 ? h->bytes_t : h->bytes_f) +=
        E * ((packed ? 4 : 6) + (int64_t)w * esz) + (packed ? nsteps * 4 : 0) + (int64_t)tstep.size() * 4 +
        (b.out_affine ? 0 : nseg * 4);
    return VBC_OK;
}

// Stored width of a transposed bucket.  Widths whose rows do not split into 16-B lane vectors
// with a power-of-two slot count (w = 3, 5, 6, 7) run the shuffle-scan path with 4-8-B loads; padding
// them with zero columns buys 16-B loads and the DPP scan for 14-60 % more value bytes.  The padding
// columns multiply x[row] by 0 into outputs that are never written (the forward product, which would
// gather x beyond the stripe, is never padded).  VBC_PAD="w:wp,..." overrides (A/B).
static int padded_width(const vbc_handle *h, int w)
{
    static const int def64[9] = {0, 1, 2, 4, 4, 5, 6, 8, 8};
    static const int def32[9] = {0, 1, 2, 4, 4, 5, 8, 8, 8};
    int wp = w <= 8 ? (h->esz == 8 ? def64[w] : def32[w]) : w;
    if (const char *e = tuning_knob("VBC_PAD")) {
        wp = w;
        for (const char *p = e; *p;) {
            int a = 0, b = 0, n = 0;
            if (sscanf(p, "%d:%d%n", &a, &b, &n) != 2) break;
            if (a == w && b >= w && b <= 64) wp = b;
            p += n;
            if (*p == ',') p++;
        }
    }
    return wp;
}

// Runs with holes (SlotBin::holes) for a bucket of the fused small-matrix split: when the stripes' rows do
// not all come in aligned runs of R consecutive rows (slot_runs) but grouping every stripe's rows by
// row / R adds at most kHoleFill padding rows, each group becomes a whole run of R entries -- the absent
// rows with voff = -1 (zero values; their x is taken as 0 by the kernel, so a non-finite x of a row the
// stripe does not store never reaches it, as in the reference).  One key and one R-wide x gather per
// run instead of one per row.  Fills hents / hsbeg (empty: no runs worth it).
constexpr double kHoleFill = 0.15;
static void hole_runs(const vbc_handle *h, const Stripes &s, const std::vector<int64_t> &stripes, int w,
                      std::vector<Entry> &hents, std::vector<int64_t> &hsbeg)
{
    hents.clear();
    hsbeg.clear();
    if (h->slot_runs == 0 || s.m >= (int64_t)kHoleIdx - 3) return;
    int64_t real = 0;
    for (int64_t l : stripes) real += s.rbeg[l + 1] - s.rbeg[l];
    if (real == 0) return;
    for (int R = 3; R >= 2; R--) {
        int64_t expanded = 0;
        bool exact = true, past = false;
        for (int64_t l : stripes) {
            int64_t prev = -1, groups = 0;
            for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++) {
                const int64_t k = s.rows[r] / R;
                if (k != prev) { groups++; prev = k; }
                // the kernels gather a run's R x values with one unconditional R-wide load: a run whose
                // last row lies past the operand (m % R != 0) would read beyond x's allocation
                past = past || k * R + R > s.m;
            }
            expanded += groups * R;
            exact = exact && groups * R == s.rbeg[l + 1] - s.rbeg[l];
        }
        if (exact) return;  // whole runs already: slot_runs finds them
        if (past || (double)(expanded - real) > kHoleFill * (double)real) continue;
        hsbeg.assign(1, 0);
        hents.reserve(expanded);
        for (int64_t l : stripes) {
            for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1];) {
                const int64_t k = s.rows[r] / R;
                for (int d = 0; d < R; d++) {
                    const int64_t row = k * R + d;
                    if (r < s.rbeg[l + 1] && s.rows[r] == row) {
                        hents.push_back({(uint32_t)row, s.voff[l] + (r - s.rbeg[l]) * s.vstride(l)});
                        r++;
                    } else {
                        hents.push_back({(uint32_t)row, -1});  // a hole of the run
                    }
                }
            }
            hsbeg.push_back((int64_t)hents.size());
        }
        if (layout_knob("VBC_VERBOSE"))
            fprintf(stderr, "[vbc] runs with holes: w %d R %d rows %lld -> %lld\n", w, R, (long long)real,
                    (long long)expanded);
        return;
    }
}

// Long stripes of the fused split cut into ks parts (SlotBin::ks): each stripe's rows split at run
// boundaries into ks parts of equal run counts (the last may be shorter), the stripes by decreasing
// length, 64 / ks of them per chunk, part p of the chunk's stripe i in lane p * (64 / ks) + i; lanes past
// the last stripe hold empty segments.  ents[sbeg[q] ..] are stripe q's rows, out[q] its first column.
static int build_ksplit(vbc_handle *h, int w, int ks, const std::vector<Entry> &ents, const std::vector<int64_t> &sbeg,
                        const std::vector<int32_t> &out, int64_t total, const char *val, Arena &ar, int &range0,
                        PendingSlot &ps)
{
    const int64_t n = (int64_t)sbeg.size() - 1, m = 64 / ks;
    const int R = slot_runs(h, ents, sbeg);
    std::vector<int64_t> sx{0};  // segment bounds in ents order: stripe q's part p is segment q * ks + p
    std::vector<int32_t> ox;
    for (int64_t q = 0; q < n; q++) {
        const int64_t runs = (sbeg[q + 1] - sbeg[q]) / R, per = (runs + ks - 1) / ks;
        for (int p = 0; p < ks; p++) {
            sx.push_back(sbeg[q] + std::min<int64_t>(runs, (p + 1) * per) * R);
            ox.push_back(out[q]);
        }
    }
    const int64_t nchk = (n + m - 1) / m;
    for (int64_t t = n; t < nchk * m; t++)  // empty segments: stripe slots t >= n of the last chunk
        for (int p = 0; p < ks; p++) {
            sx.push_back(sx.back());
            ox.push_back(-1);
        }
    std::vector<int64_t> byl(n);
    for (int64_t q = 0; q < n; q++) byl[q] = q;
    std::stable_sort(byl.begin(), byl.end(),
                     [&](int64_t a, int64_t b) { return sbeg[a + 1] - sbeg[a] > sbeg[b + 1] - sbeg[b]; });
    std::vector<int64_t> order((size_t)(nchk * 64));
    for (int64_t c = 0; c < nchk; c++)
        for (int p = 0; p < ks; p++)
            for (int64_t i = 0; i < m; i++) {
                const int64_t t = c * m + i;
                order[c * 64 + p * m + i] = (t < n ? byl[t] : t) * ks + p;
            }
    if (layout_knob("VBC_VERBOSE"))
        fprintf(stderr, "[vbc] long stripes: w %d, %lld stripes cut into %d parts (runs of %d), %lld chunks\n", w,
                (long long)n, ks, R, (long long)nchk);
    return build_slots(h, 0, w, w, ents, sx, ox, total, val, ar, range0, ps, order, false, ks);
}

// Column pieces (B'x layouts only): when one width wd holds >= 80 % of the stripes, a side stripe whose
// width is a multiple k·wd runs as k wd-wide stripes over the same stored rows (values addressed in
// place through Stripes::vst).  The ldoor stand-in's 'min memory' partition is 317,337 3-wide stripes
// and 32 6-wide ones: as two buckets, the 6-wide one is a single chunk whose wave walks 51 rows of
// dependent loads at the loaded-memory latency of the streaming bucket beside it (42.6 us against the
// strict partition's 33.8 us, profiles/r04_ab11_ldoor32_*.log).  Every output column keeps its
// stripe's rows in stored order, so each column is summed exactly as before (multiply_1DVBC.jl:101-104).
static bool column_pieces(const vbc_handle *h, const Stripes &s, Stripes &c)
{
    if (h->colsplit == 0 || s.L < 1) return false;
    std::map<int, int64_t> cnt;
    for (int64_t l = 0; l < s.L; l++) cnt[s.w[l]]++;
    int wd = 0;
    int64_t nd = 0;
    for (auto &kv : cnt)
        if (kv.second > nd) { nd = kv.second; wd = kv.first; }
    // VBC_COLSPLIT_W=c (A/B): every stripe wider than c as pieces of c columns (+ the remainder)
    const int cw = h->colsplit_w;
    bool any = false;
    if (cw > 0) {
        wd = cw;
        for (auto &kv : cnt) any = any || kv.first > cw;
    } else {
        if (cnt.size() < 2 || (double)nd < 0.8 * (double)s.L) return false;
        for (auto &kv : cnt) any = any || (kv.first > wd && kv.first % wd == 0);
    }
    if (!any) return false;
    c.m = s.m;
    c.n = s.n;
    c.grp = s.grp;
    c.rbeg.assign(1, 0);
    for (int64_t l = 0; l < s.L; l++) {
        const int wl = s.w[l];
        const bool cut = wl > wd && (cw > 0 || wl % wd == 0);
        for (int c0 = 0; c0 < wl; c0 += cut ? wd : wl) {
            const int wp = cut ? std::min(wd, wl - c0) : wl;
            c.col0.push_back(s.col0[l] + c0);
            c.w.push_back(wp);
            c.voff.push_back(s.voff[l] + c0);
            c.vst.push_back((int32_t)s.vstride(l));
            c.rows.insert(c.rows.end(), s.rows.begin() + s.rbeg[l], s.rows.begin() + s.rbeg[l + 1]);
            c.rbeg.push_back((int64_t)c.rows.size());
        }
    }
    c.L = (int64_t)c.w.size();
    if (layout_knob("VBC_VERBOSE"))
        fprintf(stderr, "[vbc] column pieces: %lld stripes -> %lld (dominant width %d)\n", (long long)s.L,
                (long long)c.L, wd);
    return true;
}

// Transposed layout: segments = stripes of each width, entries = their stored rows.  A bucket runs
// slotted (vbc_slots.h, every stripe of the width a segment, empty ones included) when its row counts
// are near-uniform, else merged (non-empty stripes; empty ones go to the fill list).
static int build_transposed(vbc_handle *h, const Stripes &s0, const char *val, Arena &ar,
                            std::vector<PendingBin> &pbs, std::vector<PendingSlot> &pss,
                            std::vector<PendingSweep> &pws, Launch &L, std::vector<int32_t> &fill)
{
    Stripes sp;
    const Stripes &s = column_pieces(h, s0, sp) ? sp : s0;
    std::map<int, std::vector<int64_t>> buckets;  // w -> stripes
    for (int64_t l = 0; l < s.L; l++) buckets[s.w[l]].push_back(l);
    const int64_t total = (int64_t)s.rows.size();
    int range0 = 0, srange0 = 0, tile0 = 0;
    // Small matrices with several width buckets (a SuiteSparse operator's strict stripes: ct20stif's are
    // 1..6 wide; filled / mixed partitions): every bucket planar (any width 1..8, one stripe per lane)
    // and split, P waves per 64-stripe chunk, all buckets in ONE launch (Launch::fuse_split) -- instead
    // of a slotted launch, one launch per planar bucket and the merge kernel for the buckets whose
    // chunks are too long to balance one wave each.  Taken when the chunks of all buckets together fill
    // at most half the wave slots (the split rule of build_slots) and every chunk keeps >= split_rows
    // (fp64) rows per wave; P is common to the launch.  VBC_SMALL_FUSE=0 turns it off.
    h->small_split = 0;
    h->fuse_w = 0;
    // A single-width small matrix runs the fused split when its bucket would otherwise take the merge
    // layout (chunks too long to balance one wave each: the 3dtube stand-in's 'overlap' partition, 15,110
    // 3-wide stripes of ~71 rows, fp64 16.4 -> 7.8 us, fp32 14.2 -> 6.8 us); a bucket the planar layouts
    // take keeps them (ldoor's 1/8 stripe shard: masked planar 12.4 us, fused 14.3 us,
    // profiles/r04_ab13_*.log, r04_ab15_*.log).  VBC_SMALL_FUSE=2 fuses every single-width one.
    // (a bucket headed for the merge layout: no slotted / planar layout balances its chunks)
    auto merge_bound = [&](int w, const std::vector<int64_t> &stripes) {
        if (w > 8 || sweep_possible(h, w, s.m)) return false;
        const int wps = slot_planar(h, 0, w) ? w : (h->esz == 8 && w == 3) ? 3 : padded_width(h, w);
        std::vector<int64_t> sb{0}, order;
        for (int64_t l : stripes) sb.push_back(sb.back() + s.rbeg[l + 1] - s.rbeg[l]);
        bool mask = false;
        return want_slots(h, 0, wps, sb, total, s.m, order, &mask, w) == 0;
    };
    int fuse_min = h->small_fuse >= 2 ? 1 : 2;
    if (fuse_min == 2 && h->small_fuse == 1 && buckets.size() == 1 && merge_bound(buckets.begin()->first, buckets.begin()->second))
        fuse_min = 1;
    // Long stripes (SlotBin::ks): a chunk runs on one CU and costs its longest stripe's rows, so a few
    // chunks of long stripes (a 'min blocks' partition's widest, fullest stripes: 3.4x the mean chunk on
    // the ct20stif stand-in) set the product's time.  A stripe whose work (rows x width, values per
    // lane) exceeds ksplit x the mean chunk's is cut into 2 (4 above twice that) parts of whole runs,
    // laid side by side in the lanes of one chunk and summed across them before the store.
    std::vector<uint8_t> kst;  // per stripe: parts (empty: none cut)
    // (auto layouts only: a forced VBC_SLOTS / VBC_SLOT_PLANAR keeps the layout the tests ask for)
    if (h->planar_split != 0 && h->small_fuse != 0 && h->slot_planar < 0 && h->slots_mode < 0 && (int)buckets.size() >= fuse_min &&
        (int)buckets.size() <= kSplitParts && buckets.rbegin()->first <= 8 && !sweep_possible(h, 1, s.m)) {
        // the fused buckets: all of them; or, when their chunks would overflow the launch and one bucket
        // holds most of them, every bucket but that one (a large operator's dominant width keeps its
        // streaming layout, and its small side buckets -- a time-model partition's few 1-, 4- and 5-wide
        // stripes beside 305,000 3-wide ones -- run as one fused launch instead of one launch each)
        const double slots0 = (double)h->target_ranges_p;
        int64_t nall = 0, nmax = 0;
        int wmax = 0;
        for (auto &kv : buckets) {
            const int64_t c = ((int64_t)kv.second.size() + 63) / 64;
            nall += c;
            if (c > nmax) { nmax = c; wmax = kv.first; }
        }
        for (auto &kv : buckets) h->fuse_w |= 1u << kv.first;
        // a dominant bucket headed for the merge layout is better fused too, up to one chunk per wave slot
        // (the ldoor stand-in's fp64 'min blocks', 2,358 chunks of 6-wide stripes of 69 rows: merge kernel
        // 131.5 us + the fused side launch 11.5 us; all fused 131.5 us, profiles/r04_ab17_ldoor64_blocks.log)
        const bool dom_merge = h->side_fuse < 0 && (double)nmax >= 0.8 * (double)nall && (double)nall <= slots0 &&
                               merge_bound(wmax, buckets[wmax]);
        const bool side = h->side_fuse < 0 ? (double)nall * 2 > slots0 && buckets.size() >= 3 && (double)nmax >= 0.8 * (double)nall && !dom_merge
                                           : h->side_fuse == 1 && (double)nmax >= 0.8 * (double)nall;
        if (side) h->fuse_w &= ~(1u << wmax);
        auto fused_w = [&](int w) { return ((h->fuse_w >> w) & 1) != 0; };
        if (h->ksplit > 0) {
            double work = 0;
            int64_t nw = 0;
            for (auto &kv : buckets) {  // chunks of the length-sorted buckets
                if (!fused_w(kv.first)) continue;
                std::vector<int64_t> len;
                for (int64_t l : kv.second) len.push_back(s.rbeg[l + 1] - s.rbeg[l]);
                std::sort(len.begin(), len.end(), std::greater<int64_t>());
                for (size_t i = 0; i < len.size(); i += 64, nw++) work += (double)len[i] * kv.first;
            }
            // never below a CU's share of the whole: with many chunks per CU (the ldoor stand-in's 'min
            // blocks', 2550 chunks) a long chunk is averaged out, and cutting only adds chunks (70 -> 107 us)
            const double thr = std::max(h->ksplit * work / (double)std::max<int64_t>(nw, 1), work / (double)h->cus);
            kst.assign(s.L, 1);
            int parts = 0, cut = 0;
            for (auto &kv : buckets) {
                if (!fused_w(kv.first)) continue;
                int cls = 0;
                for (int64_t l : kv.second) {
                    const double wk = (double)(s.rbeg[l + 1] - s.rbeg[l]) * kv.first;
                    kst[l] = wk > 2 * thr ? 4 : wk > thr ? 2 : 1;
                    cls |= kst[l];
                }
                parts += __builtin_popcount(cls);
                cut += cls > 1;
            }
            if (parts > kSplitParts || cut == 0 || !(thr > 0)) kst.clear();
        }
        int64_t nch = 0, rows = 0;
        int nf = 0;
        for (auto &kv : buckets) {
            if (!fused_w(kv.first)) continue;
            nf++;
            int64_t cnt[5] = {0, 0, 0, 0, 0};
            for (int64_t l : kv.second) {
                cnt[kst.empty() ? 1 : kst[l]]++;
                rows += s.rbeg[l + 1] - s.rbeg[l];
            }
            for (int k = 1; k <= 4; k *= 2) nch += (cnt[k] * k + 63) / 64;
        }
        const double slots = (double)h->target_ranges_p;
        const double avg = (double)rows / (double)std::max<int64_t>(nch, 1) / 64.0 * 1.1;  // rows per chunk (sorted)
        // (the batched slice loop costs a round trip per batch, not per step: thinner slices than the
        // single-bucket rule's split_rows pay off -- ct20stif 'min blocks' P = 4 / 8: 15.7 / 14.7 us)
        const double minrows = (double)h->small_rows * h->esz / 8.0;
        if ((double)nch * (dom_merge ? 1 : 2) <= slots && nf >= fuse_min) {
            int P = 1;
            while (P < h->fuse_pmax && (double)nch * P * 2 <= 2 * slots && avg / (P * 2) >= minrows) P *= 2;
            // fusing pays even when the chunks are too short to split: one launch instead of one per
            // bucket (the thermal1 stand-in's 'min blocks', 8 buckets of 16-row chunks: 41 us unfused)
            P = std::max(P, 2);
            // many chunks (more waves than one round of the chip): P that fills whole rounds of resident
            // waves -- the ldoor stand-in's 'min blocks', 2550 chunks: P = 2 / 4 / 8 give 1.25 / 2.5 / 5.0
            // rounds of 4096 fp32 waves (70.9 / 70.1 / 66.0 us, profiles/r04_ab7_ldoor32_blocks.log)
            auto rounds = [&](int p) {
                const double cap = (double)h->cus * std::max(1, h->occ_multi[p == 2 ? 1 : p == 4 ? 2 : 3]);
                return (double)nch * p / cap;
            };
            if (rounds(P) > 1.0) {
                auto eff = [&](int p) { const double r = rounds(p); return r / std::ceil(r); };
                for (int p = 2; p <= h->fuse_pmax; p *= 2)
                    if (eff(p) > eff(P) + 0.05) P = p;
            }
            if (h->planar_split > 1) P = h->planar_split;
            if (P > 1) h->small_split = P;
        }
        if (h->small_split <= 1) {
            kst.clear();
            h->fuse_w = 0;
        }
        if (layout_knob("VBC_VERBOSE"))
            fprintf(stderr, "[vbc] small fused split: %d of %d buckets (width mask 0x%x), %lld chunks, %.1f rows per "
                    "chunk -> P = %d%s\n", nf, (int)buckets.size(), h->fuse_w, (long long)nch, avg, h->small_split,
                    kst.empty() ? "" : ", long stripes cut");
    }
    // the bins: a width bucket, or (long stripes cut) its stripes of each part count ks
    std::vector<std::pair<int, std::vector<int64_t>>> subs;
    std::vector<int> subk;
    for (auto &kv : buckets) {
        if (kst.empty()) {
            subs.emplace_back(kv.first, std::move(kv.second));
            subk.push_back(1);
            continue;
        }
        for (int k = 1; k <= 4; k *= 2) {
            std::vector<int64_t> v;
            for (int64_t l : kv.second)
                if (kst[l] == k) v.push_back(l);
            if (v.empty()) continue;
            subs.emplace_back(kv.first, std::move(v));
            subk.push_back(k);
        }
    }
    for (size_t si = 0; si < subs.size(); si++) {
        const auto &kv = subs[si];
        const int ks = subk[si];
        const int w = kv.first;
        if (sweep_possible(h, w, s.m)) {
            std::vector<int64_t> sb{0};
            std::vector<Entry> ents;
            std::vector<int32_t> out;
            ents.reserve(s.rbeg[s.L] - s.rbeg[0]);
            for (int64_t l : kv.second) {
                sb.push_back(sb.back() + s.rbeg[l + 1] - s.rbeg[l]);
                out.push_back((int32_t)s.col0[l]);
                for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++)
                    ents.push_back({(uint32_t)s.rows[r], s.voff[l] + (r - s.rbeg[l]) * s.vstride(l)});
            }
            if (want_sweep(h, w, s.m, sb, ents)) {
                PendingSweep pw;
                if (int st = build_sweep(h, 0, w, sb, ents, out, val, ar, tile0, pw)) return st;
                pw.work = (double)ents.size() * (4.0 + (double)w * h->esz);
                pws.push_back(pw);
                continue;
            }
        }
        const int wp = padded_width(h, w);
        // the slotted kernel has no scan to feed: fp64 w = 3 runs unpadded (8-B lanes), measured
        // 117 -> 106 us on the ldoor stand-in (fp32 keeps 3 -> 4: 73 vs 84 us unpadded)
        const int wps = slot_planar(h, 0, w) ? w : (h->esz == 8 && w == 3 && !tuning_knob("VBC_PAD")) ? 3 : wp;
        std::vector<int64_t> sbeg{0}, order;
        for (int64_t l : kv.second) sbeg.push_back(sbeg.back() + s.rbeg[l + 1] - s.rbeg[l]);
        bool mask = false;
        // fused small split: rows that ALMOST come in aligned runs (a stiffness operator's dof rows, some
        // stripes missing one of a node's rows -- the structural zeros of ct20stif-like matrices) are
        // padded to whole runs, the absent rows marked in the run's key (hole_runs)
        // Only a bucket of the fused launch takes them: its bins run the split product (build_slots gives a
        // fused bucket split = small_split), the one kernel family that folds absent rows (voff < 0); a
        // side bucket, a lane-stream or an unfused slotted / pair layout keeps the plain rows.
        std::vector<Entry> hents;
        std::vector<int64_t> hsbeg;
        const bool fused_bucket = h->small_split > 1 && w <= 8 && ((h->fuse_w >> w) & 1) != 0;
        if (fused_bucket && slot_planar(h, 0, w)) hole_runs(h, s, kv.second, w, hents, hsbeg);
        if (!hsbeg.empty()) {
            std::vector<int32_t> out0;
            for (int64_t l : kv.second) out0.push_back((int32_t)s.col0[l]);
            std::vector<int64_t> order0;
            bool mask0 = false;
            if (want_slots(h, 0, wps, sbeg, total, s.m, order0, &mask0, w) && want_lanes(h, wps, w, sbeg, out0, total, mask0)) {
                hents.clear();
                hsbeg.clear();
            }
        }
        const std::vector<int64_t> &sb = hsbeg.empty() ? sbeg : hsbeg;
        if (ks > 1) {  // long stripes of the fused split, cut into ks lane parts
            std::vector<Entry> ents;
            std::vector<int32_t> out;
            for (int64_t l : kv.second) out.push_back((int32_t)s.col0[l]);
            if (!hsbeg.empty()) {
                ents.swap(hents);
                sbeg.swap(hsbeg);
            } else {
                for (int64_t l : kv.second)
                    for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++)
                        ents.push_back({(uint32_t)s.rows[r], s.voff[l] + (r - s.rbeg[l]) * s.vstride(l)});
            }
            PendingSlot ps;
            if (int st = build_ksplit(h, w, ks, ents, sbeg, out, total, val, ar, srange0, ps)) return st;
            pss.push_back(std::move(ps));
            continue;
        }
        if (want_slots(h, 0, wps, sb, hsbeg.empty() ? total : total + (hsbeg.back() - sbeg.back()), s.m, order, &mask, w)) {
            std::vector<Entry> ents;
            std::vector<int32_t> out;
            for (int64_t l : kv.second) out.push_back((int32_t)s.col0[l]);
            const bool holes = !hsbeg.empty();
            if (holes) {
                ents.swap(hents);
                sbeg.swap(hsbeg);
            } else {
                ents.reserve(sbeg.back());
                for (int64_t l : kv.second)
                    for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++)
                        ents.push_back({(uint32_t)s.rows[r], s.voff[l] + (r - s.rbeg[l]) * s.vstride(l)});
            }
            PendingSlot ps;
            if (!holes && want_lanes(h, wps, w, sbeg, out, total, mask)) {
                if (int st = build_lanes(h, w, ents, sbeg, out, slot_runs(h, ents, sbeg), total, val, ar, ps)) return st;
            } else if (int st = build_slots(h, 0, wps, w, ents, sbeg, out, total, val, ar, srange0, ps, order, mask)) {
                return st;
            }
            pss.push_back(std::move(ps));
            continue;
        }
        std::vector<Entry> ents;
        std::vector<int32_t> out;
        for (int64_t l : kv.second) {
            if (s.rbeg[l + 1] == s.rbeg[l]) {
                for (int c = 0; c < s.w[l]; c++) fill.push_back((int32_t)(s.col0[l] + c));
                continue;
            }
            out.push_back((int32_t)s.col0[l]);
            for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++)
                ents.push_back({(uint32_t)s.rows[r] | (r == s.rbeg[l] ? kHead : 0u),
                                s.voff[l] + (r - s.rbeg[l]) * s.vstride(l)});
        }
        if (ents.empty()) continue;
        PendingBin pb;
        if (int st = build_bucket(h, 0, wp, ents, out, total, val, ar, range0, pb, w)) return st;
        h->bytes_t += (int64_t)ents.size() * (4 + (int64_t)wp * h->esz) + (int64_t)out.size() * 4;
        pb.work = (double)ents.size() * (4.0 + (double)wp * h->esz);
        pbs.push_back(pb);
    }
    commit_launch_keys(h, pss, ar);
    for (const PendingSlot &ps : pss) {  // slotted bins: padded rows x (index bytes + values)
        if (ps.b.lanes) {  // lanes: real rows' values, one key per run, nlive per row, the tile tables
            h->bytes_t += ps.real * (int64_t)ps.b.w * h->esz + ps.key_bytes + ps.rows * 4 + (int64_t)ps.b.ntiles * (8 + 128);
        } else if (ps.b.mask) {  // masked: padding lanes fetch nothing; + the per-row live counts
            const double f = (double)ps.real / (double)std::max<int64_t>(1, ps.rows * ps.b.rpi);
            h->bytes_t += ps.real * (int64_t)ps.b.w * h->esz + (int64_t)(f * (double)ps.key_bytes) + ps.rows * 4;
        } else {
            h->bytes_t += ps.rows * ps.b.rpi * (int64_t)ps.b.w * h->esz + ps.key_bytes;
        }
    }
    L.total_ranges = range0;
    L.slot_ranges = srange0;
    L.sweep_tiles = tile0;
    L.fuse_p = h->small_split;  // (the handle's field is rebuilt by the next build_transposed call)
    L.sweep_tile_bytes = h->sweep_tile;
    if (const char *e = ablation_knob("VBC_SWEEP_DIAG")) L.sweep_diag = atoi(e);
    h->bytes_t += (s.m + s.n) * h->esz;  // x read once, y written once
    return VBC_OK;
}

// Forward row runs (the forward counterpart of slot_runs): the largest R in {3, 2} such that the
// output rows come in aligned runs of R (rows R*q .. R*q+R-1, m divisible by R) with identical stripe
// lists -- the dof rows of a node in a stiffness operator.  sbeg: every row a segment (natural order).
static int fwd_runs(const vbc_handle *h, int w, int64_t m, const std::vector<Entry> &ents,
                    const std::vector<int64_t> &sbeg)
{
    if (h->slot_runs == 0 || h->slot_planar == 0 || w < 2 || w > 4 || m <= 0) return 1;
    for (int R = 3; R >= 2; R--) {
        if (m % R || R * w > 12) continue;
        bool ok = true;
        for (int64_t q = 0; q < m && ok; q += R) {
            const int64_t b0 = sbeg[q], len = sbeg[q + 1] - b0;
            for (int r = 1; r < R && ok; r++) {
                const int64_t br = sbeg[q + r];
                if (sbeg[q + r + 1] - br != len) { ok = false; break; }
                for (int64_t k = 0; k < len; k++)
                    if ((ents[br + k].key & kSlotIdx) != (ents[b0 + k].key & kSlotIdx)) { ok = false; break; }
            }
        }
        if (ok) return R;
    }
    return 1;
}

// Planar forward bin (vbc_planar.h run_planar_fwd): segment q = output rows R*q .. R*q+R-1, one per
// lane, 64 per chunk; chunk row k = the k-th block (stripe) of each segment, its R x w values stored
// column-group-major over the chunk (planar_off with width R*w, element r*w + c); one key per block =
// the stripe's first column (the gathered x slice).  Natural order: y offsets affine (R*q).
// Returns false (and builds nothing) when the padded rows exceed slots_pad x the real ones.
static bool build_fwd_runs(vbc_handle *h, int w, int R, const std::vector<Entry> &ents, const std::vector<int64_t> &sbeg,
                           int64_t m, const char *val, Arena &ar, int &range0, PendingSlot &ps)
{
    const int esz = h->esz, RPI = 64, WV = R * w;
    const int64_t nseg = m / R;
    const int64_t nch = (nseg + RPI - 1) / RPI;
    // run-segment lengths; natural order first, else sorted by length in windows of kSortWindow chunks
    // (y offsets from a table then)
    std::vector<int64_t> rb(nseg + 1, 0), order;
    for (int64_t q = 0; q < nseg; q++) rb[q + 1] = rb[q] + sbeg[R * q + 1] - sbeg[R * q];
    const int64_t real = rb[nseg];
    std::vector<int32_t> cr = chunk_rows(rb, RPI);
    int64_t rows = 0;
    for (int32_t c : cr) rows += c;
    if (real == 0) return false;
    bool mask = false;
    // few chunks: natural order for the split product below, unless it pads by more than half
    const bool few = h->planar_split != 0 && (double)nch * 2 <= (double)h->target_ranges_p &&
                     (double)(rows * RPI) <= 1.5 * (double)real;
    if (!few && (double)(rows * RPI) > h->slots_pad * (double)real) {
        if (h->slots_sort == 0) return false;
        if (h->planar_mask != 0) {  // masked chunk-local length order (SlotBin::mask, as the B'x planar bins)
            order = chunk_sorted_order(rb, RPI * h->mask_window);
            cr = chunk_rows(permuted_sbeg(rb, order), RPI);
            rows = 0;
            for (int32_t c : cr) rows += c;
            mask = (double)(rows * RPI) <= kMaskPad * (double)real;
        }
        if (!mask) {
            order = sorted_order(rb, RPI);
            cr = chunk_rows(permuted_sbeg(rb, order), RPI);
            rows = 0;
            for (int32_t c : cr) rows += c;
            if ((double)(rows * RPI) > h->slots_pad * (double)real) return false;
        }
    }
    auto seg_of = [&](int64_t p) { return order.empty() ? p : order[p]; };  // layout position -> run-segment
    // few chunks (natural order): P waves per chunk (spmv_planar_fwd_split), the rule of the B'x split
    // product with its rows counted in values (>= 36 fp64 / 18 fp32 values per lane per wave: 4 blocks
    // of a 3 x 3 node block in fp64)
    int split = 1;
    if (h->planar_split != 0 && order.empty()) {
        const double share = (double)h->target_ranges_p;
        if (h->planar_split > 1) split = h->planar_split;
        else if ((double)nch * 2 <= share) {
            const double avg = (double)rows / (double)std::max<int64_t>(nch, 1);
            const double minrows = std::max(1.0, (double)h->split_rows * 3.0 * esz / 8.0 / WV);
            while (split < 8 && (double)nch * split * 2 <= 2 * share && avg / (split * 2) >= minrows) split *= 2;
        }
    }
    // ranges of >= fwd_min_rows chunk rows: the kernel's two-stage pipeline loads up to 3U rows past a
    // short range's end (clamped duplicates); ldoor's 1/8 stripe shard (4.8 rows per range at 3072
    // ranges) ran 30.8 us, 16.0 us as 1024 ranges (profiles/r03_fwdshard2.log)
    // (the B'x rule of at most planar_wps waves per SIMD does not carry over: ldoor fp32 B·x 34.3 ->
    // 37.9 us with it, profiles/r03_wps_fwd_*.log)
    const int64_t nr = split > 1 ? nch
                                 : std::max<int64_t>(1, std::min<int64_t>({(int64_t)h->target_ranges_p, nch,
                                                                           rows / std::max(1, h->fwd_min_rows)}));
    std::vector<int32_t> rrow{0}, rchunk{0};
    int64_t acc = 0;
    for (int64_t c = 0; c < nch; c++) {
        acc += cr[c];
        if (c + 1 < nch && (split > 1 || ((int64_t)rrow.size() < nr && acc * nr >= (int64_t)rrow.size() * rows))) {
            rrow.push_back((int32_t)acc);
            rchunk.push_back((int32_t)(c + 1));
        }
    }
    rrow.push_back((int32_t)rows);
    if (layout_knob("VBC_VERBOSE"))
        fprintf(stderr, "[vbc] forward runs bin w %d R %d segments %lld chunks %lld rows %lld (real %lld) mask %d sorted %d "
                "split %d ranges %zu\n", w, R, (long long)nseg, (long long)nch, (long long)rows, (long long)real, (int)mask,
                (int)(!order.empty() && !mask), split, rchunk.size());
    ps = PendingSlot{};
    SlotBin &b = ps.b;
    b.kind = 1;
    b.wkey = w;
    b.w = w;
    b.wst = w;
    b.rpi = RPI;
    b.range0 = 0;  // its own launch
    b.nranges = (int32_t)rchunk.size();
    b.nseg = (int32_t)nseg;
    b.u = h->slot_u;
    b.diag = h->diag;
    b.xcd = split > 1 ? 0 : h->xcd_p;
    b.spl = 1;
    b.planar = 1;
    b.run = R;
    b.split = split;
    b.pair = 0;
    b.mask = mask ? 1 : 0;
    b.out_affine = order.empty() ? 1 : 0;
    b.out_base = 0;
    b.out_stride = R;
    b.contig = b.out_affine;
    const int64_t E = rows * RPI;
    ps.rows = rows;
    ps.real = real;
    if (mask) ps.o_nlive = ar.reserve((size_t)rows * 4);
    ps.keys.resize(E);
    ps.o_val = ar.reserve(E * WV * esz);
    ps.o_out = ar.reserve(std::max<int64_t>(order.size(), 1) * 4);
    for (size_t p = 0; p < order.size(); p++) ar.at<int32_t>(ps.o_out)[p] = (int32_t)(R * order[p]);
    ps.o_rrow = ar.reserve(rrow.size() * 4);
    ps.o_rchunk = ar.reserve(rchunk.size() * 4);
    std::memcpy(ar.at<int32_t>(ps.o_rrow), rrow.data(), rrow.size() * 4);
    std::memcpy(ar.at<int32_t>(ps.o_rchunk), rchunk.data(), rchunk.size() * 4);
    char *vv = ar.at<char>(ps.o_val);
    int64_t row = 0;
    for (int64_t c = 0; c < nch; c++) {
        for (int32_t k = 0; k < cr[c]; k++, row++) {
            const uint32_t last = k + 1 == cr[c] ? kLast : 0u;
            char *rowp = vv + row * RPI * WV * esz;
            if (mask) {  // live lanes of this chunk row: a prefix in chunk-local length order
                uint32_t nl = 0;
                for (int sl = 0; sl < RPI; sl++) {
                    const int64_t p = c * RPI + sl;
                    if (p < nseg && sbeg[R * seg_of(p)] + k < sbeg[R * seg_of(p) + 1]) {
                        if (nl != (uint32_t)sl) return false;
                        nl++;
                    }
                }
                ar.at<uint32_t>(ps.o_nlive)[row] = nl;
            }
            for (int sl = 0; sl < RPI; sl++) {
                const int64_t p = c * RPI + sl, e = row * RPI + sl;
                const int64_t q = p < nseg ? seg_of(p) : 0;
                const bool real_blk = p < nseg && sbeg[R * q] + k < sbeg[R * q + 1];
                ps.keys[e] = real_blk ? ((ents[sbeg[R * q] + k].key & kSlotIdx) | last) : (kPad | last);
                for (int r = 0; r < R; r++)
                    for (int cc = 0; cc < w; cc++) {
                        char *dst = rowp + planar_off(esz, WV, sl, r * w + cc) * esz;
                        if (real_blk) std::memcpy(dst, val + (ents[sbeg[R * q + r] + k].voff + cc) * esz, (size_t)esz);
                        else std::memset(dst, 0, (size_t)esz);
                    }
            }
        }
    }
    ps.kc_ok = h->slot_keys16 != 0 && (split == 1 || h->split_kc) && slot_keys_compressible(ps.keys, rows, RPI);
    h->slot_rows_padded += E;
    h->slot_rows_real += real;
    (void)range0;
    return true;
}

// Forward lane streams (VBC_PLANAR_LANES as for B'x): the B'x lane-stream kernel (run_planar_lanes) with
// a node block's rows and columns exchanged.  Segment q = output rows R*q .. R*q+R-1 (the kernel's W = R
// outputs per stripe slot); the k-th block of the segment (stripe j, w columns) is one "run" of w
// consecutive x rows (the kernel's RUN = w, one w-wide gather) whose d-th row holds A[R*q + 0..R-1][j + d],
// so the kernel folds acc[r] += A[R*q + r][j + d] * x[j + d] for d = 0..w-1, blocks in stripe order.
// Chosen where the forward run layout would need the masked order (natural chunks pad beyond
// slots_pad), with few empty segments and >= 256 segments per resident wave -- FE-3D.
static bool want_fwd_lanes(const vbc_handle *h, int w, int R, int64_t m, const std::vector<int64_t> &sbeg)
{
    if (h->planar_lanes == 0 || w < 1 || w > 3 || !slot_planar(h, 0, R) || m % R) return false;
    const int64_t nseg = m / R;
    if (nseg < 64 || nseg >= (int64_t(1) << 31)) return false;
    if (h->planar_lanes == 1) return true;
    std::vector<int64_t> rb(nseg + 1, 0);
    int64_t empty = 0;
    for (int64_t q = 0; q < nseg; q++) {
        rb[q + 1] = rb[q] + sbeg[R * q + 1] - sbeg[R * q];
        empty += sbeg[R * q + 1] == sbeg[R * q];
    }
    int64_t rows = 0;
    for (int32_t c : chunk_rows(rb, 64)) rows += c;
    if ((double)(rows * 64) <= h->slots_pad * (double)rb[nseg] || empty * 100 > nseg) return false;
    return (double)nseg >= 256.0 * std::max(1, h->target_ranges_l);
}

static int build_fwd_lanes(vbc_handle *h, int w, int R, const std::vector<Entry> &ents, const std::vector<int64_t> &sbeg,
                           int64_t m, const char *val, Arena &ar, PendingSlot &ps)
{
    const int esz = h->esz;
    const int64_t nseg = m / R;
    std::vector<int64_t> sb(nseg + 1, 0);
    for (int64_t q = 0; q < nseg; q++) sb[q + 1] = sb[q] + (sbeg[R * q + 1] - sbeg[R * q]) * w;
    std::vector<Entry> e2((size_t)sb[nseg]);
    std::vector<char> tv((size_t)sb[nseg] * R * esz);  // the blocks transposed: [block][d][r]
    for (int64_t q = 0; q < nseg; q++) {
        const int64_t nb = sbeg[R * q + 1] - sbeg[R * q];
        for (int64_t k = 0; k < nb; k++) {
            const uint32_t col = ents[sbeg[R * q] + k].key & kSlotIdx;
            for (int d = 0; d < w; d++) {
                const int64_t i = sb[q] + k * w + d;
                e2[i] = {col + (uint32_t)d, i * R};
                for (int r = 0; r < R; r++)
                    std::memcpy(tv.data() + (i * R + r) * esz, val + (ents[sbeg[R * q + r] + k].voff + d) * esz, (size_t)esz);
            }
        }
    }
    std::vector<int32_t> out(nseg);
    for (int64_t q = 0; q < nseg; q++) out[q] = (int32_t)(R * q);
    return build_lanes(h, R, e2, sb, out, w, sb[nseg], tv.data(), ar, ps);
}

// Forward lane pairs (round 6): fp64 3 x 3 node blocks (w = 3 stripes, output rows in runs of R = 3) in the
// lane-pair layout of the B'x product (run_pair) with every block TRANSPOSED -- a "stripe" of that layout is
// an output node run q (rows 3q .. 3q+2), its runs the node's blocks in stripe order, a run's 3 "rows" the
// block's columns d gathering x[j + d] -- folded in DOT mode (SlotBin::dot: each output row's dot product with
// the block's x slice added per block, the reference's forward association, multiply_1DVBC.jl:34, :62-71).
// The forward row-run layout (build_fwd_runs) gathers a 24-B x slice per lane per block in two requests; the
// lane pair shares one 16-B gather per lane (ldoor stand-in fp64: its B'x in this layout runs 0.81 of the
// HBM roofline, the forward row runs 0.69).  Returns kBuildDeclined (nothing built) when the bucket would not
// take the pair layout (too few blocks per node, or a small matrix that takes the split product).
static int build_fwd_pair(vbc_handle *h, int w, int R, const std::vector<Entry> &ents, const std::vector<int64_t> &sbeg,
                          int64_t m, int64_t n, const char *val, Arena &ar, PendingSlot &ps)
{
    if (h->esz != 8 || w != 3 || R != 3 || h->planar_pair == 0 || h->slot_planar == 0 || h->slot_runs == 0 || m % R)
        return kBuildDeclined;
    const int esz = h->esz;
    const int64_t nseg = m / R;
    std::vector<int64_t> sb(nseg + 1, 0);
    for (int64_t q = 0; q < nseg; q++) sb[q + 1] = sb[q] + (sbeg[R * q + 1] - sbeg[R * q]) * w;
    if (sb[nseg] == 0 || sb[nseg] >= (int64_t(1) << 31)) return kBuildDeclined;
    std::vector<Entry> e2((size_t)sb[nseg]);
    std::vector<char> tv((size_t)sb[nseg] * R * esz);  // the blocks transposed: [block][d][r]
    for (int64_t q = 0; q < nseg; q++) {
        const int64_t nb = sbeg[R * q + 1] - sbeg[R * q];
        for (int64_t k = 0; k < nb; k++) {
            const uint32_t col = ents[sbeg[R * q] + k].key & kSlotIdx;
            for (int d = 0; d < w; d++) {
                const int64_t i = sb[q] + k * w + d;
                e2[i] = {col + (uint32_t)d, i * R};
                for (int r = 0; r < R; r++)
                    std::memcpy(tv.data() + (i * R + r) * esz, val + (ents[sbeg[R * q + r] + k].voff + d) * esz, (size_t)esz);
            }
        }
    }
    std::vector<int32_t> out(nseg);
    for (int64_t q = 0; q < nseg; q++) out[q] = (int32_t)(R * q);
    std::vector<int64_t> order;
    bool mask = false;
    if (!want_slots(h, 0, w, sb, sb[nseg], n, order, &mask, w)) return kBuildDeclined;
    int zero = 0;
    const int st = build_slots(h, 0, w, w, e2, sb, out, sb[nseg], tv.data(), ar, zero, ps, order, mask, 1, true);
    if (st == VBC_OK) ps.b.dot = 1;
    return st;
}

// Forward layout: per width bucket, segments = output rows with entries of that width (ascending),
// entries = (row, stripe) blocks ordered by stripe within the row.  With a single bucket, a slotted
// layout takes every row as a segment (affine, no fill list).
// Whether the forward product is built as the transposed product of C = Bᵀ (transpose_stripes): stripes
// of two or more widths (the forward layouts would need a scale pass plus one launch per width, each
// adding into y), at most 2^23 stored rows, float eltypes, not VBC_CREATE_SERIAL (C sums each output over
// B's columns in ascending order, not stripe by stripe), VBC_FWD_T != 0.
static bool fwd_via_t_wanted(const vbc_handle *h, const Stripes &s, unsigned flags)
{
    if (h->fwd_t == 0 || (flags & VBC_CREATE_SERIAL) || h->dtype == VBC_I64) return false;
    // a forced layout family (VBC_SLOTS / VBC_SWEEP / VBC_SLOT_PLANAR) keeps the forward layouts the tests ask for
    if (h->fwd_t != 2 && (h->slots_mode >= 0 || h->sweep_mode >= 0 || h->slot_planar >= 0)) return false;
    if ((int64_t)s.rows.size() > (int64_t(1) << 23)) return false;
    int w0 = -1;
    bool mixed = false;
    for (int64_t l = 0; l < s.L && !mixed; l++) {
        if (s.rbeg[l + 1] == s.rbeg[l]) continue;
        if (w0 < 0) w0 = s.w[l];
        mixed = s.w[l] != w0;
    }
    return mixed || h->fwd_t == 2;
}

static int build_forward(vbc_handle *h, const Stripes &s, const char *val, Arena &ar,
                         std::vector<std::vector<PendingBin>> &pbs, std::vector<std::vector<PendingSlot>> &pss,
                         std::vector<std::vector<PendingSweep>> &pws, std::vector<Launch> &Ls,
                         std::vector<int32_t> &fill)
{
    std::map<int, std::vector<int64_t>> buckets;  // w -> stripes
    for (int64_t l = 0; l < s.L; l++)
        if (s.rbeg[l + 1] > s.rbeg[l]) buckets[s.w[l]].push_back(l);
    std::vector<int64_t> cnt(s.m + 1), cur(s.m);
    std::vector<char> any(s.m, 0);
    for (auto &kv : buckets) {
        const int w = kv.first;
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int64_t l : kv.second)
            for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++) cnt[s.rows[r] + 1]++;
        for (int64_t i = 0; i < s.m; i++) cnt[i + 1] += cnt[i];
        const bool single = buckets.size() == 1;
        // swept only as the single bucket: with several, every bucket's launch would sweep x and all of
        // y again (mixed-width NS fp64: 904 -> 1280 us measured)
        if ((single || h->sweep_mode == 1) && sweep_possible(h, w, s.n)) {
            // every output row a segment (rows without blocks in this bucket keep beta * y)
            std::vector<Entry> ents(cnt[s.m]);
            for (int64_t i = 0; i < s.m; i++) cur[i] = cnt[i];
            for (int64_t l : kv.second)
                for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++)
                    ents[cur[s.rows[r]]++] = {(uint32_t)s.col0[l], s.voff[l] + (r - s.rbeg[l]) * w};
            std::vector<int64_t> sb(cnt.begin(), cnt.end());
            if (want_sweep(h, w, s.n, sb, ents)) {
                std::vector<int32_t> out(s.m);
                for (int64_t i = 0; i < s.m; i++) out[i] = (int32_t)i;
                PendingSweep pw;
                int tile0 = 0;
                if (int st = build_sweep(h, 1, w, sb, ents, out, val, ar, tile0, pw)) return st;
                h->bytes_f += s.m * h->esz;  // y written once per bucket
                std::fill(any.begin(), any.end(), 1);
                Ls.emplace_back();
                Ls.back().sweep_tiles = tile0;
                Ls.back().sweep_tile_bytes = h->sweep_tile;
                if (const char *e = ablation_knob("VBC_SWEEP_DIAG")) Ls.back().sweep_diag = atoi(e);
                pbs.push_back({});
                pss.push_back({});
                pws.push_back({pw});
                continue;
            }
        }
        std::vector<int64_t> sbeg{0};
        std::vector<int32_t> sout;
        for (int64_t i = 0; i < s.m; i++)
            if (single || cnt[i + 1] > cnt[i]) { sbeg.push_back(cnt[i + 1]); sout.push_back((int32_t)i); }
        std::vector<int64_t> order;
        const bool slotted = want_slots(h, 1, w, sbeg, (int64_t)cnt[s.m], s.n, order) != 0;
        std::vector<Entry> ents(cnt[s.m]);
        for (int64_t i = 0; i < s.m; i++) cur[i] = cnt[i];
        for (int64_t l : kv.second)
            for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++) {
                const int64_t i = s.rows[r];
                const int64_t e = cur[i]++;
                ents[e] = {(uint32_t)s.col0[l] | (!slotted && e == cnt[i] ? kHead : 0u), s.voff[l] + (r - s.rbeg[l]) * w};
            }
        Ls.emplace_back();
        if (single) {  // node-blocked rows: the planar forward layout with row runs (or lane streams)
            const int R = fwd_runs(h, w, s.m, ents, sbeg);
            PendingSlot ps;
            int zero = 0;
            const bool lanes = R > 1 && want_fwd_lanes(h, w, R, s.m, sbeg);
            if (lanes) {
                if (int st = build_fwd_lanes(h, w, R, ents, sbeg, s.m, val, ar, ps)) return st;
            }
            bool fpair = false;
            if (!lanes && R == 3) {
                const int st = build_fwd_pair(h, w, R, ents, sbeg, s.m, s.n, val, ar, ps);
                if (st != VBC_OK && st != kBuildDeclined) return st;
                fpair = st == VBC_OK;
            }
            if (lanes || fpair || (R > 1 && build_fwd_runs(h, w, R, ents, sbeg, s.m, val, ar, zero, ps))) {
                std::vector<PendingSlot> one;
                one.push_back(std::move(ps));
                commit_launch_keys(h, one, ar);
                const PendingSlot &p1 = one[0];
                if (lanes)  // real values, one key per block, nlive per row, the tile tables, y
                    h->bytes_f += p1.real * (int64_t)R * h->esz + p1.key_bytes + p1.rows * 4 +
                                  (int64_t)p1.b.ntiles * (8 + 128) + s.m * h->esz;
                else if (fpair)  // run-rows of 32 blocks (288 values), one key per block, y
                    h->bytes_f += p1.rows * 288 * (int64_t)h->esz + p1.key_bytes + (p1.b.mask ? p1.rows * 4 : 0) +
                                  s.m * h->esz;
                else
                    h->bytes_f += p1.rows * p1.b.rpi * (int64_t)w * R * h->esz + p1.key_bytes + s.m * h->esz;
                std::fill(any.begin(), any.end(), 1);
                pbs.push_back({});
                pss.push_back(std::move(one));
                pws.push_back({});
                continue;
            }
        }
        if (slotted) {
            PendingSlot ps;
            int srange0 = 0;
            if (int st = build_slots(h, 1, w, w, ents, sbeg, sout, (int64_t)ents.size(), val, ar, srange0, ps, order)) return st;
            std::vector<PendingSlot> one;
            one.push_back(std::move(ps));
            commit_launch_keys(h, one, ar);
            const PendingSlot &p1 = one[0];
            h->bytes_f += p1.rows * p1.b.rpi * (int64_t)w * h->esz + p1.key_bytes +
                          (int64_t)sout.size() * h->esz;
            for (int32_t i : sout) any[i] = 1;
            pbs.push_back({});
            pss.push_back(std::move(one));
            pws.push_back({});
            Ls.back().slot_ranges = srange0;
            continue;
        }
        std::vector<int32_t> out;
        for (int64_t i = 0; i < s.m; i++)
            if (cnt[i + 1] > cnt[i]) { out.push_back((int32_t)i); any[i] = 1; }
        PendingBin pb;
        int range0 = 0;
        if (int st = build_bucket(h, 1, w, ents, out, (int64_t)ents.size(), val, ar, range0, pb)) return st;
        h->bytes_f += (int64_t)ents.size() * (4 + (int64_t)w * h->esz) + (int64_t)out.size() * (4 + h->esz);
        pbs.push_back({pb});
        pss.push_back({});
        pws.push_back({});
        Ls.back().total_ranges = range0;
    }
    h->f_scale = buckets.size() > 1;
    if (buckets.size() <= 1)
        for (int64_t i = 0; i < s.m; i++)
            if (!any[i]) fill.push_back((int32_t)i);
    if (h->f_scale) h->bytes_f += s.m * h->esz * 2 * (int64_t)buckets.size();
    h->bytes_f += s.n * h->esz;
    return VBC_OK;
}

struct PendingPanel {
    PanelBin b;
    TileBin tb;  // tile: a small-tile bucket (vbc_tiles.h; o_rgrp = its range table)
    bool tile = false;
    size_t o_key, o_val, o_out, o_rgrp, o_rseg;
};

// Tile layout (vbc_tiles.h) of one width bucket (w <= 4, whole stripes) of the multi-RHS product: each
// stripe's stored rows grouped into tiles of consecutive rows of one row group -- Π's block rows (tgrp:
// their 0-based starts + m; a SparseMatrixVBC's u x w blocks, constructors_VBC.jl:95-105) or, for a 1DVBC,
// aligned runs of R rows (R in {4, 3, 2}: the node runs of a stiffness operator; the R adding the fewest
// tiles within kTilePad of padding).  A tile slot holds ub rows x w values (rows the tile does not store:
// zeros, masked in its key).  Stripes in natural order are cut into ranges (one wave each) of at most
// smax stripes (the LDS output stage) balanced by tiles, a whole number of rounds of resident waves; each
// range into 4 streams of consecutive stripes balanced by tiles (the wave's 16-lane rows), every stream
// padded to the longest with invalid tiles.  Returns false (nothing built) when the bucket does not fit:
// a tile taller than 4 rows, too much padding, too few rows per tile (auto), rows >= 2^26.
constexpr double kTilePad = 1.25;

// Launch order of the tile ranges (round 6): BFS balls of K ranges over the graph "two ranges store a tile of
// the same X row group", ball after ball.  Each XCD takes a contiguous run of the launch's ranges and keeps
// about K of them resident (K = one XCD's share of the wave slots), so at any moment it folds one ball: a
// compact region of the operator whose X rows -- its groups plus one layer -- fit the XCD's 4 MB L2, where
// the natural order's resident ranges form a slab of consecutive stripes whose X window (a 3D mesh's +-g^2
// rows) does not.  Only the order changes: every range keeps its stripes, streams and data.
// rg_off / rg_grp: the distinct row groups of each range (CSR, ranges in natural order).
static std::vector<int64_t> cluster_ranges(int64_t nrg, const std::vector<int64_t> &rg_off,
                                           const std::vector<int32_t> &rg_grp, int64_t ngroups, int64_t K)
{
    std::vector<int64_t> gcnt(ngroups + 1, 0);  // row group -> ranges (CSR)
    for (int32_t g : rg_grp) gcnt[g + 1]++;
    for (int64_t g = 0; g < ngroups; g++) gcnt[g + 1] += gcnt[g];
    std::vector<int32_t> grg(rg_grp.size());
    {
        std::vector<int64_t> pos(gcnt.begin(), gcnt.end() - 1);
        for (int64_t r = 0; r < nrg; r++)
            for (int64_t q = rg_off[r]; q < rg_off[r + 1]; q++) grg[pos[rg_grp[q]]++] = (int32_t)r;
    }
    std::vector<int64_t> order;
    order.reserve(nrg);
    std::vector<char> done(nrg, 0), gseen(ngroups, 0);
    std::vector<int64_t> touched;  // groups expanded by the current ball (reset after it)
    int64_t seed = 0;
    while ((int64_t)order.size() < nrg) {
        while (done[seed]) seed++;
        const size_t b0 = order.size();
        order.push_back(seed);
        done[seed] = 1;
        for (size_t h = b0; h < order.size() && (int64_t)(order.size() - b0) < K; h++) {
            const int64_t r = order[h];
            for (int64_t q = rg_off[r]; q < rg_off[r + 1] && (int64_t)(order.size() - b0) < K; q++) {
                const int32_t g = rg_grp[q];
                if (gseen[g]) continue;
                gseen[g] = 1;
                touched.push_back(g);
                for (int64_t t = gcnt[g]; t < gcnt[g + 1] && (int64_t)(order.size() - b0) < K; t++) {
                    const int32_t r2 = grg[t];
                    if (!done[r2]) {
                        done[r2] = 1;
                        order.push_back(r2);
                    }
                }
            }
        }
        for (int64_t g : touched) gseen[g] = 0;
        touched.clear();
    }
    return order;
}

static bool build_tiles(vbc_handle *h, const Stripes &s, const std::vector<int64_t> &stripes_in, int w,
                        const std::vector<int64_t> *tgrp, const char *val, Arena &ar, PendingPanel &pp)
{
    const std::vector<int64_t> &stripes = stripes_in;  // (natural order)
    if (h->panel_tiles == 0 || w < 1 || w > 4 || stripes.empty() || s.m >= (int64_t)kTileRow) return false;
    for (int64_t l : stripes)
        if (s.w[l] != w || s.vstride(l) != w) return false;
    const int esz = h->esz;
    int64_t rows = 0;
    for (int64_t l : stripes) rows += s.rbeg[l + 1] - s.rbeg[l];
    // group of a row: base row and height
    std::vector<int32_t> gk;  // tgrp: row -> block row
    if (tgrp) {
        gk.assign((size_t)s.m, 0);
        for (size_t k = 0; k + 1 < tgrp->size(); k++)
            for (int64_t i = (*tgrp)[k]; i < (*tgrp)[k + 1] && i < s.m; i++) gk[i] = (int32_t)k;
    }
    // tiles of a stripe under grouping R (R = 0: tgrp): consecutive stored rows of one group, a repeated
    // slot row (a hand-built stripe storing a row twice) starting a new tile
    auto group_of = [&](int64_t row, int R, int64_t &base, int &u) {
        if (R == 0) {
            const int32_t k = gk[row];
            base = (*tgrp)[k];
            u = (int)((*tgrp)[k + 1] - base);
        } else {
            base = row / R * R;
            u = R;
        }
    };
    auto count = [&](int R, int64_t &tiles, int &ub) {
        tiles = 0;
        ub = 1;
        for (int64_t l : stripes) {
            int64_t cb = -1;
            unsigned seen = 0;
            for (int64_t q = s.rbeg[l]; q < s.rbeg[l + 1]; q++) {
                int64_t base;
                int u;
                group_of(s.rows[q], R, base, u);
                if (u > 4) return false;
                const unsigned bit = 1u << (s.rows[q] - base);
                if (base != cb || (seen & bit)) {
                    tiles++;
                    cb = base;
                    seen = 0;
                }
                seen |= bit;
                ub = std::max(ub, u);
            }
        }
        return true;
    };
    int R = 0, ub = 1;
    int64_t tiles = 0;
    if (tgrp) {
        if (!count(0, tiles, ub)) return false;
        if ((double)tiles * ub > kTilePad * (double)std::max<int64_t>(rows, 1) && h->panel_tiles < 0) return false;
    } else {
        int64_t best = -1;
        for (int Rc = 4; Rc >= 1; Rc--) {
            int64_t t;
            int u;
            count(Rc, t, u);
            if (Rc > 1 && (double)t * Rc > kTilePad * (double)std::max<int64_t>(rows, 1)) continue;
            if (best < 0 || t < best) {
                best = t;
                R = Rc;
                ub = Rc;
                tiles = t;
            }
        }
    }
    // auto: only when tiles carry work (>= 1.5 rows each); VBC_PANEL_TILES=1 takes any
    if (h->panel_tiles < 0 && (double)rows < 1.5 * (double)std::max<int64_t>(tiles, 1)) return false;
    const int TV = ub * w;
    const int64_t n = (int64_t)stripes.size();
    std::vector<int64_t> tl(n);  // tiles per stripe (an empty stripe: one invalid LAST tile)
    {
        for (int64_t i = 0; i < n; i++) {
            const int64_t l = stripes[i];
            int64_t t = 0, cb = -1;
            unsigned seen = 0;
            for (int64_t q = s.rbeg[l]; q < s.rbeg[l + 1]; q++) {
                int64_t base;
                int u;
                group_of(s.rows[q], R, base, u);
                const unsigned bit = 1u << (s.rows[q] - base);
                if (base != cb || (seen & bit)) {
                    t++;
                    cb = base;
                    seen = 0;
                }
                seen |= bit;
            }
            tl[i] = std::max<int64_t>(t, 1);
        }
    }
    // ranges: <= smax stripes (the LDS stage), a whole number of rounds of resident waves, balanced by tiles
    const int64_t smax = std::max<int64_t>(1, kTileStageBytes / (w * 16 * esz));
    const int64_t slots = (int64_t)h->cus * std::max(1, h->occ_tiles);
    int64_t total = 0;
    for (int64_t t : tl) total += t;
    const int nbt = h->tile_nbt;  // the kernel's batch (streams padded to whole pairs of batches)
    // Ranges of ~tile_spr stripes: the hardware dispatches workgroups in order and each XCD takes a
    // contiguous run of ranges (xcd_block), so the stripes in flight on an XCD span its resident waves x
    // the range length -- and a 3D mesh's X rows are reused across +-g^2 nodes, so that front must stay
    // narrow for the X tiles to hit in the XCD's 4 MB L2 (c5-mesh: 28 stripes per range, L2 hit rate 57 %).
    int64_t nr = std::max<int64_t>((n + smax - 1) / smax, 1);
    nr = std::max<int64_t>(nr, (n + h->tile_spr - 1) / std::max(1, h->tile_spr));
    // few ranges: a whole number of rounds of resident waves, but no range so short that its streams'
    // padding to whole key pairs dominates (>= 4 batch pairs per stream on average)
    if (nr < 2 * slots) {
        const int64_t nr_cap = std::max<int64_t>(nr, total / (4 * 8 * nbt));
        nr = std::min<int64_t>(nr_cap, (nr + slots - 1) / slots * slots);
    }
    nr = std::min<int64_t>(n, nr);
    if (const char *e = tuning_knob("VBC_TILE_RANGES")) nr = std::min<int64_t>(n, std::max<int64_t>(1, atoll(e)));
    std::vector<int64_t> rb{0};  // range starts (stripe index)
    {
        int64_t cum = 0;
        for (int64_t i = 0; i < n; i++) {
            const int64_t cnt = i - rb.back();
            if (cnt > 0 && (cnt >= smax || (cum * nr >= (int64_t)rb.size() * total && (int64_t)rb.size() < nr))) rb.push_back(i);
            cum += tl[i];
        }
        rb.push_back(n);
    }
    const int64_t nrg = (int64_t)rb.size() - 1;
    // streams of each range: 4 runs of consecutive stripes balanced by tiles
    std::vector<int32_t> rinfo((size_t)nrg * 8, 0);
    std::vector<std::array<int64_t, 5>> sb(nrg);
    int64_t slot_total = 0;
    for (int64_t r = 0; r < nrg; r++) {
        const int64_t a = rb[r], e = rb[r + 1];
        int64_t rt = 0;
        for (int64_t i = a; i < e; i++) rt += tl[i];
        auto &b = sb[r];
        b[0] = a;
        int64_t cum = 0, i = a;
        for (int k = 1; k < 4; k++) {
            // first stripe of stream k: where the cumulative tiles pass k / 4 of the range's (closer side)
            while (i < e && (cum + tl[i]) * 4 <= k * rt) cum += tl[i++];
            if (i < e && (cum + tl[i]) * 4 - k * rt < k * rt - cum * 4) cum += tl[i++];
            b[k] = i;
        }
        b[4] = e;
        int64_t len = 0;
        for (int k = 0; k < 4; k++) {
            int64_t t = 0;
            for (int64_t q = b[k]; q < b[k + 1]; q++) t += tl[q];
            len = std::max(len, t);
        }
        len = (len + 2 * nbt - 1) / (2 * nbt) * (2 * nbt);  // whole key pairs (vbc_tiles.h)
        int32_t *ri = &rinfo[(size_t)r * 8];
        ri[0] = (int32_t)slot_total;
        ri[1] = (int32_t)len;
        ri[2] = (int32_t)a;
        ri[3] = (int32_t)(e - a);
        for (int k = 1; k < 4; k++) ri[3 + k] = (int32_t)(b[k] - a);
        slot_total += 4 * len;
        if (slot_total >= (int64_t(1) << 31) / std::max(1, TV)) return false;
    }
    // over-read padding past the last stream: keys 3 D batches ahead, values 2 D (vbc_tiles.h)
    const int dep = h->tile_depth;
    const int64_t kpad = 3 * dep * nbt + 16, vpad = (int64_t)(2 * dep * nbt + 2) * TV + 64;
    pp = PendingPanel{};
    pp.tile = true;
    TileBin &tb = pp.tb;
    tb.w = w;
    tb.ub = ub;
    tb.nbt = nbt;
    tb.depth = dep;
    if (const char *e = ablation_knob("VBC_TILE_DIAG")) tb.diag = atoi(e);
    {
        int64_t most = 1;
        for (size_t r = 0; r + 1 < rb.size(); r++) most = std::max<int64_t>(most, rb[r + 1] - rb[r]);
        tb.stage_bytes = (int32_t)((most * w * 16 * esz + 15) / 16 * 16);
    }
    tb.nranges = (int32_t)nrg;
    std::vector<int32_t> out(n);
    for (int64_t i = 0; i < n; i++) out[i] = (int32_t)s.col0[stripes[i]];
    tb.out_affine = 1;
    tb.out_base = out[0];
    tb.out_stride = n > 1 ? out[1] - out[0] : w;
    for (int64_t i = 1; i < n && tb.out_affine; i++) tb.out_affine = (int64_t)out[i] == (int64_t)out[0] + i * tb.out_stride;
    pp.o_key = ar.reserve((slot_total + kpad) * 4);
    pp.o_val = ar.reserve((slot_total * TV + vpad) * esz);
    pp.o_out = ar.reserve(n * 4);
    pp.o_rgrp = ar.reserve(rinfo.size() * 4);
    std::memcpy(ar.at<int32_t>(pp.o_out), out.data(), out.size() * 4);
    std::memcpy(ar.at<int32_t>(pp.o_rgrp), rinfo.data(), rinfo.size() * 4);
    uint32_t *key = ar.at<uint32_t>(pp.o_key);
    char *vv = ar.at<char>(pp.o_val);
    std::fill(key, key + slot_total + kpad, kTileRow);  // padding: invalid tiles (row field all ones)
    std::memset(vv, 0, (size_t)(slot_total * TV + vpad) * esz);
    bool masku = false;
    // the distinct X row groups of each range (cluster_ranges): group = block row (tgrp) or row / R
    // (VBC_TILE_CLUSTER=2: any range count, balls of an eighth of the ranges -- small-scale tests)
    const int64_t K = h->tile_cluster == 2 ? std::max<int64_t>(1, nrg / 8) : std::max<int64_t>(1, slots / 8);
    const bool cluster = h->tile_cluster == 2 ? nrg >= 2 : h->tile_cluster && nrg >= 4 * K;
    const int64_t ngroups = R == 0 ? (int64_t)tgrp->size() : s.m / R + 1;
    std::vector<int64_t> rg_off{0};
    std::vector<int32_t> rg_grp, last;
    if (cluster) last.assign((size_t)ngroups, -1);
    for (int64_t r = 0; r < nrg; r++) {
        const int32_t *ri = &rinfo[(size_t)r * 8];
        const int64_t len = ri[1];
        for (int k = 0; k < 4; k++) {
            int64_t slot = ri[0] + k * len;  // this stream's next tile slot
            for (int64_t i = sb[r][k]; i < sb[r][k + 1]; i++) {
                const int64_t l = stripes[i];
                if (s.rbeg[l + 1] == s.rbeg[l]) {  // empty stripe: one invalid LAST tile (its columns get beta * Y)
                    key[slot++] = kTileLast | kTileRow;
                    continue;
                }
                int64_t cb = -1, kbase = 0;
                unsigned seen = 0;
                for (int64_t q = s.rbeg[l]; q < s.rbeg[l + 1]; q++) {
                    int64_t base;
                    int u;
                    group_of(s.rows[q], R, base, u);
                    const int rr = (int)(s.rows[q] - base);
                    const unsigned bit = 1u << rr;
                    if (base != cb || (seen & bit)) {
                        if (cluster) {
                            const int64_t gi = R == 0 ? gk[base] : base / R;
                            if (last[gi] != r) {
                                last[gi] = (int32_t)r;
                                rg_grp.push_back((int32_t)gi);
                            }
                        }
                        if (cb >= 0) {
                            key[slot] = (uint32_t)kbase | kTileValid | (seen << kTileMaskShift);
                            masku = masku || seen != (1u << ub) - 1;
                            slot++;
                        }
                        cb = base;
                        kbase = base;
                        seen = 0;
                    }
                    seen |= bit;
                    std::memcpy(vv + (slot * TV + (int64_t)rr * w) * esz, val + (s.voff[l] + (q - s.rbeg[l]) * w) * esz,
                                (size_t)w * esz);
                }
                key[slot] = (uint32_t)kbase | kTileValid | (seen << kTileMaskShift) | kTileLast;
                masku = masku || seen != (1u << ub) - 1;
                slot++;
            }
        }
        if (cluster) rg_off.push_back((int64_t)rg_grp.size());
    }
    if (cluster) {  // launch the ranges ball by ball (the arena's rinfo rows permuted; the data stays put)
        const std::vector<int64_t> ord = cluster_ranges(nrg, rg_off, rg_grp, ngroups, K);
        int32_t *dst = ar.at<int32_t>(pp.o_rgrp);
        for (int64_t q = 0; q < nrg; q++) std::memcpy(dst + q * 8, &rinfo[(size_t)ord[q] * 8], 8 * sizeof(int32_t));
    }
    tb.masku = masku ? 1 : 0;
    h->bytes_m += slot_total * (4 + (int64_t)TV * esz) + nrg * 32;
    if (layout_knob("VBC_VERBOSE"))
        fprintf(stderr, "[vbc] tiles: w %d, %lld stripes, %lld rows -> %lld tiles of <= %d rows (%s), %lld ranges, %lld slots%s%s\n",
                w, (long long)n, (long long)rows, (long long)total, ub, R == 0 ? "block rows" : "row runs", (long long)nrg,
                (long long)slot_total, masku ? ", masked rows" : "", cluster ? ", clustered launch order" : "");
    return true;
}

// Panel layout (vbc_panel.h) of the transposed product: per width bucket (stripes wider than 16 are
// cut into 16-column pieces that share the stripe's rows), S = 16/w consecutive stripes per panel,
// each panel's rows padded to a multiple of 4, ranges of whole panels balanced by rows.
static int build_panel(vbc_handle *h, const Stripes &s, const char *val, Arena &ar,
                       std::vector<PendingPanel> &pps, PanelLaunch &L, std::vector<int32_t> &fill,
                       const std::vector<int64_t> *tgrp = nullptr)
{
    struct Piece {
        int64_t l;
        int c0;
    };
    std::map<int, std::vector<Piece>> buckets;  // piece width -> pieces
    // Stripes that store no row stay in the layout with one HEAD sentinel row (zero contribution), so
    // uniform-width matrices keep an affine stripe -> column map and no fill list is needed.
    (void)fill;
    for (int64_t l = 0; l < s.L; l++)
        for (int c0 = 0; c0 < s.w[l]; c0 += 16) buckets[std::min(16, s.w[l] - c0)].push_back({l, c0});
    // small tiles (u, w <= 4): the tile-granular layout (vbc_tiles.h) instead of panels
    if (!tgrp && !s.grp.empty()) tgrp = &s.grp;
    for (auto it = buckets.begin(); it != buckets.end();) {
        bool whole = it->first <= 4;
        std::vector<int64_t> st;
        for (const Piece &pc : it->second) {
            whole = whole && pc.c0 == 0;
            st.push_back(pc.l);
        }
        PendingPanel pp;
        if (whole && build_tiles(h, s, st, it->first, tgrp, val, ar, pp)) {
            pps.push_back(pp);
            it = buckets.erase(it);
        } else {
            ++it;
        }
    }
    const int esz = h->esz;
    // groups of every bucket first: ranges are spread over the launch in proportion to them
    std::map<int, std::vector<int64_t>> pgroups;  // w -> groups per panel
    int64_t total_groups = 0;
    for (auto &kv : buckets) {
        const int S = 16 / kv.first;
        auto &pg = pgroups[kv.first];
        for (size_t p0 = 0; p0 < kv.second.size(); p0 += S) {
            int64_t rows = 0;
            for (size_t p = p0; p < std::min(kv.second.size(), p0 + S); p++)
                rows += std::max<int64_t>(1, s.rbeg[kv.second[p].l + 1] - s.rbeg[kv.second[p].l]);
            pg.push_back((rows + 3) / 4);
            total_groups += pg.back();
        }
    }
    if (total_groups >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "matrix too large for the panel layout");
    int range0 = 0;
    for (auto &kv : buckets) {
        const int w = kv.first, S = 16 / w;
        const std::vector<Piece> &pcs = kv.second;
        const std::vector<int64_t> &pg = pgroups[w];
        int64_t G = 0;
        for (int64_t g : pg) G += g;
        int64_t nr = (int64_t)std::llround((double)h->target_ranges_m * (double)G / (double)std::max<int64_t>(total_groups, 1));
        nr = std::max<int64_t>(1, std::min<int64_t>(nr, (int64_t)pg.size()));
        std::vector<int32_t> rgrp{0}, rseg{0};
        int64_t acc = 0;
        for (size_t p = 0; p < pg.size(); p++) {
            acc += pg[p];
            // close a range once it holds its share of the bucket's groups
            if (p + 1 < pg.size() && (int64_t)rgrp.size() < nr && acc * nr >= (int64_t)rgrp.size() * G) {
                rgrp.push_back((int32_t)acc);
                rseg.push_back((int32_t)((p + 1) * S));
            }
        }
        rgrp.push_back((int32_t)acc);
        nr = (int64_t)rseg.size();
        PendingPanel pp{};
        pp.b.w = w;
        pp.b.S = S;
        pp.b.range0 = range0;
        pp.b.nranges = (int32_t)nr;
        range0 += (int)nr;
        std::vector<int32_t> out(pcs.size());
        for (size_t p = 0; p < pcs.size(); p++) out[p] = (int32_t)(s.col0[pcs[p].l] + pcs[p].c0);
        pp.b.out_affine = 1;
        pp.b.out_base = out[0];
        pp.b.out_stride = out.size() > 1 ? out[1] - out[0] : 0;
        for (size_t q = 1; q < out.size() && pp.b.out_affine; q++)
            pp.b.out_affine = (int64_t)out[q] == (int64_t)out[0] + (int64_t)q * pp.b.out_stride;
        const int64_t Rp = acc * 4;
        const int64_t Ra = Rp + kPanelTail;  // over-read padding (vbc_panel.h)
        h->panel_val_bytes = std::max<int64_t>(h->panel_val_bytes, Ra * w * esz);
        pp.b.val_bytes = (int32_t)std::min<int64_t>(Ra * w * esz, 0x7FFFFFFF);
        pp.o_key = ar.reserve(Ra * 4);
        pp.o_val = ar.reserve(Ra * w * esz);
        pp.o_out = ar.reserve(out.size() * 4);
        pp.o_rgrp = ar.reserve(rgrp.size() * 4);
        pp.o_rseg = ar.reserve(rseg.size() * 4);
        std::memcpy(ar.at<int32_t>(pp.o_out), out.data(), out.size() * 4);
        std::memcpy(ar.at<int32_t>(pp.o_rgrp), rgrp.data(), rgrp.size() * 4);
        std::memcpy(ar.at<int32_t>(pp.o_rseg), rseg.data(), rseg.size() * 4);
        uint32_t *key = ar.at<uint32_t>(pp.o_key);
        char *vv = ar.at<char>(pp.o_val);
        int64_t row = 0;
        for (size_t p0 = 0; p0 < pcs.size(); p0 += S) {
            for (size_t p = p0; p < std::min(pcs.size(), p0 + S); p++) {
                const int64_t l = pcs[p].l;
                const int wl = s.w[l];
                for (int64_t q = s.rbeg[l]; q < s.rbeg[l + 1]; q++, row++) {
                    key[row] = (uint32_t)s.rows[q] | (q == s.rbeg[l] ? kHead : 0u);
                    std::memcpy(vv + row * w * esz, val + (s.voff[l] + (q - s.rbeg[l]) * wl + pcs[p].c0) * esz,
                                (size_t)w * esz);
                }
                if (s.rbeg[l + 1] == s.rbeg[l]) {  // empty stripe: one HEAD sentinel row
                    key[row] = kPanelSentinel | kHead;
                    std::memset(vv + row * w * esz, 0, (size_t)w * esz);
                    row++;
                }
            }
            for (; row % 4; row++) {
                key[row] = kPanelSentinel;
                std::memset(vv + row * w * esz, 0, (size_t)w * esz);
            }
        }
        for (; row < Ra; row++) {
            key[row] = kPanelSentinel;
            std::memset(vv + row * w * esz, 0, (size_t)w * esz);
        }
        h->bytes_m += Rp * (4 + (int64_t)w * esz) + (int64_t)out.size() * 4;
        pps.push_back(pp);
    }
    L.total_ranges = range0;
    return VBC_OK;
}

// C = Bᵀ as stripes (the layouts of B's forward product built as transposed products of C): C's stripes
// are B's output row groups g (rows [a_g, a_g + u_g), u_g <= maxu): Π's block rows for a SparseMatrixVBC,
// else runs of consecutive rows whose stripe lists are identical (a node's dof rows), else single rows.
// Every stripe l of B that stores rows of group g contributes w_l stored rows of C (its columns c,
// ascending), each holding the u_g values B[a_g .. a_g+u_g-1, col0_l + c] and gathering x row col0_l + c.
// Groups in row order, their stripes in stripe order (the reference's forward loop,
// multiply_VBC.jl:68-77).  Every row of a group is stored by the same stripes, so C holds exactly the
// values (fill zeros included) the reference multiplies.
static int transpose_stripes(const vbc_handle *h, const Stripes &s, const char *val, int maxu, Stripes &c,
                             std::vector<char> &cv)
{
    const int esz = h->esz;
    const int64_t m = s.m;
    // row groups
    std::vector<int64_t> a;
    if (!s.grp.empty()) {
        for (size_t k = 0; k + 1 < s.grp.size(); k++)
            for (int64_t i = s.grp[k]; i < s.grp[k + 1]; i += maxu) a.push_back(i);  // taller blocks: pieces
    } else {
        // the stripes storing each row (rows ascend inside a stripe, so each list comes out sorted)
        std::vector<int64_t> cnt(m + 1, 0);
        for (int64_t q = 0; q < (int64_t)s.rows.size(); q++) cnt[s.rows[q] + 1]++;
        for (int64_t i = 0; i < m; i++) cnt[i + 1] += cnt[i];
        std::vector<int64_t> lst(s.rows.size()), fillp(cnt.begin(), cnt.end() - 1);
        for (int64_t l = 0; l < s.L; l++)
            for (int64_t q = s.rbeg[l]; q < s.rbeg[l + 1]; q++) lst[fillp[s.rows[q]]++] = l;
        auto same = [&](int64_t i, int64_t j) {
            return cnt[i + 1] - cnt[i] == cnt[j + 1] - cnt[j] &&
                   std::equal(lst.begin() + cnt[i], lst.begin() + cnt[i + 1], lst.begin() + cnt[j]);
        };
        for (int64_t i = 0; i < m;) {
            int64_t e = i + 1;
            while (e < m && e - i < maxu && cnt[i + 1] > cnt[i] && same(i, e)) e++;
            a.push_back(i);
            i = e;
        }
    }
    a.push_back(m);
    const int64_t ng = (int64_t)a.size() - 1;
    std::vector<int64_t> gof(m);
    for (int64_t g = 0; g < ng; g++)
        for (int64_t i = a[g]; i < a[g + 1]; i++) gof[i] = g;
    // (group, stripe) blocks: stored rows of B grouped
    struct Blk {
        int64_t g, l, q0;  // q0: first stored row of the stripe inside the group
    };
    std::vector<Blk> blks;
    for (int64_t l = 0; l < s.L; l++) {
        int64_t prev = -1;
        for (int64_t q = s.rbeg[l]; q < s.rbeg[l + 1]; q++) {
            const int64_t g = gof[s.rows[q]];
            if (g != prev) blks.push_back({g, l, q});
            prev = g;
        }
    }
    std::stable_sort(blks.begin(), blks.end(), [](const Blk &x, const Blk &y) { return x.g < y.g; });
    c = Stripes{};
    c.m = s.n;  // C = Bᵀ: its x is B's x (length n), its y is B's y (length m)
    c.n = m;
    c.L = ng;
    c.col0.resize(ng);
    c.w.resize(ng);
    c.rbeg.assign(ng + 1, 0);
    c.voff.resize(ng);
    for (int64_t g = 0; g < ng; g++) {
        c.col0[g] = a[g];
        c.w[g] = (int32_t)(a[g + 1] - a[g]);
    }
    for (const Blk &b : blks) c.rbeg[b.g + 1] += s.w[b.l];
    for (int64_t g = 0; g < ng; g++) c.rbeg[g + 1] += c.rbeg[g];
    const int64_t rows = c.rbeg[ng];
    if (rows >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "matrix too large for the forward panel layout");
    c.rows.resize(rows);
    int64_t nv = 0;
    for (int64_t g = 0; g < ng; g++) {
        c.voff[g] = nv;
        nv += (c.rbeg[g + 1] - c.rbeg[g]) * c.w[g];
    }
    cv.assign((size_t)std::max<int64_t>(nv, 1) * esz, 0);
    std::vector<int64_t> at(c.rbeg.begin(), c.rbeg.end() - 1);  // next stored row of each group
    for (const Blk &b : blks) {
        const int64_t l = b.l, wl = s.w[l], u = c.w[b.g];
        for (int64_t cc = 0; cc < wl; cc++) {
            const int64_t row = at[b.g]++;
            c.rows[row] = (int32_t)(s.col0[l] + cc);
            char *dst = cv.data() + (c.voff[b.g] + (row - c.rbeg[b.g]) * u) * esz;
            // a stripe that stores one row twice (hand-built input; the reference's constructors never do)
            // contributes both copies: they are added into the slot, not overwritten
            for (int64_t q = b.q0; q < s.rbeg[l + 1] && gof[s.rows[q]] == b.g; q++) {
                char *d = dst + (s.rows[q] - a[b.g]) * esz;
                const char *v = val + (s.voff[l] + (q - s.rbeg[l]) * wl + cc) * esz;
                if (esz == 8) {
                    double t, u2;
                    std::memcpy(&t, d, 8);
                    std::memcpy(&u2, v, 8);
                    t += u2;
                    std::memcpy(d, &t, 8);
                } else {
                    float t, u2;
                    std::memcpy(&t, d, 4);
                    std::memcpy(&u2, v, 4);
                    t += u2;
                    std::memcpy(d, &t, 4);
                }
            }
        }
    }
    return VBC_OK;
}

// Forward panel layout (VBC_CREATE_MULTI_FORWARD): Y = B·X is the transposed product of C = Bᵀ, so the
// transposed panel layout of C (transpose_stripes, groups up to 16 rows) serves it.
static int build_forward_panel(vbc_handle *h, const Stripes &s, const char *val, Arena &ar,
                               std::vector<PendingPanel> &pps, PanelLaunch &L)
{
    Stripes c;
    std::vector<char> cv;
    if (int st = transpose_stripes(h, s, val, 16, c, cv)) return st;
    const int64_t ng = c.L;
    int32_t widest = 0;
    for (int64_t g = 0; g < ng; g++) widest = std::max(widest, c.w[g]);
    h->mf_group = widest;
    const int64_t bytes0 = h->bytes_m;
    std::vector<int32_t> fill;
    // tile groups of C's rows (B's columns): B's stripes (Φ), so a u x w block of B is a w x u tile of C
    std::vector<int64_t> cg;
    for (int64_t l = 0; l < s.L; l++) cg.push_back(s.col0[l]);
    cg.push_back(s.n);
    const int st = build_panel(h, c, cv.data(), ar, pps, L, fill, &cg);
    h->bytes_mf = h->bytes_m - bytes0;
    h->bytes_m = bytes0;
    return st;
}

static int finalize_panel(vbc_handle *h, const std::vector<PendingPanel> &pps, PanelLaunch &L)
{
    L.bins.clear();
    L.tbins.clear();
    char *base = static_cast<char *>(h->d_arena);
    for (const PendingPanel &pp : pps) {
        if (pp.tile) {
            TileBin t = pp.tb;
            t.key = reinterpret_cast<const uint32_t *>(base + pp.o_key);
            t.val = base + pp.o_val;
            t.out = reinterpret_cast<const int32_t *>(base + pp.o_out);
            t.rinfo = reinterpret_cast<const int32_t *>(base + pp.o_rgrp);
            L.tbins.push_back(t);
            continue;
        }
        PanelBin b = pp.b;
        b.key = reinterpret_cast<const uint32_t *>(base + pp.o_key);
        b.val = base + pp.o_val;
        b.out = reinterpret_cast<const int32_t *>(base + pp.o_out);
        b.rgrp = reinterpret_cast<const int32_t *>(base + pp.o_rgrp);
        b.rseg = reinterpret_cast<const int32_t *>(base + pp.o_rseg);
        L.bins.push_back(b);
    }
    L.d_fill = reinterpret_cast<const int32_t *>(base + L.o_fill);
    if (!L.bins.empty()) {
        VBC_HIP(hipMalloc(&L.d_bins, L.bins.size() * sizeof(PanelBin)));
        VBC_HIP(hipMemcpy(L.d_bins, L.bins.data(), L.bins.size() * sizeof(PanelBin), hipMemcpyHostToDevice));
    }
    return VBC_OK;
}

static int finalize_launch(vbc_handle *h, const std::vector<PendingBin> &pbs, const std::vector<PendingSlot> &pss,
                           Launch &L, const std::vector<PendingSweep> &pws = {})
{
    L.bins.clear();
    L.sbins.clear();
    L.wbins.clear();
    char *base = static_cast<char *>(h->d_arena);
    for (const PendingSweep &pw : pws) {
        SweepBin b = pw.b;
        b.tstep = reinterpret_cast<const int32_t *>(base + pw.o_tstep);
        b.key = reinterpret_cast<const uint32_t *>(base + pw.o_key);
        b.loc = reinterpret_cast<const uint16_t *>(base + pw.o_loc);
        b.sbase = reinterpret_cast<const uint32_t *>(base + pw.o_sbase);
        b.val = base + pw.o_val;
        b.out = reinterpret_cast<const int32_t *>(base + pw.o_out);
        L.wbins.push_back(b);
    }
    if (!L.wbins.empty()) {
        VBC_HIP(hipMalloc(&L.d_wbins, L.wbins.size() * sizeof(SweepBin)));
        VBC_HIP(hipMemcpy(L.d_wbins, L.wbins.data(), L.wbins.size() * sizeof(SweepBin), hipMemcpyHostToDevice));
    }
    for (const PendingBin &pb : pbs) {
        Bin b = pb.b;
        b.key = reinterpret_cast<const uint32_t *>(base + pb.o_key);
        b.val = base + pb.o_val;
        b.rseg = reinterpret_cast<const int32_t *>(base + pb.o_rseg);
        b.out = reinterpret_cast<const int32_t *>(base + pb.o_out);
        b.carry = base + pb.o_carry;
        b.carry_seg = reinterpret_cast<int32_t *>(base + pb.o_cseg);
        L.bins.push_back(b);
    }
    L.pbins.clear();
    for (const PendingSlot &ps : pss) {
        SlotBin b = ps.b;
        b.key = reinterpret_cast<const uint32_t *>(base + ps.o_key);
        b.val = base + ps.o_val;
        b.out = reinterpret_cast<const int32_t *>(base + ps.o_out);
        b.rrow = reinterpret_cast<const int32_t *>(base + ps.o_rrow);
        b.rchunk = reinterpret_cast<const int32_t *>(base + ps.o_rchunk);
        b.base = reinterpret_cast<const uint32_t *>(base + ps.o_base);
        b.kdoff = reinterpret_cast<const uint32_t *>(base + ps.o_doff);
        b.nlive = reinterpret_cast<const uint32_t *>(base + ps.o_nlive);
        b.trow = reinterpret_cast<const int32_t *>(base + ps.o_trow);
        b.tseg = reinterpret_cast<const int32_t *>(base + ps.o_tseg);
        b.lseg = reinterpret_cast<const int16_t *>(base + ps.o_lseg);
        (b.planar ? L.pbins : L.sbins).push_back(b);
    }
    if (!L.pbins.empty()) {
        VBC_HIP(hipMalloc(&L.d_pbins, L.pbins.size() * sizeof(SlotBin)));
        VBC_HIP(hipMemcpy(L.d_pbins, L.pbins.data(), L.pbins.size() * sizeof(SlotBin), hipMemcpyHostToDevice));
    }
    // the fused small-matrix split (build_transposed): every planar bin a split bin of the common P, all
    // of them one launch of spmv_split_multi (their chunks concatenated)
    L.fuse_split = 0;
    if (L.fuse_p > 1) {
        int nfb = 0;
        bool all = true;
        for (const SlotBin &b : L.pbins) {
            if (!b.fused) continue;
            nfb++;
            all = all && b.kind == 0 && b.split == L.fuse_p && !b.kc && !b.lanes && !b.pair && !b.mask &&
                  b.diag == 0 && b.wkey >= 1 && b.wkey <= 8 && b.w == b.wkey && b.run >= 1 && b.run <= 3;
        }
        if (nfb > 0 && nfb <= kSplitParts && all) {
            SplitMulti M{};
            int c0 = 0, i = 0;
            for (const SlotBin &b : L.pbins) {
                if (!b.fused) continue;
                M.p[i++] = SplitPart{b.wkey, b.run, c0, b.nseg, b.out_affine, b.out_base, b.out_stride, b.wst, b.holes, b.ks,
                                     b.rrow, b.key, b.val, b.out};
                c0 += b.nranges;  // a split bin's ranges are its chunks
                M.pad0 = std::max<int32_t>(M.pad0, b.deep);  // slice loop (build_slots)
            }
            M.nparts = nfb;
            M.nchunks = c0;
            L.multi = M;
            L.fuse_split = L.fuse_p;
        } else {
            for (SlotBin &b : L.pbins) b.fused = 0;  // each split bin on its own launch
        }
    }
    L.d_fill = reinterpret_cast<const int32_t *>(base + L.o_fill);
    if (!L.bins.empty()) {
        VBC_HIP(hipMalloc(&L.d_bins, L.bins.size() * sizeof(Bin)));
        VBC_HIP(hipMemcpy(L.d_bins, L.bins.data(), L.bins.size() * sizeof(Bin), hipMemcpyHostToDevice));
    }
    if (!L.sbins.empty()) {
        VBC_HIP(hipMalloc(&L.d_sbins, L.sbins.size() * sizeof(SlotBin)));
        VBC_HIP(hipMemcpy(L.d_sbins, L.sbins.data(), L.sbins.size() * sizeof(SlotBin), hipMemcpyHostToDevice));
    }
    // bytes per launch group, in launch_group's order (sweep, slots, fused split, planar bins, merge)
    L.gwork.clear();
    {
        std::vector<double> pw_planar;
        double slots = 0, fused = 0, sweep = 0, merge = 0;
        size_t pi = 0;
        for (const PendingSlot &ps : pss) {
            const double wk = (double)ps.rows * ps.b.rpi * ps.b.w * h->esz + (double)ps.key_bytes;
            if (!ps.b.planar) slots += wk;
            else if (L.fuse_split && L.pbins[pi++].fused) fused += wk;
            else pw_planar.push_back(wk);
        }
        for (const PendingSweep &pw : pws) sweep += pw.work;
        for (const PendingBin &pb : pbs) merge += pb.work;
        if (L.sweep_tiles > 0) L.gwork.push_back(sweep);
        if (L.slot_ranges > 0) L.gwork.push_back(slots);
        if (L.fuse_split) L.gwork.push_back(fused);
        for (double wk : pw_planar) L.gwork.push_back(wk);
        if (L.total_ranges > 0 || L.nfill > 0) L.gwork.push_back(merge + 1.0);
    }
    return VBC_OK;
}

static void release(vbc_handle *h)
{
    if (!h) return;
    DeviceGuard g(h->device);
    if (h->lt.d_bins) (void)hipFree(h->lt.d_bins);
    if (h->lt.d_sbins) (void)hipFree(h->lt.d_sbins);
    if (h->lt.d_wbins) (void)hipFree(h->lt.d_wbins);
    if (h->lt.d_pbins) (void)hipFree(h->lt.d_pbins);
    if (h->lft.d_bins) (void)hipFree(h->lft.d_bins);
    if (h->lft.d_sbins) (void)hipFree(h->lft.d_sbins);
    if (h->lft.d_wbins) (void)hipFree(h->lft.d_wbins);
    if (h->lft.d_pbins) (void)hipFree(h->lft.d_pbins);
    for (hipStream_t q : h->lft.fork_streams) (void)hipStreamDestroy(q);
    for (hipEvent_t e : h->lft.fork_events) (void)hipEventDestroy(e);
    if (h->lm.d_bins) (void)hipFree(h->lm.d_bins);
    if (h->lmf.d_bins) (void)hipFree(h->lmf.d_bins);
    for (auto &l : h->lf) {
        if (l.d_bins) (void)hipFree(l.d_bins);
        if (l.d_sbins) (void)hipFree(l.d_sbins);
        if (l.d_wbins) (void)hipFree(l.d_wbins);
        if (l.d_pbins) (void)hipFree(l.d_pbins);
    }
    if (h->d_arena) (void)hipFree(h->d_arena);
    if (h->d_carry_mm) (void)hipFree(h->d_carry_mm);
    for (void *p : h->d_stage)
        if (p) (void)hipFree(p);
    if (h->order_ev) (void)hipEventDestroy(h->order_ev);
    for (hipStream_t q : h->lt.fork_streams) (void)hipStreamDestroy(q);
    for (hipEvent_t e : h->lt.fork_events) (void)hipEventDestroy(e);
    delete h;
}

template <typename T>
static int64_t count_nonzeros(const char *val, int64_t n)
{
    const T *v = reinterpret_cast<const T *>(val);
    int64_t c = 0;
    for (int64_t i = 0; i < n; i++) c += (v[i] != T(0));
    return c;
}

// Integer eltypes: the reference layout itself (0-based) in one arena, read by vbc_generic.hip.
static int create_int(vbc_handle *h, const Stripes &s, const int64_t *val, int64_t nval)
{
    Arena ar;
    const int64_t L = s.L, q = (int64_t)s.rows.size();
    const size_t o_col0 = ar.reserve(L * 4), o_w = ar.reserve(L * 4), o_rows = ar.reserve(q * 4);
    const size_t o_c2s = ar.reserve(s.n * 4), o_r2s = ar.reserve(q * 4);
    const size_t o_rbeg = ar.reserve((L + 1) * 8), o_voff = ar.reserve(L * 8), o_val = ar.reserve(nval * 8);
    for (int64_t l = 0; l < L; l++) {
        ar.at<int32_t>(o_col0)[l] = (int32_t)s.col0[l];
        ar.at<int32_t>(o_w)[l] = s.w[l];
        ar.at<int64_t>(o_voff)[l] = s.voff[l];
        for (int64_t c = 0; c < s.w[l]; c++) ar.at<int32_t>(o_c2s)[s.col0[l] + c] = (int32_t)l;
        for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++) ar.at<int32_t>(o_r2s)[r] = (int32_t)l;
    }
    std::memcpy(ar.at<int64_t>(o_rbeg), s.rbeg.data(), (L + 1) * 8);
    if (q) std::memcpy(ar.at<int32_t>(o_rows), s.rows.data(), q * 4);
    if (nval) std::memcpy(ar.at<int64_t>(o_val), val, nval * 8);
    h->arena_bytes = ar.host.size();
    VBC_HIP(hipMalloc(&h->d_arena, h->arena_bytes));
    VBC_HIP(hipMemcpy(h->d_arena, ar.host.data(), h->arena_bytes, hipMemcpyHostToDevice));
    char *b = static_cast<char *>(h->d_arena);
    IntLayout &li = h->li;
    li.L = L;
    li.nrows = q;
    li.col0 = reinterpret_cast<const int32_t *>(b + o_col0);
    li.w = reinterpret_cast<const int32_t *>(b + o_w);
    li.rows = reinterpret_cast<const int32_t *>(b + o_rows);
    li.col2stripe = reinterpret_cast<const int32_t *>(b + o_c2s);
    li.row2stripe = reinterpret_cast<const int32_t *>(b + o_r2s);
    li.rbeg = reinterpret_cast<const int64_t *>(b + o_rbeg);
    li.voff = reinterpret_cast<const int64_t *>(b + o_voff);
    li.val = reinterpret_cast<const int64_t *>(b + o_val);
    h->bytes_t = h->bytes_f = nval * 8 + q * 4 + (s.m + s.n) * 8;
    return VBC_OK;
}

static int create_common(vbc_handle **out, Stripes &s, const void *val, int dtype, int device,
                         unsigned flags, int64_t nval, int64_t K, int64_t nblocks)
{
    if (!out) return fail(VBC_INVALID_ARG, "out handle pointer is NULL");
    *out = nullptr;
    if (dtype != VBC_F64 && dtype != VBC_F32 && dtype != VBC_I64)
        return fail(VBC_UNSUPPORTED_DTYPE, "GPU products compute in Float64, Float32 or Int64 (see vbc_types)");
    if (int st = check_limits(s)) return st;
    int ndev = 0;
    VBC_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(VBC_INVALID_ARG, "device ordinal out of range");
    if ((flags & (VBC_CREATE_TRANSPOSED | VBC_CREATE_FORWARD | VBC_CREATE_MULTI | VBC_CREATE_MULTI_FORWARD)) == 0)
        flags |= VBC_CREATE_TRANSPOSED;

    vbc_handle *h = new vbc_handle();
    h->m = s.m;
    h->n = s.n;
    h->L = s.L;
    h->K = K;
    h->nblocks = nblocks;
    h->nrows = (int64_t)s.rows.size();
    h->nval = nval;
    h->dtype = dtype;
    h->esz = elem_size(dtype);
    h->device = device;
    const char *v = static_cast<const char *>(val);
    h->nnz = dtype == VBC_F64 ? count_nonzeros<double>(v, nval)
           : dtype == VBC_F32 ? count_nonzeros<float>(v, nval) : count_nonzeros<int64_t>(v, nval);

    DeviceGuard g(device);
    if (!g.ok) { release(h); return fail(VBC_HIP_ERROR, "hipSetDevice failed"); }
    if (hipEventCreateWithFlags(&h->order_ev, hipEventDisableTiming) != hipSuccess) {
        release(h);
        return fail(VBC_HIP_ERROR, "hipEventCreate failed");
    }
    if (dtype == VBC_I64) {  // exact integer products (vbc_generic.hip): one layout, both directions
        if (int st = create_int(h, s, static_cast<const int64_t *>(val), nval)) { release(h); return st; }
        h->has_t = (flags & (VBC_CREATE_TRANSPOSED | VBC_CREATE_MULTI)) != 0;
        h->has_f = (flags & (VBC_CREATE_FORWARD | VBC_CREATE_MULTI_FORWARD)) != 0;
        *out = h;
        return VBC_OK;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { release(h); return fail(VBC_HIP_ERROR, "hipGetDeviceProperties failed"); }
    h->tile_k = dtype == VBC_F64 ? 4 : 8;  // measured best (tools/ab.py, FE workload)
    if (const char *e = tuning_knob("VBC_TILE_K")) {
        const int k = atoi(e);
        h->tile_k = (k == 4 || k == 8) ? k : h->tile_k;
    }
    if (const char *e = tuning_knob("VBC_PIPE")) h->pipe = atoi(e) == 3 ? 3 : 2;
    if (const char *e = ablation_knob("VBC_DIAG")) h->diag = atoi(e);
    // one range per resident wave: occupancy of the kernel variant this handle will launch
    int occ[2] = {0, 0};
    occupancy_ranges(h->esz, h->tile_k, h->pipe, occ);
    for (int kd = 0; kd < 2; kd++)
        h->target_ranges_k[kd] = prop.multiProcessorCount * std::max(1, std::min(occ[kd], 8)) * kWavesPerBlock;
    if (const char *e = tuning_knob("VBC_TARGET_RANGES")) h->target_ranges_k[0] = h->target_ranges_k[1] = std::max(1, atoi(e));
    for (int kd = 0; kd < 2; kd++) {
        h->occ_s[kd] = std::max(1, std::min(occupancy_slots(h->esz, kd), 8));
        h->target_ranges_s[kd] = prop.multiProcessorCount * h->occ_s[kd] * kWavesPerBlock;
    }
    if (const char *e = tuning_knob("VBC_TARGET_RANGES_S")) {  // an explicit range count is taken as is
        h->target_ranges_s[0] = h->target_ranges_s[1] = std::max(1, atoi(e));
        h->occ_s[0] = h->occ_s[1] = 1;
    }
    if (const char *e = layout_knob("VBC_RANGE_KB")) h->range_bytes = (int64_t)std::max(0, atoi(e)) << 10;
    if (const char *e = layout_knob("VBC_SLOTS")) h->slots_mode = atoi(e) == 0 ? 0 : atoi(e) == 1 ? 1 : -1;
    if (const char *e = layout_knob("VBC_SLOTS_PAD")) h->slots_pad = atof(e);
    if (const char *e = layout_knob("VBC_SLOTS_SORT")) h->slots_sort = atoi(e);
    if (const char *e = tuning_knob("VBC_SLOT_NARROW")) h->slot_narrow = atoi(e) != 0;
    if (const char *e = layout_knob("VBC_XCD")) h->xcd = atoi(e) != 0;
    if (const char *e = layout_knob("VBC_XCD_P")) h->xcd_p = atoi(e) != 0;
    if (const char *e = layout_knob("VBC_SLOT_KEYS16")) h->slot_keys16 = atoi(e);  // 0 off, 1 auto, 2 always
    if (const char *e = layout_knob("VBC_SLOT_DEDUP")) h->slot_dedup = atoi(e) != 0;
    if (const char *e = layout_knob("VBC_SWEEP")) h->sweep_mode = atoi(e) == 0 ? 0 : atoi(e) == 1 ? 1 : -1;
    h->sweep_tile = (h->esz == 8 ? 4 : 2) * kSweepTileBytes;  // measured on NS: fp64 32 KB 473 us (16 KB 508), fp32 16 KB 313 us (32 KB 353)
    // packed swept keys: NS fp64 464.5 -> 456.2 us, mixed widths 553 -> 539 us; fp32 311 -> 316 us, so
    // fp64 only (profiles/r03_sweeppack_*.log)
    h->sweep_pack = h->esz == 8;
    if (const char *e = layout_knob("VBC_FORK")) h->fork = atoi(e) != 0;
    if (const char *e = tuning_knob("VBC_FORK_SIDE_KB")) h->fork_side_bytes = atof(e) * 1024.0;
    if (const char *e = layout_knob("VBC_SWEEP_PACK")) h->sweep_pack = atoi(e) != 0;
    if (const char *e = layout_knob("VBC_SWEEP_TILE")) h->sweep_tile = atoi(e) >= 32 ? 4 * kSweepTileBytes : atoi(e) >= 16 ? 2 * kSweepTileBytes : kSweepTileBytes;
    if (const char *e = layout_knob("VBC_SLOT_STAGE")) h->slot_stage = (atoi(e) == 4 || atoi(e) == 8) ? atoi(e) : 0;
    if (const char *e = layout_knob("VBC_SLOT_PLANAR")) h->slot_planar = atoi(e) == 0 ? 0 : atoi(e) == 1 ? 1 : -1;
    if (const char *e = layout_knob("VBC_SLOT_RUNS")) h->slot_runs = atoi(e) != 0;
    if (const char *e = layout_knob("VBC_PLANAR_PAIR")) h->planar_pair = atoi(e) == 0 ? 0 : atoi(e) == 2 ? 2 : 1;  // 2: always
    if (const char *e = layout_knob("VBC_PLANAR_MASK")) h->planar_mask = atoi(e) != 0;
    if (const char *e = layout_knob("VBC_PLANAR_MASK_PAIR")) h->planar_mask_pair = atoi(e) != 0;
    if (const char *e = layout_knob("VBC_MASK_WINDOW")) h->mask_window = std::max(1, std::min(64, atoi(e)));
    if (const char *e = layout_knob("VBC_PLANAR_SPLIT")) {  // 0 never, 1 auto, 2 / 4 / 8 forced
        const int v = atoi(e);
        h->planar_split = v == 0 ? 0 : (v == 2 || v == 4 || v == 8) ? v : -1;
    }
    if (flags & VBC_CREATE_SERIAL) {  // every stripe summed serially in stored row order:
        h->planar_split = 0;            // no split planar product (P slices meeting in LDS),
        if (h->slots_mode < 0) h->slots_mode = 1;  // and no merge layout (its segmented scan joins slot sums)
    }
    h->occ_p = std::max(1, std::min(occupancy_planar(h->esz), 8));
    h->target_ranges_l = prop.multiProcessorCount * std::max(1, std::min(occupancy_lanes(h->esz), 8)) * kWavesPerBlock;
    if (const char *e = layout_knob("VBC_PLANAR_LANES")) h->planar_lanes = atoi(e) == 0 ? 0 : atoi(e) == 1 ? 1 : -1;
    if (const char *e = layout_knob("VBC_TARGET_RANGES_L")) h->target_ranges_l = std::max(1, atoi(e));
    if (const char *e = tuning_knob("VBC_LANES_DEEP")) h->lanes_deep = atoi(e) != 0;
    if (const char *e = tuning_knob("VBC_LANES_RDIV")) h->lanes_rdiv = std::max(1, atoi(e));
    if (const char *e = layout_knob("VBC_LANES_PAIR")) h->lanes_pair = atoi(e) != 0;
    if (const char *e = tuning_knob("VBC_SPLIT_KC")) h->split_kc = atoi(e) != 0;
    if (const char *e = tuning_knob("VBC_SPLIT_ROWS")) h->split_rows = std::max(1, atoi(e));
    if (const char *e = layout_knob("VBC_SMALL_FUSE")) h->small_fuse = atoi(e);
    if (const char *e = layout_knob("VBC_SIDE_FUSE")) h->side_fuse = atoi(e) < 0 ? -1 : atoi(e) != 0;
    if (const char *e = layout_knob("VBC_COLSPLIT")) h->colsplit = atoi(e) != 0;
    if (const char *e = tuning_knob("VBC_FUSE_PMAX")) h->fuse_pmax = atoi(e) >= 8 ? 8 : atoi(e) >= 4 ? 4 : 2;
    if (const char *e = tuning_knob("VBC_COLSPLIT_W")) h->colsplit_w = std::max(0, atoi(e));
    if (const char *e = tuning_knob("VBC_SPLIT_PIPE")) h->split_pipe = atoi(e);
    if (const char *e = tuning_knob("VBC_SMALL_ROWS")) h->small_rows = std::max(1, atoi(e));
    if (const char *e = layout_knob("VBC_KSPLIT")) h->ksplit = std::max(0.0, atof(e));
    if (const char *e = layout_knob("VBC_FWD_T")) h->fwd_t = atoi(e);
    if (const char *e = tuning_knob("VBC_SPLIT_DEEP")) h->split_deep = std::max(0.0, atof(e));
    if (const char *e = tuning_knob("VBC_SPLIT_NT_MB")) h->split_nt_bytes = (int64_t)(atof(e) * (1 << 20));
    if (const char *e = tuning_knob("VBC_FWD_MIN_ROWS")) h->fwd_min_rows = std::max(1, atoi(e));
    if (const char *e = tuning_knob("VBC_PLANAR_WPS")) h->planar_wps = h->planar_wps_pair = std::max(0, atoi(e));
    if (const char *e = tuning_knob("VBC_PLANAR_WPS_PAIR")) h->planar_wps_pair = std::max(0, atoi(e));
    if (const char *e = tuning_knob("VBC_SLOT_WONLY")) h->slot_wonly = atoi(e) != 0;
    h->target_ranges_p = prop.multiProcessorCount * h->occ_p * kWavesPerBlock;
    h->cus = std::max(1, prop.multiProcessorCount);
    for (int lp = 1; lp <= 3; lp++) h->occ_multi[lp] = occupancy_split_multi(h->esz, 1 << lp);
    if (const char *e = tuning_knob("VBC_TARGET_RANGES_P")) {
        h->target_ranges_p = std::max(1, atoi(e));
        h->occ_p = 1;
    }
    h->slot_u = h->esz == 8 ? 8 : 16;  // rows per step (measured on FE: 4 / 8 rows are 4-8 % slower)
    if (flags & (VBC_CREATE_MULTI | VBC_CREATE_MULTI_FORWARD)) {
        // (round 5: half as many ranges measured 195.5 against 206.5 us in tools/ab.py's interleaved graph replays,
        // but 213-216 against 208-210 us in bench.py's own C5 line, each setting in a fresh process --
        // profiles/r05zo_c5_ranges_ab.log; the bench decides, the count stays one round of resident waves)
        const int om = occupancy_panel(h->esz);
        h->target_ranges_m = prop.multiProcessorCount * std::max(1, std::min(om, 8)) * kWavesPerBlock;
        if (const char *e = tuning_knob("VBC_TARGET_RANGES_M")) h->target_ranges_m = std::max(1, atoi(e));
        if (const char *e = ablation_knob("VBC_PANEL_VALU")) h->panel_valu = atoi(e) != 0;
        if (const char *e = ablation_knob("VBC_PANEL_DIAG")) h->panel_valu |= atoi(e) & ~1;
        if (const char *e = tuning_knob("VBC_PANEL_NOBUF")) h->panel_nobuf = atoi(e) != 0;
        if (const char *e = layout_knob("VBC_PANEL_TILES")) h->panel_tiles = atoi(e) < 0 ? -1 : atoi(e) != 0;
        if (const char *e = tuning_knob("VBC_TILE_NBT")) h->tile_nbt = atoi(e) >= 8 ? 8 : 4;
        if (const char *e = tuning_knob("VBC_TILE_SPR")) h->tile_spr = std::max(1, atoi(e));
        if (const char *e = layout_knob("VBC_TILE_CLUSTER")) h->tile_cluster = atoi(e) == 2 ? 2 : atoi(e) != 0;
        if (const char *e = tuning_knob("VBC_TILE_DEPTH")) h->tile_depth = atoi(e) == 3 ? 3 : 2;
        h->occ_tiles = occupancy_tiles(h->esz);
    }

    Arena ar;
    std::vector<PendingBin> pt;
    std::vector<PendingSlot> st_t;
    std::vector<PendingSweep> sw_t;
    std::vector<std::vector<PendingBin>> pf;
    std::vector<std::vector<PendingSlot>> sf;
    std::vector<std::vector<PendingSweep>> wf;
    std::vector<PendingPanel> pm;
    std::vector<int32_t> fill_t, fill_f, fill_m;
    int st = VBC_OK;
    if (flags & VBC_CREATE_MULTI) {
        st = build_panel(h, s, v, ar, pm, h->lm, fill_m);
        h->has_m = st == VBC_OK;
        if (st == VBC_OK) {
            h->lm.nfill = (int)fill_m.size();
            h->lm.o_fill = ar.reserve(fill_m.size() * 4);
            std::memcpy(ar.at<int32_t>(h->lm.o_fill), fill_m.data(), fill_m.size() * 4);
        }
    }
    std::vector<PendingPanel> pmf;
    if (st == VBC_OK && (flags & VBC_CREATE_MULTI_FORWARD)) {
        st = build_forward_panel(h, s, v, ar, pmf, h->lmf);
        h->has_mf = st == VBC_OK;
        if (st == VBC_OK) h->lmf.o_fill = ar.reserve(4);
    }
    if (st == VBC_OK && (flags & VBC_CREATE_TRANSPOSED)) {
        st = build_transposed(h, s, v, ar, pt, st_t, sw_t, h->lt, fill_t);
        h->has_t = st == VBC_OK;
        if (st == VBC_OK) {
            h->lt.nfill = (int)fill_t.size();
            h->lt.o_fill = ar.reserve(fill_t.size() * 4);
            std::memcpy(ar.at<int32_t>(h->lt.o_fill), fill_t.data(), fill_t.size() * 4);
        }
    }
    std::vector<PendingBin> ptf;
    std::vector<PendingSlot> stf;
    std::vector<PendingSweep> swf;
    std::vector<int32_t> fill_tf;
    if (st == VBC_OK && (flags & VBC_CREATE_FORWARD) && fwd_via_t_wanted(h, s, flags)) {
        // small mixed-width forward product as the transposed product of C = Bᵀ (one fused launch instead
        // of a scale pass and one forward launch per width bucket, each adding into y)
        Stripes c;
        std::vector<char> cv;
        st = transpose_stripes(h, s, v, 8, c, cv);
        if (st == VBC_OK) {
            const int64_t bt = h->bytes_t;
            st = build_transposed(h, c, cv.data(), ar, ptf, stf, swf, h->lft, fill_tf);
            h->bytes_f = h->bytes_t - bt;
            h->bytes_t = bt;
        }
        if (st == VBC_OK) {
            h->has_f = h->has_ft = true;
            h->lft.nfill = (int)fill_tf.size();
            h->lft.o_fill = ar.reserve(fill_tf.size() * 4);
            std::memcpy(ar.at<int32_t>(h->lft.o_fill), fill_tf.data(), fill_tf.size() * 4);
        }
    } else if (st == VBC_OK && (flags & VBC_CREATE_FORWARD)) {
        st = build_forward(h, s, v, ar, pf, sf, wf, h->lf, fill_f);
        h->has_f = st == VBC_OK;
        if (st == VBC_OK) {
            if (h->lf.empty()) h->lf.emplace_back();  // no entries: the fill list alone writes y
            h->lf[0].nfill = (int)fill_f.size();
            h->lf[0].o_fill = ar.reserve(fill_f.size() * 4);
            std::memcpy(ar.at<int32_t>(h->lf[0].o_fill), fill_f.data(), fill_f.size() * 4);
        }
    }
    if (st != VBC_OK) { release(h); return st; }
    h->arena_bytes = std::max<size_t>(ar.host.size(), 256);
    if (hipMalloc(&h->d_arena, h->arena_bytes) != hipSuccess) {
        release(h);
        return fail(VBC_HIP_ERROR, "hipMalloc of the matrix arena failed");
    }
    if (!ar.host.empty() &&
        hipMemcpy(h->d_arena, ar.host.data(), ar.host.size(), hipMemcpyHostToDevice) != hipSuccess) {
        release(h);
        return fail(VBC_HIP_ERROR, "hipMemcpy of the matrix arena failed");
    }
    if (h->has_t && (st = finalize_launch(h, pt, st_t, h->lt, sw_t))) { release(h); return st; }
    if (h->has_ft && (st = finalize_launch(h, ptf, stf, h->lft, swf))) { release(h); return st; }
    for (Launch *lp : {&h->lt, &h->lft}) {  // side streams for the independent groups of a transposed launch
        Launch &Lx = *lp;
        if (!(lp == &h->lt ? h->has_t : h->has_ft) || !h->fork || launch_groups(Lx) < 2) continue;
        // no fork beside one dominant group when the others are more than a few waves of work: they are
        // latency-bound, and beside a launch that saturates HBM their dependent loads wait on a loaded
        // memory system while holding its wave slots (the ldoor stand-in's fp64 'min blocks': merge
        // kernel 131.5 us + fused side launch 11.5 us one after another, 160.3 / 88.7 us side by side;
        // 154 against 188 us per product, profiles/r04_bprof_*).  A side group of a few chunks still
        // forks (its one wave hides under the big launch).
        if ((int)Lx.gwork.size() == launch_groups(Lx)) {
            double tot = 0, big = 0;
            for (double wk : Lx.gwork) { tot += wk; big = std::max(big, wk); }
            if (big >= 0.9 * tot && tot - big > h->fork_side_bytes) continue;
        }
        const int ns = std::min(launch_groups(Lx) - 1, 3);
        for (int i = 0; i < ns; i++) {
            hipStream_t q = nullptr;
            if (hipStreamCreateWithFlags(&q, hipStreamNonBlocking) != hipSuccess) { release(h); return fail(VBC_HIP_ERROR, "hipStreamCreate failed"); }
            Lx.fork_streams.push_back(q);
        }
        for (int i = 0; i <= ns; i++) {
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) { release(h); return fail(VBC_HIP_ERROR, "hipEventCreate failed"); }
            Lx.fork_events.push_back(e);
        }
    }
    if (h->has_m && (st = finalize_panel(h, pm, h->lm))) { release(h); return st; }
    if (h->has_mf && (st = finalize_panel(h, pmf, h->lmf))) { release(h); return st; }
    for (size_t b = 0; b < pf.size(); b++)
        if ((st = finalize_launch(h, pf[b], sf[b], h->lf[b], wf[b]))) { release(h); return st; }
    if (h->has_f && !h->has_ft && pf.empty() && (st = finalize_launch(h, {}, {}, h->lf[0]))) { release(h); return st; }
    h->has_scratch = (h->has_t && !h->lt.bins.empty()) || (h->has_ft && !h->lft.bins.empty());
    for (const Launch &l : h->lf) h->has_scratch = h->has_scratch || (h->has_f && !l.bins.empty());
    *out = h;
    return VBC_OK;
}

}  // namespace vbc

using namespace vbc;

extern "C" {

static_assert(sizeof(vbc_info) == VBC_INFO_SIZE, "vbc_info layout changed: bump VBC_VERSION and VBC_INFO_SIZE");

int vbc_version(void) { return VBC_VERSION; }

int vbc_last_error(char *buf, size_t n)
{
    if (buf && n) {
        std::strncpy(buf, g_err.c_str(), n - 1);
        buf[n - 1] = 0;
    }
    return (int)g_err.size();
}

int vbc1d_create(vbc_handle **out, int64_t m, int64_t n, int64_t W, int64_t L, const int64_t *spl,
                 const int64_t *pos, const int64_t *idx, const int64_t *ofs, const void *val,
                 int64_t nval, int dtype, int device, unsigned flags)
{
    // SparseMatrix1DVBC{W,Tv,Ti} inner constructor checks (SparseMatrixVBCs.jl:45-50)
    if (m < 0) return fail(VBC_INVALID_ARG, "number of rows (m) must be >= 0");
    if (n < 0) return fail(VBC_INVALID_ARG, "number of columns (n) must be >= 0");
    if (W <= 0) return fail(VBC_INVALID_ARG, "W must be > 0");
    if (L < 0 || !spl || !pos || !ofs) return fail(VBC_INVALID_ARG, "bad stripe arrays");
    if (spl[0] != 1 || spl[L] != n + 1) return fail(VBC_INVALID_ARG, "Φ.spl must run from 1 to n+1");
    if (pos[0] != 1 || ofs[0] != 1) return fail(VBC_INVALID_ARG, "pos[1] and ofs[1] must be 1");
    Stripes s;
    s.m = m; s.n = n; s.L = L;
    s.col0.resize(L); s.w.resize(L); s.rbeg.resize(L + 1); s.voff.resize(L);
    const int64_t q = pos[L] - 1;
    if (q < 0 || (q > 0 && !idx)) return fail(VBC_INVALID_ARG, "bad pos");
    if (ofs[L] - 1 > nval) return fail(VBC_INVALID_ARG, "val shorter than ofs[L+1]-1");
    if (ofs[L] - 1 > 0 && !val) return fail(VBC_INVALID_ARG, "NULL val");
    for (int64_t l = 0; l < L; l++) {
        const int64_t w = spl[l + 1] - spl[l];
        if (w < 1) return fail(VBC_INVALID_ARG, "Φ.spl must be strictly increasing");
        if (w > W) return fail(VBC_ASSERTION, "AssertionError: w <= W");
        const int64_t R = pos[l + 1] - pos[l];
        if (R < 0) return fail(VBC_INVALID_ARG, "pos must be non-decreasing");
        if (ofs[l + 1] - ofs[l] != R * w) return fail(VBC_INVALID_ARG, "ofs[l+1]-ofs[l] != rows*w");
        s.col0[l] = spl[l] - 1;
        s.w[l] = (int32_t)w;
        s.rbeg[l] = pos[l] - 1;
        s.voff[l] = ofs[l] - 1;
    }
    s.rbeg[L] = q;
    s.rows.resize(q);
    for (int64_t r = 0; r < q; r++) {
        if (idx[r] < 1 || idx[r] > m) return fail(VBC_INVALID_ARG, "idx out of range 1:m");
        s.rows[r] = (int32_t)(idx[r] - 1);
    }
    return create_common(out, s, val, dtype, device, flags, ofs[L] - 1, 0, q);
}

int vbc2d_create(vbc_handle **out, int64_t m, int64_t n, int64_t U, int64_t W, int64_t K,
                 const int64_t *pspl, int64_t L, const int64_t *spl, const int64_t *pos,
                 const int64_t *idx, const int64_t *ofs, const void *val, int64_t nval, int dtype,
                 int device, unsigned flags)
{
    // SparseMatrixVBC{U,W,Tv,Ti} inner constructor checks (SparseMatrixVBCs.jl:72-79)
    if (m < 0) return fail(VBC_INVALID_ARG, "number of rows (m) must be >= 0");
    if (n < 0) return fail(VBC_INVALID_ARG, "number of columns (n) must be >= 0");
    if (U <= 0) return fail(VBC_INVALID_ARG, "U must be > 0");
    if (W <= 0) return fail(VBC_INVALID_ARG, "W must be > 0");
    if (K < 0 || L < 0 || !pspl || !spl || !pos || !ofs) return fail(VBC_INVALID_ARG, "bad partition arrays");
    if (pspl[0] != 1 || pspl[K] != m + 1) return fail(VBC_INVALID_ARG, "Π.spl must run from 1 to m+1");
    if (spl[0] != 1 || spl[L] != n + 1) return fail(VBC_INVALID_ARG, "Φ.spl must run from 1 to n+1");
    if (pos[0] != 1 || ofs[0] != 1) return fail(VBC_INVALID_ARG, "pos[1] and ofs[1] must be 1");
    for (int64_t k = 0; k < K; k++) {
        const int64_t u = pspl[k + 1] - pspl[k];
        if (u < 1) return fail(VBC_INVALID_ARG, "Π.spl must be strictly increasing");
        if (u > U) return fail(VBC_ASSERTION, "AssertionError: u <= U");
    }
    if (ofs[L] - 1 > nval) return fail(VBC_INVALID_ARG, "val shorter than ofs[L+1]-1");
    const int64_t q = pos[L] - 1;
    if (q < 0 || (q > 0 && !idx)) return fail(VBC_INVALID_ARG, "bad pos");
    for (int64_t l = 0; l < L; l++)  // every stripe's blocks lie inside idx[0 .. q-1]
        if (pos[l + 1] < pos[l] || pos[l] < 1 || pos[l + 1] - 1 > q)
            return fail(VBC_INVALID_ARG, "pos must be non-decreasing within 1:pos[L+1]");
    for (int64_t l = 0; l < L; l++)
        if (ofs[l + 1] < ofs[l]) return fail(VBC_INVALID_ARG, "ofs must be non-decreasing");
    if (ofs[L] - 1 > 0 && !val) return fail(VBC_INVALID_ARG, "NULL val");
    Stripes s;
    s.m = m; s.n = n; s.L = L;
    s.col0.resize(L); s.w.resize(L); s.rbeg.resize(L + 1); s.voff.resize(L);
    // Expand every u×w tile into u stored rows with explicit x-row indices: the tile is already
    // u row-major w-wide rows (constructors_VBC.jl:95-105), so val is used as is.
    int64_t rows = 0;
    for (int64_t l = 0; l < L; l++) {
        const int64_t w = spl[l + 1] - spl[l];
        if (w < 1) return fail(VBC_INVALID_ARG, "Φ.spl must be strictly increasing");
        if (w > W) return fail(VBC_ASSERTION, "AssertionError: w <= W");
        int64_t R = 0;
        for (int64_t Q = pos[l] - 1; Q < pos[l + 1] - 1; Q++) {
            const int64_t k = idx[Q];
            if (k < 1 || k > K) return fail(VBC_INVALID_ARG, "idx (block row) out of range 1:K");
            R += pspl[k] - pspl[k - 1];
        }
        if (ofs[l + 1] - ofs[l] != R * w) return fail(VBC_INVALID_ARG, "ofs[l+1]-ofs[l] != Σu*w");
        s.col0[l] = spl[l] - 1;
        s.w[l] = (int32_t)w;
        s.rbeg[l] = rows;
        s.voff[l] = ofs[l] - 1;
        rows += R;
    }
    s.rbeg[L] = rows;
    s.rows.resize(rows);
    int64_t r = 0;
    for (int64_t Q = 0; Q < q; Q++) {
        const int64_t k = idx[Q];
        for (int64_t i = pspl[k - 1] - 1; i < pspl[k] - 1; i++) s.rows[r++] = (int32_t)i;
    }
    s.grp.resize(K + 1);
    for (int64_t k = 0; k <= K; k++) s.grp[k] = pspl[k] - 1;
    return create_common(out, s, val, dtype, device, flags, ofs[L] - 1, K, q);
}

int vbc_csc_create(vbc_handle **out, int64_t m, int64_t n, const int64_t *colptr,
                   const int64_t *rowval, const void *nzval, int dtype, int device, unsigned flags)
{
    if (m < 0 || n < 0) return fail(VBC_INVALID_ARG, "number of rows/columns must be >= 0");
    if (!colptr || colptr[0] != 1) return fail(VBC_INVALID_ARG, "colptr[1] must be 1");
    Stripes s;
    s.m = m; s.n = n; s.L = n;
    s.col0.resize(n); s.w.assign(n, 1); s.rbeg.resize(n + 1); s.voff.resize(n);
    for (int64_t j = 0; j < n; j++) {
        if (colptr[j + 1] < colptr[j]) return fail(VBC_INVALID_ARG, "colptr must be non-decreasing");
        s.col0[j] = j;
        s.rbeg[j] = colptr[j] - 1;
        s.voff[j] = colptr[j] - 1;
    }
    const int64_t nnz = colptr[n] - 1;
    if (nnz > 0 && (!rowval || !nzval)) return fail(VBC_INVALID_ARG, "NULL rowval or nzval");
    s.rbeg[n] = nnz;
    s.rows.resize(nnz);
    for (int64_t p = 0; p < nnz; p++) {
        if (rowval[p] < 1 || rowval[p] > m) return fail(VBC_INVALID_ARG, "rowval out of range 1:m");
        s.rows[p] = (int32_t)(rowval[p] - 1);
    }
    // Column blocking: runs of up to 8 consecutive columns with identical row patterns (the dof
    // columns of a node in a stiffness matrix) become one w-wide stripe, so TrSpMV! runs the blocked
    // kernels (planar with row runs for 3-dof operators).  Each output y[j] still sums its column in
    // stored row order (TrSpMV.jl:10-16), so the result is that of the unit-width layout, bit for bit.
    // VBC_CSC_BLOCK=0 keeps unit stripes.
    const char *eb = layout_knob("VBC_CSC_BLOCK");
    if (!(eb && atoi(eb) == 0) && n > 1 && (dtype == VBC_F64 || dtype == VBC_F32 || dtype == VBC_I64)) {
        std::vector<int64_t> g0;  // first column of each group
        for (int64_t j = 0; j < n;) {
            int64_t e = j + 1;
            const int64_t len = colptr[j + 1] - colptr[j];
            while (e < n && e - j < 8 && colptr[e + 1] - colptr[e] == len &&
                   std::equal(rowval + colptr[j] - 1, rowval + colptr[j + 1] - 1, rowval + colptr[e] - 1))
                e++;
            g0.push_back(j);
            j = e;
        }
        if ((int64_t)g0.size() < n) {
            const int64_t L = (int64_t)g0.size();
            const int esz = elem_size(dtype);
            Stripes b;
            b.m = m; b.n = n; b.L = L;
            b.col0.resize(L); b.w.resize(L); b.rbeg.resize(L + 1); b.voff.resize(L);
            std::vector<char> bv((size_t)std::max<int64_t>(nnz, 1) * esz);
            const char *src = static_cast<const char *>(nzval);
            int64_t q = 0;
            for (int64_t l = 0; l < L; l++) {
                const int64_t j = g0[l], w = (l + 1 < L ? g0[l + 1] : n) - j, R = colptr[j + 1] - colptr[j];
                b.col0[l] = j;
                b.w[l] = (int32_t)w;
                b.rbeg[l] = q;
                q += R;
            }
            b.rbeg[L] = q;
            b.rows.resize(q);
            int64_t v = 0;
            for (int64_t l = 0; l < L; l++) {
                const int64_t j = g0[l], w = b.w[l], R = colptr[j + 1] - colptr[j];
                b.voff[l] = v;
                for (int64_t r = 0; r < R; r++) {
                    b.rows[b.rbeg[l] + r] = (int32_t)(rowval[colptr[j] - 1 + r] - 1);
                    for (int64_t c = 0; c < w; c++)
                        std::memcpy(bv.data() + (v + r * w + c) * esz, src + (colptr[j + c] - 1 + r) * esz, (size_t)esz);
                }
                v += R * w;
            }
            return create_common(out, b, bv.data(), dtype, device, flags, nnz, 0, q);
        }
    }
    return create_common(out, s, nzval, dtype, device, flags, nnz, 0, nnz);
}

int vbc_destroy(vbc_handle *h)
{
    release(h);
    return VBC_OK;
}

int vbc_get_info(const vbc_handle *h, vbc_info *info)
{
    if (!h || !info) return fail(VBC_INVALID_ARG, "NULL handle or info");
    std::memset(info, 0, sizeof(*info));
    info->m = h->m;
    info->n = h->n;
    info->L = h->L;
    info->K = h->K;
    info->nblocks = h->nblocks;
    info->nrows = h->nrows;
    info->nval = h->nval;
    info->nnz_hint = h->nnz;
    info->dtype = h->dtype;
    info->device = h->device;
    info->bins_t = h->has_t ? (int32_t)h->lt.bins.size() : 0;
    int32_t bf = 0;
    for (auto &l : h->lf) bf += (int32_t)l.bins.size();
    if (h->has_ft) bf += (int32_t)(h->lft.bins.size() + h->lft.sbins.size() + h->lft.pbins.size() + h->lft.wbins.size());
    info->bins_f = h->has_f ? bf : 0;
    if (h->has_ft) info->planar_mask |= 256;  // the forward product runs on the transposed layout of C = Bᵀ
    info->device_bytes = (int64_t)h->arena_bytes;
    info->bytes_t = h->bytes_t;
    info->bytes_f = h->bytes_f;
    info->bins_m = h->has_m ? (int32_t)(h->lm.bins.size() + h->lm.tbins.size())
                 : h->has_mf ? (int32_t)(h->lmf.bins.size() + h->lmf.tbins.size()) : 0;
    if ((h->has_m && !h->lm.tbins.empty()) || (h->has_mf && !h->lmf.tbins.empty()))
        info->planar_mask |= 512;  // multi-RHS buckets in the tile-granular layout (spmm_tiles)
    int32_t sl = h->has_t ? (int32_t)(h->lt.sbins.size() + h->lt.pbins.size()) : 0;  // planar bins are slotted too
    for (auto &l : h->lf) sl += h->has_f ? (int32_t)(l.sbins.size() + l.pbins.size()) : 0;  // + planar forward
    if (h->has_ft) sl += (int32_t)(h->lft.sbins.size() + h->lft.pbins.size());  // forward on C = Bᵀ's layout
    info->slot_bins = sl;
    int32_t sw = h->has_t ? (int32_t)h->lt.wbins.size() : 0;
    for (auto &l : h->lf) sw += h->has_f ? (int32_t)l.wbins.size() : 0;
    info->sweep_bins = sw;
    int32_t pl = h->has_t ? (int32_t)h->lt.pbins.size() : 0;
    info->planar_bins = pl;
    info->planar_run = 1;
    info->planar_split = 1;
    if (h->has_t)
        for (const auto &b : h->lt.pbins) {
            info->planar_run = std::max<int32_t>(info->planar_run, b.run);
            info->planar_split = std::max<int32_t>(info->planar_split, b.split);
            info->planar_pair = std::max<int32_t>(info->planar_pair, b.pair);
            info->planar_mask = std::max<int32_t>(info->planar_mask & 1, b.mask) | (info->planar_mask & ~1);
            if (b.lanes) info->planar_mask |= 4;
        }
    if (h->has_t && h->lt.fuse_split) info->planar_mask |= 32;  // the B'x planar bins run as one fused split launch
    if (h->has_t)
        for (const SlotBin &b : h->lt.pbins)
            if (b.ks > 1) info->planar_mask |= 64;  // long stripes cut into lane parts (SlotBin::ks)
    info->fwd_run = 1;
    if (h->has_f)
        for (const auto &l : h->lf)
            for (const auto &b : l.pbins) {
                info->fwd_run = std::max<int32_t>(info->fwd_run, b.lanes ? b.wkey : b.run);  // lanes: W = R rows
                if (b.mask && !b.lanes) info->planar_mask |= 2;
                if (b.split > 1) info->planar_mask |= 8;
                if (b.lanes) info->planar_mask |= 16;
                if (b.dot) info->planar_mask |= 2048;  // forward lane pairs (run_pair DOT)
            }
    if (h->has_ft)  // the forward product on C = Bᵀ: its split bins sum P slices too (bit 3, as a split forward)
        for (const SlotBin &b : h->lft.pbins)
            if (b.split > 1) info->planar_mask |= 8;
    info->bytes_m = h->has_m ? h->bytes_m : h->bytes_mf;  // a forward-only multi handle: its Bᵀ panel layout
    return VBC_OK;
}

static int check_mul(const vbc_handle *h, int trans, int64_t nx, int64_t ny, bool mat = false)
{
    if (!h) return fail(VBC_INVALID_ARG, "NULL handle");
    // DimensionMismatch checks: multiply_1DVBC.jl:44-45 (forward), :139-140 (transposed)
    const int64_t want_x = trans ? h->m : h->n, want_y = trans ? h->n : h->m;
    if (nx != want_x || ny != want_y) return fail(VBC_DIM_MISMATCH, "DimensionMismatch");
    if (trans && !h->has_t && !(mat && h->has_m))
        return fail(VBC_INVALID_ARG, mat ? "handle built without VBC_CREATE_TRANSPOSED or VBC_CREATE_MULTI"
                                         : "handle built without VBC_CREATE_TRANSPOSED");
    if (!trans && !h->has_f && !(mat && h->has_mf))
        return fail(VBC_INVALID_ARG, mat ? "handle built without VBC_CREATE_FORWARD or VBC_CREATE_MULTI_FORWARD"
                                         : "handle built without VBC_CREATE_FORWARD");
    return VBC_OK;
}

static void apply_quirks(int trans, unsigned flags, double &alpha, double &beta)
{
    if (!(flags & VBC_MUL_REFERENCE_QUIRKS)) return;
    alpha = 1.0;             // forward drops α; transposed overwrites y
    if (trans) beta = 0.0;
}

// Orders the products of a handle whose layout has shared scratch (vbc_handle::has_scratch):
// a product on a different stream than the previous one waits for that one's completion event.
// The caller holds h->mu from before begin() until after end().  Inside a stream capture the
// captured order is the stream's own, so the event chain is skipped.
struct ProductOrder {
    vbc_handle *h;
    hipStream_t s;
    bool active = false;
    bool force = false;  // the product uses the handle's staging buffers on the device path
    ProductOrder(vbc_handle *h_, hipStream_t s_, bool force_ = false) : h(h_), s(s_), force(force_) {}
    int begin()
    {
        if (!h->has_scratch && !force) return VBC_OK;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) != hipSuccess) return fail(VBC_HIP_ERROR, "hipStreamIsCapturing failed");
        if (cs != hipStreamCaptureStatusNone) return VBC_OK;
        active = true;
        if (h->order_valid && h->order_stream != s && hipStreamWaitEvent(s, h->order_ev, 0) != hipSuccess)
            return fail(VBC_HIP_ERROR, "hipStreamWaitEvent failed");
        return VBC_OK;
    }
    int end()
    {
        if (!active) return VBC_OK;
        if (hipEventRecord(h->order_ev, s) != hipSuccess) return fail(VBC_HIP_ERROR, "hipEventRecord failed");
        h->order_stream = s;
        h->order_valid = true;
        return VBC_OK;
    }
};

// Cached device staging buffer `which` (0: x / X, 1: y / Y) of at least `bytes` (caller holds h->mu).
static int stage_buffer(vbc_handle *h, int which, size_t bytes, void **out)
{
    bytes = std::max<size_t>(bytes, 256);
    if (h->stage_bytes[which] < bytes) {
        // every host-pointer call synchronises its stream before returning: the old buffer is idle
        const size_t grow = std::max(bytes, h->stage_bytes[which] + h->stage_bytes[which] / 2);
        if (h->d_stage[which]) (void)hipFree(h->d_stage[which]);
        h->d_stage[which] = nullptr;
        h->stage_bytes[which] = 0;
        if (hipMalloc(&h->d_stage[which], grow) != hipSuccess)
            return fail(VBC_HIP_ERROR, "hipMalloc of a staging buffer failed");
        h->stage_bytes[which] = grow;
    }
    *out = h->d_stage[which];
    return VBC_OK;
}

int vbc_mul(vbc_handle *h, int trans, const void *x, int64_t nx, void *y, int64_t ny, double alpha,
            double beta, int mem, void *stream, unsigned flags)
{
    if (int st = check_mul(h, trans, nx, ny)) return st;
    apply_quirks(trans, flags, alpha, beta);
    const int64_t esz = h->esz;
    if (ny > 0 && x == y) return fail(VBC_INVALID_ARG, "x and y must not alias");
    if ((nx > 0 && !x) || (ny > 0 && !y)) return fail(VBC_INVALID_ARG, "NULL x or y");
    if (mem != VBC_MEM_DEVICE && mem != VBC_MEM_HOST)
        return fail(VBC_INVALID_ARG, "mem must be VBC_MEM_DEVICE or VBC_MEM_HOST");
    DeviceGuard g(h->device);
    if (!g.ok) return fail(VBC_HIP_ERROR, "hipSetDevice failed");
    hipStream_t s = (hipStream_t)stream;
    if (mem == VBC_MEM_DEVICE) {
        if (!h->has_scratch) return mul_dispatch(h, trans, x, y, alpha, beta, s);  // lock-free: no shared state
        std::lock_guard<std::mutex> lk(h->mu);
        ProductOrder po(h, s);
        int st = po.begin();
        if (st == VBC_OK) st = mul_dispatch(h, trans, x, y, alpha, beta, s);
        if (st == VBC_OK) st = po.end();
        return st;
    }
    // Host pointers: stage through the handle's cached device buffers (no per-call allocation).
    std::lock_guard<std::mutex> lk(h->mu);
    void *dx = nullptr, *dy = nullptr;
    if (int st = stage_buffer(h, 0, nx * esz, &dx)) return st;
    if (int st = stage_buffer(h, 1, ny * esz, &dy)) return st;
    ProductOrder po(h, s);
    if (int st = po.begin()) return st;
    if (nx > 0 && hipMemcpyAsync(dx, x, nx * esz, hipMemcpyHostToDevice, s) != hipSuccess)
        return fail(VBC_HIP_ERROR, "staging copy of x failed");
    if (beta != 0.0 && ny > 0 && hipMemcpyAsync(dy, y, ny * esz, hipMemcpyHostToDevice, s) != hipSuccess)
        return fail(VBC_HIP_ERROR, "staging copy of y failed");
    if (int st = mul_dispatch(h, trans, dx, dy, alpha, beta, s)) return st;
    if (ny > 0 && hipMemcpyAsync(y, dy, ny * esz, hipMemcpyDeviceToHost, s) != hipSuccess)
        return fail(VBC_HIP_ERROR, "result copy failed");
    if (int st = po.end()) return st;
    if (hipStreamSynchronize(s) != hipSuccess) return fail(VBC_HIP_ERROR, "hipStreamSynchronize failed");
    return VBC_OK;
}

// 2D copy of `rows` rows of `width` bytes between pitched buffers (no-op when empty).
static bool copy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t rows,
                   hipMemcpyKind kind, hipStream_t s)
{
    if (width == 0 || rows == 0) return true;
    return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, kind, s) == hipSuccess;
}

static int mul_mat_device(vbc_handle *h, int trans, int64_t nrhs, const char *dX, int64_t ldx, int64_t nx,
                          char *dY, int64_t ldy, int64_t ny, double alpha, double beta, bool rowmajor,
                          hipStream_t s)
{
    const int64_t esz = h->esz;
    int st = VBC_OK;
    bool fused = rowmajor && trans && nrhs > 0 && h->n > 0 && h->has_t && h->dtype != VBC_I64;
    for (const Bin &b : h->lt.bins) fused = fused && b.wkey != 0;  // runtime-width buckets: per column
    fused = fused && h->lt.sbins.empty() && h->lt.wbins.empty() && h->lt.pbins.empty();  // the fused vector kernel reads the merge layout only
    if (trans ? (h->has_m && nrhs > 0 && h->n > 0) : (h->has_mf && nrhs > 0 && h->m > 0)) {  // matrix-core panels
        const int64_t sxr = rowmajor ? ldx : 1, sxc = rowmajor ? 1 : ldx;
        const int64_t syr = rowmajor ? ldy : 1, syc = rowmajor ? 1 : ldy;
        return mulmat_panel_any(h, trans, nrhs, dX, sxr, sxc, dY, syr, syc, alpha, beta, s);
    }
    if (fused) return mulmat_rowmajor(h, nrhs, dX, ldx, dY, ldy, alpha, beta, s);
    if (!rowmajor) {
        for (int64_t r = 0; r < nrhs && st == VBC_OK; r++)
            st = mul_dispatch(h, trans, dX + r * ldx * esz, dY + r * ldy * esz, alpha, beta, s);
        return st;
    }
    // row-major, per column through the handle's cached contiguous temporaries (strided 2D copies);
    // the caller holds h->mu, and the stream orders the columns -- no allocation, no synchronisation
    void *tx = nullptr, *ty = nullptr;
    if (int e = stage_buffer(h, 2, std::max<int64_t>(nx, 1) * esz, &tx)) return e;
    if (int e = stage_buffer(h, 3, std::max<int64_t>(ny, 1) * esz, &ty)) return e;
    for (int64_t r = 0; r < nrhs && st == VBC_OK; r++) {
        if (!copy2d(tx, esz, dX + r * esz, ldx * esz, esz, nx, hipMemcpyDeviceToDevice, s))
            st = fail(VBC_HIP_ERROR, "column gather failed");
        if (st == VBC_OK && beta != 0.0 && !copy2d(ty, esz, dY + r * esz, ldy * esz, esz, ny, hipMemcpyDeviceToDevice, s))
            st = fail(VBC_HIP_ERROR, "column gather failed");
        if (st == VBC_OK) st = mul_dispatch(h, trans, tx, ty, alpha, beta, s);
        if (st == VBC_OK && !copy2d(dY + r * esz, ldy * esz, ty, esz, esz, ny, hipMemcpyDeviceToDevice, s))
            st = fail(VBC_HIP_ERROR, "column scatter failed");
    }
    return st;
}

int vbc_mul_mat(vbc_handle *h, int trans, int64_t nrhs, const void *X, int64_t ldx, int64_t nx,
                void *Y, int64_t ldy, int64_t ny, double alpha, double beta, int mem, void *stream,
                unsigned flags)
{
    if (int st = check_mul(h, trans, nx, ny, true)) return st;
    const bool rowmajor = (flags & VBC_MAT_ROWMAJOR) != 0;
    if (nrhs < 0 || (!rowmajor && (ldx < std::max<int64_t>(nx, 1) || ldy < std::max<int64_t>(ny, 1))) ||
        (rowmajor && (ldx < std::max<int64_t>(nrhs, 1) || ldy < std::max<int64_t>(nrhs, 1))))
        return fail(VBC_INVALID_ARG, "bad nrhs / leading dimensions");
    if (X == Y && nrhs > 0) return fail(VBC_INVALID_ARG, "X and Y must not alias");
    if (nrhs > 0 && ((nx > 0 && !X) || (ny > 0 && !Y))) return fail(VBC_INVALID_ARG, "NULL X or Y");
    if (mem != VBC_MEM_DEVICE && mem != VBC_MEM_HOST)
        return fail(VBC_INVALID_ARG, "mem must be VBC_MEM_DEVICE or VBC_MEM_HOST");
    apply_quirks(trans, flags, alpha, beta);
    const int64_t esz = h->esz;
    DeviceGuard g(h->device);
    if (!g.ok) return fail(VBC_HIP_ERROR, "hipSetDevice failed");
    hipStream_t s = (hipStream_t)stream;
    std::lock_guard<std::mutex> lk(h->mu);  // the fused kernel's carry buffer and the staging buffers
    ProductOrder po(h, s, rowmajor);          // row-major per-column products share the column temporaries
    if (mem == VBC_MEM_DEVICE) {
        int st = po.begin();
        if (st == VBC_OK)
            st = mul_mat_device(h, trans, nrhs, static_cast<const char *>(X), ldx, nx, static_cast<char *>(Y), ldy,
                                ny, alpha, beta, rowmajor, s);
        if (st == VBC_OK) st = po.end();
        return st;
    }
    // Host operands: only the logical extent moves (pitched 2D copies into packed device buffers),
    // so the padding of a caller's view (ld > extent) is never read or written.
    const int64_t xr = rowmajor ? nx : nrhs, xw = rowmajor ? nrhs : nx;  // rows x row-width (elements)
    const int64_t yr = rowmajor ? ny : nrhs, yw = rowmajor ? nrhs : ny;
    void *sx = nullptr, *sy = nullptr;
    if (int st = stage_buffer(h, 0, xr * xw * esz, &sx)) return st;
    if (int st = stage_buffer(h, 1, yr * yw * esz, &sy)) return st;
    if (int st = po.begin()) return st;
    if (!copy2d(sx, xw * esz, X, ldx * esz, xw * esz, xr, hipMemcpyHostToDevice, s))
        return fail(VBC_HIP_ERROR, "staging copy of X failed");
    if (beta != 0.0 && !copy2d(sy, yw * esz, Y, ldy * esz, yw * esz, yr, hipMemcpyHostToDevice, s))
        return fail(VBC_HIP_ERROR, "staging copy of Y failed");
    if (int st = mul_mat_device(h, trans, nrhs, static_cast<const char *>(sx), std::max<int64_t>(xw, 1), nx,
                                static_cast<char *>(sy), std::max<int64_t>(yw, 1), ny, alpha, beta, rowmajor, s))
        return st;
    if (!copy2d(Y, ldy * esz, sy, yw * esz, yw * esz, yr, hipMemcpyDeviceToHost, s))
        return fail(VBC_HIP_ERROR, "result copy failed");
    if (int st = po.end()) return st;
    if (hipStreamSynchronize(s) != hipSuccess) return fail(VBC_HIP_ERROR, "hipStreamSynchronize failed");
    return VBC_OK;
}

// ---------------------------------------------------------------------------------------------
// Generic eltypes and index widths (vbc_types), strided operands
// ---------------------------------------------------------------------------------------------

extern "C++" {  // helpers of the typed entry points (templates need C++ linkage)
static bool is_float(int dt) { return dt == VBC_F64 || dt == VBC_F32; }
static bool known_dtype(int dt) { return dt >= VBC_F64 && dt <= VBC_BOOL; }

// Values converted to the compute eltype (empty when no conversion is needed: use `val` as is).
static int convert_values(const void *val, int64_t nval, const vbc_types *t, std::vector<char> &out)
{
    if (t->val_dtype == t->compute_dtype) return VBC_OK;
    if (nval > 0 && !val) return fail(VBC_INVALID_ARG, "NULL val");
    out.resize((size_t)std::max<int64_t>(nval, 1) * elem_size(t->compute_dtype));
    if (t->compute_dtype == VBC_F64) host_convert(val, t->val_dtype, nval, 1, reinterpret_cast<double *>(out.data()));
    else if (t->compute_dtype == VBC_F32) host_convert(val, t->val_dtype, nval, 1, reinterpret_cast<float *>(out.data()));
    else host_convert(val, t->val_dtype, nval, 1, reinterpret_cast<int64_t *>(out.data()));
    return VBC_OK;
}

static int check_types(const vbc_types *t)
{
    if (!t) return fail(VBC_INVALID_ARG, "NULL vbc_types");
    if (t->reserved != 0) return fail(VBC_INVALID_ARG, "vbc_types.reserved must be 0");
    if (t->index_bits != 32 && t->index_bits != 64) return fail(VBC_INVALID_ARG, "index_bits must be 32 or 64");
    if (!known_dtype(t->val_dtype)) return fail(VBC_UNSUPPORTED_DTYPE, "unknown val_dtype");
    if (t->compute_dtype != VBC_F64 && t->compute_dtype != VBC_F32 && t->compute_dtype != VBC_I64)
        return fail(VBC_UNSUPPORTED_DTYPE, "compute_dtype must be VBC_F64, VBC_F32 or VBC_I64");
    if (t->compute_dtype == VBC_I64 && is_float(t->val_dtype))
        return fail(VBC_UNSUPPORTED_DTYPE, "floating-point values on an integer handle (InexactError)");
    return VBC_OK;
}

// Index array as Int64 (a copy only for Ti = Int32).
struct Idx64 {
    std::vector<int64_t> buf;
    const int64_t *p = nullptr;
    void set(const void *src, int bits, int64_t n)
    {
        if (!src || bits == 64) {
            p = static_cast<const int64_t *>(src);
            return;
        }
        const int32_t *s32 = static_cast<const int32_t *>(src);
        buf.assign(s32, s32 + std::max<int64_t>(n, 0));
        p = buf.data();
    }
};

}  // extern "C++"

int vbc1d_create_ex(vbc_handle **out, int64_t m, int64_t n, int64_t W, int64_t L, const void *spl, const void *pos,
                    const void *idx, const void *ofs, const void *val, int64_t nval, const vbc_types *t, int device,
                    unsigned flags)
{
    if (int st = check_types(t)) return st;
    if (L < 0 || !spl || !pos || !ofs) return fail(VBC_INVALID_ARG, "bad stripe arrays");
    Idx64 S, P, I, O;
    S.set(spl, t->index_bits, L + 1);
    P.set(pos, t->index_bits, L + 1);
    O.set(ofs, t->index_bits, L + 1);
    const int64_t q = P.p[L] - 1;
    if (q < 0 || (q > 0 && !idx)) return fail(VBC_INVALID_ARG, "bad pos");
    I.set(idx, t->index_bits, q);
    std::vector<char> cv;
    if (int st = convert_values(val, nval, t, cv)) return st;
    return vbc1d_create(out, m, n, W, L, S.p, P.p, I.p, O.p, cv.empty() ? val : cv.data(), nval, t->compute_dtype,
                        device, flags);
}

int vbc2d_create_ex(vbc_handle **out, int64_t m, int64_t n, int64_t U, int64_t W, int64_t K, const void *pspl,
                    int64_t L, const void *spl, const void *pos, const void *idx, const void *ofs, const void *val,
                    int64_t nval, const vbc_types *t, int device, unsigned flags)
{
    if (int st = check_types(t)) return st;
    if (K < 0 || L < 0 || !pspl || !spl || !pos || !ofs) return fail(VBC_INVALID_ARG, "bad partition arrays");
    Idx64 PS, S, P, I, O;
    PS.set(pspl, t->index_bits, K + 1);
    S.set(spl, t->index_bits, L + 1);
    P.set(pos, t->index_bits, L + 1);
    O.set(ofs, t->index_bits, L + 1);
    const int64_t q = P.p[L] - 1;
    if (q < 0 || (q > 0 && !idx)) return fail(VBC_INVALID_ARG, "bad pos");
    I.set(idx, t->index_bits, q);
    std::vector<char> cv;
    if (int st = convert_values(val, nval, t, cv)) return st;
    return vbc2d_create(out, m, n, U, W, K, PS.p, L, S.p, P.p, I.p, O.p, cv.empty() ? val : cv.data(), nval,
                        t->compute_dtype, device, flags);
}

int vbc_csc_create_ex(vbc_handle **out, int64_t m, int64_t n, const void *colptr, const void *rowval,
                      const void *nzval, const vbc_types *t, int device, unsigned flags)
{
    if (int st = check_types(t)) return st;
    if (n < 0 || !colptr) return fail(VBC_INVALID_ARG, "colptr[1] must be 1");
    Idx64 CP, RV;
    CP.set(colptr, t->index_bits, n + 1);
    const int64_t nnz = CP.p[n] - 1;
    if (nnz < 0) return fail(VBC_INVALID_ARG, "bad colptr");
    RV.set(rowval, t->index_bits, nnz);
    std::vector<char> cv;
    if (int st = convert_values(nzval, nnz, t, cv)) return st;
    return vbc_csc_create(out, m, n, CP.p, RV.p, cv.empty() ? nzval : cv.data(), t->compute_dtype, device, flags);
}

int vbc_mul_ex(vbc_handle *h, int trans, const void *x, int x_dtype, int64_t incx, int64_t nx, void *y, int y_dtype,
               int64_t incy, int64_t ny, double alpha, double beta, int mem, void *stream, unsigned flags)
{
    if (int st = check_mul(h, trans, nx, ny)) return st;
    const int cdt = h->dtype;
    if (!known_dtype(x_dtype) || !known_dtype(y_dtype)) return fail(VBC_UNSUPPORTED_DTYPE, "unknown eltype");
    if (cdt == VBC_I64 && is_float(x_dtype))
        return fail(VBC_UNSUPPORTED_DTYPE, "floating-point x on an integer handle (InexactError)");
    if (is_float(cdt) ? y_dtype != cdt : (y_dtype != VBC_I64 && y_dtype != VBC_I32))
        return fail(VBC_UNSUPPORTED_DTYPE, "eltype(y) must be the handle's compute eltype (or Int32 on an Int64 handle)");
    if ((nx > 0 && incx == 0) || (ny > 0 && incy == 0)) return fail(VBC_INVALID_ARG, "zero stride");
    if ((nx > 0 && !x) || (ny > 0 && !y)) return fail(VBC_INVALID_ARG, "NULL x or y");
    if (cdt == VBC_I64 && (alpha != std::trunc(alpha) || beta != std::trunc(beta)))
        return fail(VBC_INVALID_ARG, "alpha and beta must be integers on an integer handle (InexactError)");
    if (mem != VBC_MEM_DEVICE && mem != VBC_MEM_HOST)
        return fail(VBC_INVALID_ARG, "mem must be VBC_MEM_DEVICE or VBC_MEM_HOST");
    const bool direct_x = x_dtype == cdt && (incx == 1 || nx <= 1);
    const bool direct_y = y_dtype == cdt && (incy == 1 || ny <= 1);
    if (direct_x && direct_y) return vbc_mul(h, trans, x, nx, y, ny, alpha, beta, mem, stream, flags);
    const int64_t esz = h->esz;
    if (mem == VBC_MEM_HOST) {  // convert on the host, then the contiguous host path
        std::vector<char> xs, ys((size_t)std::max<int64_t>(ny, 1) * esz);
        const void *xp = x;
        if (!direct_x) {
            xs.resize((size_t)std::max<int64_t>(nx, 1) * esz);
            host_convert_to(x, x_dtype, nx, incx, xs.data(), cdt);
            xp = xs.data();
        }
        if (beta != 0.0) host_convert_to(y, y_dtype, ny, incy, ys.data(), cdt);
        if (int st = vbc_mul(h, trans, xp, nx, ys.data(), ny, alpha, beta, mem, stream, flags)) return st;
        host_store(ys.data(), cdt, ny, y, y_dtype, incy);
        return VBC_OK;
    }
    // device operands: conversion kernels into / out of the handle's staging buffers
    apply_quirks(trans, flags, alpha, beta);
    DeviceGuard g(h->device);
    if (!g.ok) return fail(VBC_HIP_ERROR, "hipSetDevice failed");
    hipStream_t s = (hipStream_t)stream;
    std::lock_guard<std::mutex> lk(h->mu);
    ProductOrder po(h, s, true);
    void *dx = const_cast<void *>(x), *dy = y;
    if (!direct_x) {
        if (int st = stage_buffer(h, 0, nx * esz, &dx)) return st;
    }
    if (!direct_y) {
        if (int st = stage_buffer(h, 1, ny * esz, &dy)) return st;
    }
    if (int st = po.begin()) return st;
    if (!direct_x) {
        if (int st = convert_gather(x, x_dtype, incx, dx, cdt, nx, s)) return st;
    }
    if (!direct_y && beta != 0.0) {
        if (int st = convert_gather(y, y_dtype, incy, dy, cdt, ny, s)) return st;
    }
    if (int st = mul_dispatch(h, trans, dx, dy, alpha, beta, s)) return st;
    if (!direct_y) {
        if (int st = convert_scatter(dy, cdt, y, y_dtype, incy, ny, s)) return st;
    }
    return po.end();
}

int vbc_mul_mat_ex(vbc_handle *h, int trans, int64_t nrhs, const void *X, int X_dtype, int64_t ldx, int64_t nx,
                   void *Y, int Y_dtype, int64_t ldy, int64_t ny, double alpha, double beta, int mem, void *stream,
                   unsigned flags)
{
    if (!h) return fail(VBC_INVALID_ARG, "NULL handle");
    if (!known_dtype(X_dtype) || !known_dtype(Y_dtype)) return fail(VBC_UNSUPPORTED_DTYPE, "unknown eltype");
    if (X_dtype != h->dtype || Y_dtype != h->dtype)
        return fail(VBC_UNSUPPORTED_DTYPE, "the matrix product takes X and Y of the handle's compute eltype "
                                           "(other eltypes: vbc_mul_ex column by column)");
    return vbc_mul_mat(h, trans, nrhs, X, ldx, nx, Y, ldy, ny, alpha, beta, mem, stream, flags);
}

}  // extern "C"
