// libvbc device side: handle creation (reference layout -> binned HBM layout), product launches
// and the C ABI of include/vbc.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "vbc_internal.h"
#include "vbc_kernels.h"

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

#define VBC_HIP(call)                                                                             \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            set_error("%s failed: %s", #call, hipGetErrorString(e_));                             \
            return VBC_HIP_ERROR;                                                                 \
        }                                                                                         \
    } while (0)

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

constexpr int kGroupSizes[] = {4, 8, 16, 32, 64};

// Smallest lane group that covers `elems` values of a segment of width w in one pass.
static int choose_group(int esz, int w, int64_t elems)
{
    const int V = w <= 8 ? vec_elems(esz, w) : 1;
    const int LPR = w / V;
    for (int G : kGroupSizes) {
        if (G < LPR) continue;
        const int64_t per_pass = (int64_t)(G / LPR) * LPR * V;
        if (per_pass >= elems) return G;
    }
    return 64;
}

// One fused launch: a bin table (device) plus its host copy.
struct Launch {
    std::vector<Bin> bins;
    Bin *d_bins = nullptr;
    int total_vblocks = 0;
    int grid = 0;
};

// Host description of the input stripes, common to 1D, 2D (expanded) and CSC inputs.
struct Stripes {
    int64_t m = 0, n = 0, L = 0;
    std::vector<int64_t> col0;  // 0-based first column of stripe l
    std::vector<int32_t> w;     // width
    std::vector<int64_t> rbeg;  // L+1 prefix into rows
    std::vector<int32_t> rows;  // 0-based x row of each stored w-wide row
    std::vector<int64_t> voff;  // element offset of the stripe's first value in the input val
};

}  // namespace vbc

struct vbc_handle {
    int64_t m = 0, n = 0, L = 0, K = 0, nblocks = 0, nrows = 0, nval = 0, nnz = 0;
    int dtype = 0, esz = 8, device = 0;
    void *d_arena = nullptr;
    size_t arena_bytes = 0;
    bool has_t = false, has_f = false;
    vbc::Launch lt;                 // transposed product
    std::vector<vbc::Launch> lf;    // forward product: one launch per width bucket
    int64_t bytes_t = 0, bytes_f = 0;
    int grid_cap = 2048;
};

namespace vbc {

// Arena builder: reserves aligned regions, fills a host image, uploads once.
struct Arena {
    std::vector<char> host;
    size_t reserve(size_t bytes)
    {
        size_t off = (host.size() + 255) & ~size_t(255);
        host.resize(off + bytes);
        return off;
    }
    template <typename U>
    U *at(size_t off) { return reinterpret_cast<U *>(host.data() + off); }
};

struct PendingBin {
    Bin b;
    size_t o_rptr, o_out, o_idx, o_val;
};

static int check_limits(const Stripes &s)
{
    if (s.m >= (int64_t(1) << 31) || s.n >= (int64_t(1) << 31))
        return fail(VBC_INVALID_ARG, "m and n must be < 2^31 on the GPU path");
    for (int32_t w : s.w)
        if (w > 64) return fail(VBC_UNSUPPORTED_DTYPE, "stripe width > 64 is not supported on the GPU path");
    return VBC_OK;
}

// Transposed layout: segments = stripes, binned by (w, G).
static int build_transposed(vbc_handle *h, const Stripes &s, const char *val, Arena &ar,
                            std::vector<PendingBin> &out)
{
    const int esz = h->esz;
    std::map<std::pair<int, int>, std::vector<int64_t>> bins;  // (w, G) -> stripes
    for (int64_t l = 0; l < s.L; l++) {
        const int64_t R = s.rbeg[l + 1] - s.rbeg[l];
        bins[{s.w[l], choose_group(esz, s.w[l], R * s.w[l])}].push_back(l);
    }
    int vblock = 0;
    for (auto &kv : bins) {
        const int w = kv.first.first, G = kv.first.second;
        const std::vector<int64_t> &segs = kv.second;
        int64_t rows = 0;
        for (int64_t l : segs) rows += s.rbeg[l + 1] - s.rbeg[l];
        if (rows >= (int64_t(1) << 31) || (int64_t)segs.size() >= (int64_t(1) << 31))
            return fail(VBC_INVALID_ARG, "bin too large for int32 offsets");
        PendingBin pb{};
        pb.b.w = w;
        pb.b.G = G;
        pb.b.key = make_key(0, w <= 8 ? w : 0, G);
        pb.b.nseg = (int32_t)segs.size();
        const int per_vb = kWavesPerBlock * (64 / G);
        const int64_t nvb = ((int64_t)segs.size() + per_vb - 1) / per_vb;
        if ((int64_t)vblock + nvb >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "too many blocks");
        pb.b.vblock0 = vblock;
        pb.b.nvblock = (int32_t)nvb;
        vblock += (int)nvb;
        pb.o_rptr = ar.reserve((segs.size() + 1) * 4);
        pb.o_out = ar.reserve(segs.size() * 4);
        pb.o_idx = ar.reserve(rows * 4);
        pb.o_val = ar.reserve(rows * w * esz);
        int32_t *rptr = ar.at<int32_t>(pb.o_rptr);
        int32_t *o = ar.at<int32_t>(pb.o_out);
        int32_t *ix = ar.at<int32_t>(pb.o_idx);
        char *vv = ar.at<char>(pb.o_val);
        int64_t r = 0;
        for (size_t q = 0; q < segs.size(); q++) {
            const int64_t l = segs[q];
            const int64_t R = s.rbeg[l + 1] - s.rbeg[l];
            rptr[q] = (int32_t)r;
            o[q] = (int32_t)s.col0[l];
            std::memcpy(ix + r, s.rows.data() + s.rbeg[l], R * 4);
            std::memcpy(vv + r * w * esz, val + s.voff[l] * esz, R * w * esz);
            r += R;
        }
        rptr[segs.size()] = (int32_t)r;
        h->bytes_t += (int64_t)(segs.size() + 1) * 4 + (int64_t)segs.size() * 4 + rows * 4 + rows * w * esz;
        out.push_back(pb);
    }
    h->bytes_t += (s.m + s.n) * esz;  // x read once, y written once
    return VBC_OK;
}

// Forward layout: per width bucket, segments = output rows, entries ordered by stripe.
static int build_forward(vbc_handle *h, const Stripes &s, const char *val, Arena &ar,
                         std::vector<std::vector<PendingBin>> &out)
{
    const int esz = h->esz;
    std::map<int, std::vector<int64_t>> buckets;  // w -> stripes
    for (int64_t l = 0; l < s.L; l++) buckets[s.w[l]].push_back(l);
    if (buckets.empty()) buckets[1];  // still need one launch to apply beta to y
    bool first = true;
    std::vector<int64_t> cnt(s.m), cur(s.m);
    for (auto &kv : buckets) {
        const int w = kv.first;
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int64_t l : kv.second)
            for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++) cnt[s.rows[r]]++;
        // segments per G
        std::map<int, std::vector<int64_t>> groups;
        for (int64_t i = 0; i < s.m; i++)
            if (cnt[i] > 0 || first) groups[choose_group(esz, w, cnt[i] * w)].push_back(i);
        std::vector<PendingBin> launch;
        int vblock = 0;
        for (auto &gv : groups) {
            const int G = gv.first;
            const std::vector<int64_t> &segs = gv.second;
            int64_t ents = 0;
            for (int64_t i : segs) ents += cnt[i];
            if (ents >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "bin too large for int32 offsets");
            PendingBin pb{};
            pb.b.w = w;
            pb.b.G = G;
            pb.b.key = make_key(1, w <= 8 ? w : 0, G);
            pb.b.nseg = (int32_t)segs.size();
            const int per_vb = kWavesPerBlock * (64 / G);
            const int64_t nvb = ((int64_t)segs.size() + per_vb - 1) / per_vb;
            if ((int64_t)vblock + nvb >= (int64_t(1) << 31)) return fail(VBC_INVALID_ARG, "too many blocks");
            pb.b.vblock0 = vblock;
            pb.b.nvblock = (int32_t)nvb;
            vblock += (int)nvb;
            pb.o_rptr = ar.reserve((segs.size() + 1) * 4);
            pb.o_out = ar.reserve(segs.size() * 4);
            pb.o_idx = ar.reserve(ents * 4);
            pb.o_val = ar.reserve(ents * w * esz);
            int32_t *rptr = ar.at<int32_t>(pb.o_rptr);
            int32_t *o = ar.at<int32_t>(pb.o_out);
            int64_t e = 0;
            for (size_t q = 0; q < segs.size(); q++) {
                rptr[q] = (int32_t)e;
                o[q] = (int32_t)segs[q];
                cur[segs[q]] = e;  // write cursor of row segs[q] within this bin
                e += cnt[segs[q]];
            }
            rptr[segs.size()] = (int32_t)e;
            h->bytes_f += (int64_t)(segs.size() + 1) * 4 + (int64_t)segs.size() * 4 + ents * 4 + ents * w * esz;
            h->bytes_f += (int64_t)segs.size() * esz * (first ? 1 : 2);  // y write (+ read when accumulating)
            launch.push_back(pb);
        }
        // scatter entries into their row segments, stripe-ascending
        std::vector<int> bin_of(s.m, -1);
        for (size_t bi = 0; bi < launch.size(); bi++) {
            const int32_t *o = ar.at<int32_t>(launch[bi].o_out);
            for (int32_t q = 0; q < launch[bi].b.nseg; q++) bin_of[o[q]] = (int)bi;
        }
        for (int64_t l : kv.second) {
            for (int64_t r = s.rbeg[l]; r < s.rbeg[l + 1]; r++) {
                const int64_t i = s.rows[r];
                PendingBin &pb = launch[bin_of[i]];
                const int64_t e = cur[i]++;
                ar.at<int32_t>(pb.o_idx)[e] = (int32_t)s.col0[l];
                std::memcpy(ar.at<char>(pb.o_val) + e * w * esz,
                            val + (s.voff[l] + (r - s.rbeg[l]) * w) * esz, (size_t)w * esz);
            }
        }
        h->bytes_f += s.n * esz;  // x slices (read once, ideally)
        out.push_back(std::move(launch));
        first = false;
    }
    return VBC_OK;
}

static int finalize_launch(vbc_handle *h, const std::vector<PendingBin> &pbs, Launch &L)
{
    L.bins.clear();
    for (const PendingBin &pb : pbs) {
        Bin b = pb.b;
        char *base = static_cast<char *>(h->d_arena);
        b.rptr = reinterpret_cast<const int32_t *>(base + pb.o_rptr);
        b.out = reinterpret_cast<const int32_t *>(base + pb.o_out);
        b.idx = reinterpret_cast<const int32_t *>(base + pb.o_idx);
        b.val = base + pb.o_val;
        L.bins.push_back(b);
    }
    L.total_vblocks = 0;
    for (const Bin &b : L.bins) L.total_vblocks = std::max(L.total_vblocks, b.vblock0 + b.nvblock);
    L.grid = std::max(1, std::min(L.total_vblocks, h->grid_cap));
    if (!L.bins.empty()) {
        VBC_HIP(hipMalloc(&L.d_bins, L.bins.size() * sizeof(Bin)));
        VBC_HIP(hipMemcpy(L.d_bins, L.bins.data(), L.bins.size() * sizeof(Bin), hipMemcpyHostToDevice));
    }
    return VBC_OK;
}

static void release(vbc_handle *h)
{
    if (!h) return;
    DeviceGuard g(h->device);
    if (h->lt.d_bins) (void)hipFree(h->lt.d_bins);
    for (auto &l : h->lf)
        if (l.d_bins) (void)hipFree(l.d_bins);
    if (h->d_arena) (void)hipFree(h->d_arena);
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

static int create_common(vbc_handle **out, Stripes &s, const void *val, int dtype, int device,
                         unsigned flags, int64_t nval, int64_t K, int64_t nblocks)
{
    if (!out) return fail(VBC_INVALID_ARG, "out handle pointer is NULL");
    *out = nullptr;
    if (dtype != VBC_F64 && dtype != VBC_F32)
        return fail(VBC_UNSUPPORTED_DTYPE, "GPU path supports Float64 and Float32 eltypes");
    if (int st = check_limits(s)) return st;
    int ndev = 0;
    VBC_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(VBC_INVALID_ARG, "device ordinal out of range");
    if ((flags & (VBC_CREATE_TRANSPOSED | VBC_CREATE_FORWARD)) == 0) flags |= VBC_CREATE_TRANSPOSED;

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
    h->nnz = dtype == VBC_F64 ? count_nonzeros<double>(v, nval) : count_nonzeros<float>(v, nval);

    DeviceGuard g(device);
    if (!g.ok) { release(h); return fail(VBC_HIP_ERROR, "hipSetDevice failed"); }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { release(h); return fail(VBC_HIP_ERROR, "hipGetDeviceProperties failed"); }
    int occ = 0;
    if (dtype == VBC_F64)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_bins<double, 0>, kBlockThreads, 0);
    else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spmv_bins<float, 0>, kBlockThreads, 0);
    h->grid_cap = prop.multiProcessorCount * std::max(1, std::min(occ, 8));

    Arena ar;
    std::vector<PendingBin> pt;
    std::vector<std::vector<PendingBin>> pf;
    int st = VBC_OK;
    if (flags & VBC_CREATE_TRANSPOSED) {
        st = build_transposed(h, s, v, ar, pt);
        h->has_t = st == VBC_OK;
    }
    if (st == VBC_OK && (flags & VBC_CREATE_FORWARD)) {
        st = build_forward(h, s, v, ar, pf);
        h->has_f = st == VBC_OK;
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
    if (h->has_t && (st = finalize_launch(h, pt, h->lt))) { release(h); return st; }
    for (auto &p : pf) {
        h->lf.emplace_back();
        if ((st = finalize_launch(h, p, h->lf.back()))) { release(h); return st; }
    }
    *out = h;
    return VBC_OK;
}

template <typename T>
static int launch(const vbc_handle *h, const Launch &L, int kind, const void *x, void *y, double alpha,
                  double beta, bool rd, hipStream_t stream)
{
    if (L.bins.empty() || L.total_vblocks == 0) return VBC_OK;
    if (kind == 0)
        hipLaunchKernelGGL((spmv_bins<T, 0>), dim3(L.grid), dim3(kBlockThreads), 0, stream, L.d_bins,
                           (int)L.bins.size(), L.total_vblocks, static_cast<const T *>(x),
                           static_cast<T *>(y), (T)alpha, (T)beta, (int)rd);
    else
        hipLaunchKernelGGL((spmv_bins<T, 1>), dim3(L.grid), dim3(kBlockThreads), 0, stream, L.d_bins,
                           (int)L.bins.size(), L.total_vblocks, static_cast<const T *>(x),
                           static_cast<T *>(y), (T)alpha, (T)beta, (int)rd);
    VBC_HIP(hipGetLastError());
    (void)h;
    return VBC_OK;
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
    for (size_t b = 0; b < h->lf.size(); b++) {
        const bool first = b == 0;
        if (int st = launch<T>(h, h->lf[b], 1, x, y, alpha, first ? beta : 1.0,
                               first ? beta != 0.0 : true, stream))
            return st;
    }
    return VBC_OK;
}

static int mul_dispatch(const vbc_handle *h, int trans, const void *x, void *y, double alpha,
                        double beta, hipStream_t stream)
{
    return h->dtype == VBC_F64 ? mul_device<double>(h, trans, x, y, alpha, beta, stream)
                               : mul_device<float>(h, trans, x, y, alpha, beta, stream);
}

}  // namespace vbc

using namespace vbc;

extern "C" {

int vbc_version(void) { return 100; }

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
    s.rbeg[n] = nnz;
    s.rows.resize(nnz);
    for (int64_t p = 0; p < nnz; p++) {
        if (rowval[p] < 1 || rowval[p] > m) return fail(VBC_INVALID_ARG, "rowval out of range 1:m");
        s.rows[p] = (int32_t)(rowval[p] - 1);
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
    info->bins_f = h->has_f ? bf : 0;
    info->device_bytes = (int64_t)h->arena_bytes;
    info->bytes_t = h->bytes_t;
    info->bytes_f = h->bytes_f;
    return VBC_OK;
}

static int check_mul(const vbc_handle *h, int trans, int64_t nx, int64_t ny)
{
    if (!h) return fail(VBC_INVALID_ARG, "NULL handle");
    // DimensionMismatch checks: multiply_1DVBC.jl:44-45 (forward), :139-140 (transposed)
    const int64_t want_x = trans ? h->m : h->n, want_y = trans ? h->n : h->m;
    if (nx != want_x || ny != want_y) return fail(VBC_DIM_MISMATCH, "DimensionMismatch");
    if (trans && !h->has_t) return fail(VBC_INVALID_ARG, "handle built without VBC_CREATE_TRANSPOSED");
    if (!trans && !h->has_f) return fail(VBC_INVALID_ARG, "handle built without VBC_CREATE_FORWARD");
    return VBC_OK;
}

static void apply_quirks(int trans, unsigned flags, double &alpha, double &beta)
{
    if (!(flags & VBC_MUL_REFERENCE_QUIRKS)) return;
    alpha = 1.0;             // forward drops α; transposed overwrites y
    if (trans) beta = 0.0;
}

int vbc_mul(vbc_handle *h, int trans, const void *x, int64_t nx, void *y, int64_t ny, double alpha,
            double beta, int mem, void *stream, unsigned flags)
{
    if (int st = check_mul(h, trans, nx, ny)) return st;
    apply_quirks(trans, flags, alpha, beta);
    const int64_t esz = h->esz;
    if (ny > 0 && x == y) return fail(VBC_INVALID_ARG, "x and y must not alias");
    DeviceGuard g(h->device);
    if (!g.ok) return fail(VBC_HIP_ERROR, "hipSetDevice failed");
    if (mem == VBC_MEM_DEVICE) return mul_dispatch(h, trans, x, y, alpha, beta, (hipStream_t)stream);
    if (mem != VBC_MEM_HOST) return fail(VBC_INVALID_ARG, "mem must be VBC_MEM_DEVICE or VBC_MEM_HOST");
    void *dx = nullptr, *dy = nullptr;
    int st = VBC_OK;
    hipStream_t s = (hipStream_t)stream;
    if (hipMalloc(&dx, std::max<int64_t>(nx, 1) * esz) != hipSuccess ||
        hipMalloc(&dy, std::max<int64_t>(ny, 1) * esz) != hipSuccess) {
        st = fail(VBC_HIP_ERROR, "hipMalloc of staging buffers failed");
    } else if (hipMemcpyAsync(dx, x, nx * esz, hipMemcpyHostToDevice, s) != hipSuccess ||
               (beta != 0.0 && hipMemcpyAsync(dy, y, ny * esz, hipMemcpyHostToDevice, s) != hipSuccess)) {
        st = fail(VBC_HIP_ERROR, "staging copy failed");
    } else if ((st = mul_dispatch(h, trans, dx, dy, alpha, beta, s)) == VBC_OK) {
        if (hipMemcpyAsync(y, dy, ny * esz, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            st = fail(VBC_HIP_ERROR, "result copy failed");
    }
    if (dx) (void)hipFree(dx);
    if (dy) (void)hipFree(dy);
    return st;
}

int vbc_mul_mat(vbc_handle *h, int trans, int64_t nrhs, const void *X, int64_t ldx, int64_t nx,
                void *Y, int64_t ldy, int64_t ny, double alpha, double beta, int mem, void *stream,
                unsigned flags)
{
    if (int st = check_mul(h, trans, nx, ny)) return st;
    if (nrhs < 0 || ldx < std::max<int64_t>(nx, 1) || ldy < std::max<int64_t>(ny, 1))
        return fail(VBC_INVALID_ARG, "bad nrhs / leading dimensions");
    apply_quirks(trans, flags, alpha, beta);
    const int64_t esz = h->esz;
    DeviceGuard g(h->device);
    if (!g.ok) return fail(VBC_HIP_ERROR, "hipSetDevice failed");
    hipStream_t s = (hipStream_t)stream;
    const char *dX = static_cast<const char *>(X);
    char *dY = static_cast<char *>(Y);
    void *sx = nullptr, *sy = nullptr;
    if (mem == VBC_MEM_HOST) {
        if (hipMalloc(&sx, std::max<int64_t>(ldx * nrhs, 1) * esz) != hipSuccess ||
            hipMalloc(&sy, std::max<int64_t>(ldy * nrhs, 1) * esz) != hipSuccess) {
            if (sx) (void)hipFree(sx);
            return fail(VBC_HIP_ERROR, "hipMalloc of staging buffers failed");
        }
        (void)hipMemcpyAsync(sx, X, ldx * nrhs * esz, hipMemcpyHostToDevice, s);
        if (beta != 0.0) (void)hipMemcpyAsync(sy, Y, ldy * nrhs * esz, hipMemcpyHostToDevice, s);
        dX = static_cast<const char *>(sx);
        dY = static_cast<char *>(sy);
    } else if (mem != VBC_MEM_DEVICE) {
        return fail(VBC_INVALID_ARG, "mem must be VBC_MEM_DEVICE or VBC_MEM_HOST");
    }
    int st = VBC_OK;
    for (int64_t r = 0; r < nrhs && st == VBC_OK; r++)
        st = mul_dispatch(h, trans, dX + r * ldx * esz, dY + r * ldy * esz, alpha, beta, s);
    if (mem == VBC_MEM_HOST) {
        if (st == VBC_OK && (hipMemcpyAsync(Y, sy, ldy * nrhs * esz, hipMemcpyDeviceToHost, s) != hipSuccess ||
                             hipStreamSynchronize(s) != hipSuccess))
            st = fail(VBC_HIP_ERROR, "result copy failed");
        (void)hipFree(sx);
        (void)hipFree(sy);
    }
    return st;
}

}  // extern "C"
