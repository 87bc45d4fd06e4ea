// libvbc multi-GPU handles (include/vbc.h: vbc1d_create_sharded, vbc_sharded_mul): ONE process
// driving several GPUs of a node -- the configuration a Julia session with AMDGPU.jl has -- with RCCL
// over xGMI for the exchange steps.  (One process per GPU with torch.distributed is the other
// configuration; sparsematrixvbcs.jl_amd/distributed.py builds it on top of the single-GPU handles.)
//
// The reference's only parallel region is the threaded stripe loop of the transposed product
// (multiply_1DVBC.jl:169-177); here the matrix is cut into contiguous ranges balanced by HBM bytes,
// one libvbc handle per GPU:
//   VBC_SPLIT_STRIPES  shard g = stripes [l_g, l_g+1) = columns [c_g, c_g+1) of B
//       B'x: x replicated (ncclBroadcast from the root), y[c_g : c_g+1) written by GPU g and sent to
//            the root's y (ncclSend / ncclRecv) -- no reduction;
//       B x: x[c_g : c_g+1) sent to GPU g, partial y on every GPU, ncclReduce(sum) into the root's y.
//   VBC_SPLIT_ROWS     shard g = the stored rows [r_g, r_g+1) of every stripe (stored order kept, so
//                      each stripe's summation order is the reference's)
//       B x: x replicated, y[r_g : r_g+1) per GPU, gathered on the root -- no reduction;
//       B'x: x[r_g : r_g+1) per GPU, partial y, ncclReduce(sum).
// Disjoint outputs are bit-identical to the single-GPU product; reduced ones differ only in the
// order the partial sums are added.
//
// When every shard is on the SAME device (devices = {d, d, ...}: oversubscription, or the tests of a
// one-GPU box) the exchange needs no communication at all: shards read x and write y through pointer
// offsets on that device, and reduced outputs accumulate shard after shard (β = 1) on the caller's
// stream.  RCCL refuses two ranks on one GPU, so that mode never creates communicators.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "vbc_internal.h"

using vbc::fail;

struct vbc_sharded {
    int64_t m = 0, n = 0;
    int ngpus = 0, split = 0, cdt = 0, esz = 8;
    bool local = false;              // all shards on one device: no communicators
    std::vector<int> dev;
    std::vector<vbc_handle *> h;
    std::vector<int64_t> cut;        // ngpus+1 0-based cuts of the split dimension (columns or rows)
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> st;     // per shard: internal stream (root: host-pointer products only)
    std::vector<hipEvent_t> done;    // per shard: end of its part of a product
    hipEvent_t start = nullptr;      // root stream: start of a product
    std::vector<void *> xb, yb;      // per non-root shard: x / y buffers (max(m, n) elements each)
    void *hx = nullptr, *hy = nullptr;  // root: host-pointer staging
    std::mutex mu;                   // products are issued one at a time (collective order, buffers)
};

namespace {

struct DevGuard {
    int prev = -1;
    bool ok = false;
    explicit DevGuard(int d)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(d) == hipSuccess;
    }
    ~DevGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int nccl_fail(ncclResult_t r, const char *what)
{
    vbc::set_error("%s failed: %s", what, ncclGetErrorString(r));
    return VBC_RCCL_ERROR;
}

#define VBC_NCCL(call)                                                                            \
    do {                                                                                          \
        ncclResult_t r_ = (call);                                                                 \
        if (r_ != ncclSuccess) return nccl_fail(r_, #call);                                       \
    } while (0)
#define VBC_HIPS(call)                                                                            \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            vbc::set_error("%s failed: %s", #call, hipGetErrorString(e_));                        \
            return VBC_HIP_ERROR;                                                                 \
        }                                                                                         \
    } while (0)

ncclDataType_t nccl_type(int cdt)
{
    return cdt == VBC_F64 ? ncclFloat64 : cdt == VBC_F32 ? ncclFloat32 : ncclInt64;
}

std::vector<int64_t> as64(const void *p, int bits, int64_t n)
{
    std::vector<int64_t> v((size_t)std::max<int64_t>(n, 0));
    if (bits == 64) std::memcpy(v.data(), p, v.size() * 8);
    else
        for (size_t i = 0; i < v.size(); i++) v[i] = static_cast<const int32_t *>(p)[i];
    return v;
}

// Cuts 0 = k_0 <= ... <= k_parts = N of a prefix-summed cost (N+1 entries) into parts of equal cost:
// k_p = first index whose prefix reaches p/parts of the total (distributed.py stripe_split / row_split).
std::vector<int64_t> balanced_cuts(const std::vector<double> &cost, int parts)
{
    const int64_t N = (int64_t)cost.size() - 1;
    std::vector<int64_t> k(parts + 1, 0);
    k[parts] = N;
    for (int p = 1; p < parts; p++) {
        const double target = cost[N] * (double)p / (double)parts;
        int64_t c = std::lower_bound(cost.begin(), cost.end(), target) - cost.begin();
        k[p] = std::max(k[p - 1], std::min(c, N));
    }
    return k;
}

// The product's exchange pattern: disjoint y slices (x replicated) or partial y (x sliced) + reduce.
bool disjoint_output(int split, int trans) { return (split == VBC_SPLIT_STRIPES) == (trans != 0); }

void destroy_all(vbc_sharded *s)
{
    for (size_t g = 0; g < s->st.size(); g++) {
        DevGuard dg(s->dev[g]);
        if (s->st[g]) (void)hipStreamSynchronize(s->st[g]);
    }
    for (ncclComm_t c : s->comm)
        if (c) (void)ncclCommDestroy(c);
    for (size_t g = 0; g < s->dev.size(); g++) {
        DevGuard dg(s->dev[g]);
        if (g < s->xb.size() && s->xb[g]) (void)hipFree(s->xb[g]);
        if (g < s->yb.size() && s->yb[g]) (void)hipFree(s->yb[g]);
        if (g < s->done.size() && s->done[g]) (void)hipEventDestroy(s->done[g]);
        if (g < s->st.size() && s->st[g]) (void)hipStreamDestroy(s->st[g]);
        if (g == 0) {
            if (s->start) (void)hipEventDestroy(s->start);
            if (s->hx) (void)hipFree(s->hx);
            if (s->hy) (void)hipFree(s->hy);
        }
    }
    for (vbc_handle *h : s->h)
        if (h) (void)vbc_destroy(h);
    delete s;
}

// One product on device operands of the root (devices[0]), enqueued on the root stream s0.
int mul_device(vbc_sharded *s, int trans, const char *x, int64_t nx, char *y, int64_t ny, double alpha,
               double beta, hipStream_t s0)
{
    const int G = s->ngpus;
    const int64_t esz = s->esz;
    const bool disj = disjoint_output(s->split, trans);
    auto lo = [&](int g) { return s->cut[g]; };
    auto len = [&](int g) { return s->cut[g + 1] - s->cut[g]; };
    if (s->local) {  // every shard on the root's device: pointer offsets, one stream
        for (int g = 0; g < G; g++) {
            int st;
            if (disj) st = vbc_mul(s->h[g], trans, x, nx, y + lo(g) * esz, len(g), alpha, beta, VBC_MEM_DEVICE, s0, 0);
            else st = vbc_mul(s->h[g], trans, x + lo(g) * esz, len(g), y, ny, alpha, g == 0 ? beta : 1.0,
                              VBC_MEM_DEVICE, s0, 0);
            if (st) return st;
        }
        return VBC_OK;
    }
    const ncclDataType_t dt = nccl_type(s->cdt);
    {
        DevGuard dg(s->dev[0]);
        VBC_HIPS(hipEventRecord(s->start, s0));
    }
    for (int g = 1; g < G; g++) {
        DevGuard dg(s->dev[g]);
        VBC_HIPS(hipStreamWaitEvent(s->st[g], s->start, 0));
    }
    auto stream = [&](int g) { return g == 0 ? s0 : s->st[g]; };
    // 1. x to the shards: broadcast (replicated x) or one slice each
    if (!s->comm.empty()) {
        VBC_NCCL(ncclGroupStart());
        for (int g = 0; g < G; g++) {
            if (disj) {
                VBC_NCCL(ncclBroadcast(x, g == 0 ? (void *)x : s->xb[g], (size_t)nx, dt, 0, s->comm[g], stream(g)));
            } else if (g > 0 && len(g) > 0) {
                VBC_NCCL(ncclSend(x + lo(g) * esz, (size_t)len(g), dt, g, s->comm[0], s0));
                VBC_NCCL(ncclRecv(s->xb[g], (size_t)len(g), dt, 0, s->comm[g], s->st[g]));
            }
        }
        VBC_NCCL(ncclGroupEnd());
        // β y of a disjoint slice lives on the root: send it to its shard first
        if (disj && beta != 0.0) {
            VBC_NCCL(ncclGroupStart());
            for (int g = 1; g < G; g++) {
                if (len(g) == 0) continue;
                VBC_NCCL(ncclSend(y + lo(g) * esz, (size_t)len(g), dt, g, s->comm[0], s0));
                VBC_NCCL(ncclRecv(s->yb[g], (size_t)len(g), dt, 0, s->comm[g], s->st[g]));
            }
            VBC_NCCL(ncclGroupEnd());
        }
    }
    // 2. the shards' products
    for (int g = 0; g < G; g++) {
        int st;
        if (disj) {
            st = g == 0 ? vbc_mul(s->h[0], trans, x, nx, y + lo(0) * esz, len(0), alpha, beta, VBC_MEM_DEVICE, s0, 0)
                        : vbc_mul(s->h[g], trans, s->xb[g], nx, s->yb[g], len(g), alpha, beta, VBC_MEM_DEVICE,
                                  s->st[g], 0);
        } else {
            st = g == 0 ? vbc_mul(s->h[0], trans, x + lo(0) * esz, len(0), y, ny, alpha, beta, VBC_MEM_DEVICE, s0, 0)
                        : vbc_mul(s->h[g], trans, s->xb[g], len(g), s->yb[g], ny, alpha, 0.0, VBC_MEM_DEVICE,
                                  s->st[g], 0);
        }
        if (st) return st;
    }
    // 3. y to the root: the slices, or the sum of the partials (in place on the root)
    if (!s->comm.empty()) {
        VBC_NCCL(ncclGroupStart());
        for (int g = 0; g < G; g++) {
            if (disj) {
                if (g == 0 || len(g) == 0) continue;
                VBC_NCCL(ncclSend(s->yb[g], (size_t)len(g), dt, 0, s->comm[g], s->st[g]));
                VBC_NCCL(ncclRecv(y + lo(g) * esz, (size_t)len(g), dt, g, s->comm[0], s0));
            } else {
                void *buf = g == 0 ? (void *)y : s->yb[g];
                VBC_NCCL(ncclReduce(buf, buf, (size_t)ny, dt, ncclSum, 0, s->comm[g], stream(g)));
            }
        }
        VBC_NCCL(ncclGroupEnd());
    }
    // 4. the root stream waits for every shard
    for (int g = 1; g < G; g++) {
        {
            DevGuard dg(s->dev[g]);
            VBC_HIPS(hipEventRecord(s->done[g], s->st[g]));
        }
        DevGuard dg(s->dev[0]);
        VBC_HIPS(hipStreamWaitEvent(s0, s->done[g], 0));
    }
    return VBC_OK;
}

}  // namespace

extern "C" {

int vbc1d_create_sharded(vbc_sharded **out, int64_t m, int64_t n, int64_t W, int64_t L, const void *spl,
                         const void *pos, const void *idx, const void *ofs, const void *val, int64_t nval,
                         const vbc_types *types, int ngpus, const int *devices, int split, unsigned flags)
{
    if (!out) return fail(VBC_INVALID_ARG, "NULL out");
    *out = nullptr;
    if (!types) return fail(VBC_INVALID_ARG, "NULL vbc_types");
    if (ngpus < 1 || !devices) return fail(VBC_INVALID_ARG, "ngpus must be >= 1 with a device list");
    if (split != VBC_SPLIT_STRIPES && split != VBC_SPLIT_ROWS)
        return fail(VBC_INVALID_ARG, "split must be VBC_SPLIT_STRIPES or VBC_SPLIT_ROWS");
    if (types->index_bits != 32 && types->index_bits != 64) return fail(VBC_INVALID_ARG, "index_bits must be 32 or 64");
    if (L < 0 || m < 0 || n < 0 || !spl || !pos || !ofs) return fail(VBC_INVALID_ARG, "bad stripe arrays");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return fail(VBC_HIP_ERROR, "hipGetDeviceCount failed");
    bool all_same = true, distinct = true;
    for (int g = 0; g < ngpus; g++) {
        if (devices[g] < 0 || devices[g] >= count) return fail(VBC_INVALID_ARG, "device ordinal out of range");
        all_same = all_same && devices[g] == devices[0];
        for (int k = 0; k < g; k++) distinct = distinct && devices[k] != devices[g];
    }
    if (!all_same && !distinct)
        return fail(VBC_INVALID_ARG, "devices must be all distinct (RCCL) or all the same device");
    const int bits = types->index_bits;
    const std::vector<int64_t> S = as64(spl, bits, L + 1), P = as64(pos, bits, L + 1), O = as64(ofs, bits, L + 1);
    if (S[0] != 1 || S[L] != n + 1 || P[0] != 1 || O[0] != 1) return fail(VBC_INVALID_ARG, "bad Φ.spl / pos / ofs");
    const int64_t q = P[L] - 1;
    if (q < 0 || (q > 0 && !idx)) return fail(VBC_INVALID_ARG, "bad pos");
    if (O[L] - 1 > nval || (O[L] - 1 > 0 && !val)) return fail(VBC_INVALID_ARG, "val shorter than ofs[L+1]-1");
    for (int64_t l = 0; l < L; l++)
        if (S[l + 1] <= S[l] || P[l + 1] < P[l] || O[l + 1] - O[l] != (P[l + 1] - P[l]) * (S[l + 1] - S[l]))
            return fail(VBC_INVALID_ARG, "inconsistent Φ.spl / pos / ofs");
    const std::vector<int64_t> I = as64(idx, bits, q);
    for (int64_t r = 0; r < q; r++)
        if (I[r] < 1 || I[r] > m) return fail(VBC_INVALID_ARG, "idx out of range 1:m");
    const int vsz = vbc::elem_size(types->val_dtype);
    if (vsz == 0) return fail(VBC_UNSUPPORTED_DTYPE, "unknown val_dtype");
    const int csz = vbc::elem_size(types->compute_dtype);
    const char *V = static_cast<const char *>(val);

    vbc_sharded *s = new vbc_sharded;
    s->m = m; s->n = n; s->ngpus = ngpus; s->split = split; s->cdt = types->compute_dtype;
    s->esz = csz; s->local = all_same && ngpus > 1;
    s->dev.assign(devices, devices + ngpus);
    s->h.assign(ngpus, nullptr);
    vbc_types t64 = *types;
    t64.index_bits = 64;

    // byte-balanced cuts (distributed.py stripe_split / row_split): value bytes + 4-B keys + stripe headers
    if (split == VBC_SPLIT_STRIPES) {
        std::vector<double> cost(L + 1, 0.0);
        for (int64_t l = 0; l < L; l++)
            cost[l + 1] = cost[l] + (double)((O[l + 1] - O[l]) * csz + (P[l + 1] - P[l]) * 4 + 12);
        const std::vector<int64_t> lc = balanced_cuts(cost, ngpus);
        s->cut.resize(ngpus + 1);
        for (int g = 0; g <= ngpus; g++) s->cut[g] = S[lc[g]] - 1;  // column ranges
        for (int g = 0; g < ngpus; g++) {
            const int64_t a = lc[g], b = lc[g + 1], Lg = b - a;
            std::vector<int64_t> sg(Lg + 1), pg(Lg + 1), og(Lg + 1);
            for (int64_t l = 0; l <= Lg; l++) {
                sg[l] = S[a + l] - (S[a] - 1);
                pg[l] = P[a + l] - (P[a] - 1);
                og[l] = O[a + l] - (O[a] - 1);
            }
            const int64_t nvg = og[Lg] - 1;
            int st = vbc1d_create_ex(&s->h[g], m, S[b] - S[a], W, Lg, sg.data(), pg.data(), I.data() + (P[a] - 1),
                                     og.data(), nvg > 0 ? V + (O[a] - 1) * vsz : nullptr, nvg, &t64, devices[g], flags);
            if (st) { destroy_all(s); return st; }
        }
    } else {
        std::vector<double> per_row(m + 1, 0.0);
        for (int64_t l = 0; l < L; l++)
            for (int64_t r = P[l] - 1; r < P[l + 1] - 1; r++)
                per_row[I[r]] += (double)((S[l + 1] - S[l]) * csz + 4);  // I is 1-based: prefix index
        for (int64_t i = 0; i < m; i++) per_row[i + 1] += per_row[i];
        s->cut = balanced_cuts(per_row, ngpus);  // row ranges
        for (int g = 0; g < ngpus; g++) {
            const int64_t r0 = s->cut[g], r1 = s->cut[g + 1];
            std::vector<int64_t> pg(L + 1), og(L + 1), ig;
            std::vector<char> vg;
            pg[0] = og[0] = 1;
            for (int64_t l = 0; l < L; l++) {
                const int64_t w = S[l + 1] - S[l];
                int64_t kept = 0;
                for (int64_t r = P[l] - 1; r < P[l + 1] - 1; r++) {
                    if (I[r] <= r0 || I[r] > r1) continue;
                    ig.push_back(I[r] - r0);
                    const char *src = V + (O[l] - 1 + (r - (P[l] - 1)) * w) * vsz;
                    vg.insert(vg.end(), src, src + w * vsz);
                    kept++;
                }
                pg[l + 1] = pg[l] + kept;
                og[l + 1] = og[l] + kept * w;
            }
            int st = vbc1d_create_ex(&s->h[g], r1 - r0, n, W, L, S.data(), pg.data(), ig.empty() ? nullptr : ig.data(),
                                     og.data(), vg.empty() ? nullptr : vg.data(), og[L] - 1, &t64, devices[g], flags);
            if (st) { destroy_all(s); return st; }
        }
    }

    // streams, events, exchange buffers, communicators
    const int64_t big = std::max<int64_t>(std::max(m, n), 1);
    s->st.assign(ngpus, nullptr);
    s->done.assign(ngpus, nullptr);
    s->xb.assign(ngpus, nullptr);
    s->yb.assign(ngpus, nullptr);
    for (int g = 0; g < ngpus; g++) {
        DevGuard dg(devices[g]);
        if (!dg.ok || hipStreamCreateWithFlags(&s->st[g], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&s->done[g], hipEventDisableTiming) != hipSuccess) {
            destroy_all(s);
            return fail(VBC_HIP_ERROR, "stream / event creation failed");
        }
        if (g == 0 && hipEventCreateWithFlags(&s->start, hipEventDisableTiming) != hipSuccess) {
            destroy_all(s);
            return fail(VBC_HIP_ERROR, "event creation failed");
        }
        if (g > 0 && !s->local &&
            (hipMalloc(&s->xb[g], big * csz) != hipSuccess || hipMalloc(&s->yb[g], big * csz) != hipSuccess)) {
            destroy_all(s);
            return fail(VBC_HIP_ERROR, "hipMalloc of an exchange buffer failed");
        }
    }
    if (!s->local) {  // one rank too: the same collectives, trivially (in place on the root)
        s->comm.assign(ngpus, nullptr);
        ncclResult_t r = ncclCommInitAll(s->comm.data(), ngpus, devices);
        if (r != ncclSuccess) {
            s->comm.clear();
            destroy_all(s);
            return nccl_fail(r, "ncclCommInitAll");
        }
    }
    *out = s;
    return VBC_OK;
}

int vbc_sharded_destroy(vbc_sharded *s)
{
    if (s) destroy_all(s);
    return VBC_OK;
}

int vbc_sharded_count(const vbc_sharded *s, int *ngpus)
{
    if (!s || !ngpus) return fail(VBC_INVALID_ARG, "NULL argument");
    *ngpus = s->ngpus;
    return VBC_OK;
}

int vbc_sharded_shard(const vbc_sharded *s, int g, vbc_handle **h, int64_t *lo, int64_t *hi, int *device)
{
    if (!s || g < 0 || g >= s->ngpus) return fail(VBC_INVALID_ARG, "no such shard");
    if (h) *h = s->h[g];
    if (lo) *lo = s->cut[g];
    if (hi) *hi = s->cut[g + 1];
    if (device) *device = s->dev[g];
    return VBC_OK;
}

int vbc_sharded_mul(vbc_sharded *s, int trans, const void *x, int64_t nx, void *y, int64_t ny, double alpha,
                    double beta, int mem, void *stream, unsigned flags)
{
    if (!s) return fail(VBC_INVALID_ARG, "NULL handle");
    const int64_t want_x = trans ? s->m : s->n, want_y = trans ? s->n : s->m;
    if (nx != want_x || ny != want_y) return fail(VBC_DIM_MISMATCH, "DimensionMismatch");
    if ((nx > 0 && !x) || (ny > 0 && !y)) return fail(VBC_INVALID_ARG, "NULL x or y");
    if (ny > 0 && x == y) return fail(VBC_INVALID_ARG, "x and y must not alias");
    if (mem != VBC_MEM_DEVICE && mem != VBC_MEM_HOST)
        return fail(VBC_INVALID_ARG, "mem must be VBC_MEM_DEVICE or VBC_MEM_HOST");
    if (flags & VBC_MUL_REFERENCE_QUIRKS) {  // applied here: the shards then run plain BLAS semantics
        alpha = 1.0;
        if (trans) beta = 0.0;
    }
    std::lock_guard<std::mutex> lk(s->mu);
    if (mem == VBC_MEM_DEVICE) return mul_device(s, trans, static_cast<const char *>(x), nx, static_cast<char *>(y),
                                                 ny, alpha, beta, (hipStream_t)stream);
    // host operands: staged on the root, then the device path on the root's internal stream
    DevGuard dg(s->dev[0]);
    if (!dg.ok) return fail(VBC_HIP_ERROR, "hipSetDevice failed");
    const int64_t esz = s->esz, big = std::max<int64_t>(std::max(s->m, s->n), 1);
    if (!s->hx && (hipMalloc(&s->hx, big * esz) != hipSuccess || hipMalloc(&s->hy, big * esz) != hipSuccess))
        return fail(VBC_HIP_ERROR, "hipMalloc of a staging buffer failed");
    hipStream_t s0 = s->st[0];
    if (nx > 0) VBC_HIPS(hipMemcpyAsync(s->hx, x, nx * esz, hipMemcpyHostToDevice, s0));
    if (ny > 0 && beta != 0.0) VBC_HIPS(hipMemcpyAsync(s->hy, y, ny * esz, hipMemcpyHostToDevice, s0));
    if (int st = mul_device(s, trans, static_cast<const char *>(s->hx), nx, static_cast<char *>(s->hy), ny, alpha,
                            beta, s0))
        return st;
    DevGuard dg2(s->dev[0]);
    if (ny > 0) VBC_HIPS(hipMemcpyAsync(y, s->hy, ny * esz, hipMemcpyDeviceToHost, s0));
    VBC_HIPS(hipStreamSynchronize(s0));
    return VBC_OK;
}

}  // extern "C"
