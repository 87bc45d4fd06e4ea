// libvbc multi-GPU handles (include/vbc.h: vbc1d_create_sharded, vbc2d_create_sharded,
// vbc_sharded_mul, vbc_sharded_mul_ex): ONE process
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
// A SparseMatrixVBC (multiply_VBC.jl:182-189 threads its transposed product the same way) splits the
// same two ways; its row split cuts Π's block rows, so every u×w tile stays whole on one GPU.  The
// code below treats a 1DVBC as the 2D format with unit block rows (K = m, Π.spl = 1:m+1).
// Disjoint outputs are bit-identical to the single-GPU product (unless a shard runs the split planar
// product, see vbc.h VBC_CREATE_SERIAL); reduced ones differ only in the order the partial sums are
// added.
//
// Error discipline: a product that fails after its first collective was enqueued leaves the
// communicators with a half-issued exchange (other GPUs may already wait in it), so the handle is
// marked FAILED and refuses every later product; inside an ncclGroupStart / ncclGroupEnd pair the
// first error stops further calls, and the group is always closed.
//
// When every shard is on the SAME device (devices = {d, d, ...}: oversubscription, or the tests of a
// one-GPU box) the exchange needs no communication at all: shards read x and write y through pointer
// offsets on that device, and reduced outputs accumulate shard after shard (β = 1) on the caller's
// stream.  RCCL refuses two ranks on one GPU, so that mode never creates communicators.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <mutex>
#include <vector>

#include <cmath>

#include "vbc_internal.h"

namespace vbc {  // vbc_generic.hip: strided eltype conversion kernels (vbc_mul_ex uses the same)
int convert_gather(const void *src, int src_dtype, int64_t inc, void *dst, int dst_dtype, int64_t n, hipStream_t s);
int convert_scatter(const void *src, int src_dtype, void *dst, int dst_dtype, int64_t inc, int64_t n, hipStream_t s);
}  // namespace vbc

using vbc::fail;

struct vbc_sharded {
    int64_t m = 0, n = 0;
    int ngpus = 0, split = 0, cdt = 0, esz = 8;
    bool local = false;              // all shards on one device: no communicators
    bool failed = false;             // a product failed mid-exchange: refuse further products
    std::vector<int> dev;
    std::vector<vbc_handle *> h;
    std::vector<int64_t> cut;        // ngpus+1 0-based cuts of the split dimension (columns or rows)
    std::vector<int64_t> xlo, xhi;   // per shard: the span [xlo, xhi) of x its disjoint-output product reads
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> st;     // per shard: internal stream (root: host-pointer products only)
    std::vector<hipEvent_t> done;    // per shard: end of its part of a product
    hipEvent_t start = nullptr;      // root stream: start of a product
    std::vector<void *> xb, yb;      // per non-root shard: x / y buffers (max(m, n) elements each)
    void *hx = nullptr, *hy = nullptr;  // root: staging of host / converted / strided operands
    hipEvent_t stage_ev = nullptr;   // recorded after the last product that used hx / hy
    bool stage_used = false;
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

// One ncclGroupStart / ncclGroupEnd pair: after the first failing call no further call is issued
// (ok() turns false), and end() always closes the group, returning the first error.
class NcclGroup {
  public:
    NcclGroup() { note(ncclGroupStart(), "ncclGroupStart"); opened_ = first_ == ncclSuccess; }
    ~NcclGroup() { if (opened_) (void)ncclGroupEnd(); }
    bool ok() const { return first_ == ncclSuccess; }
    void note(ncclResult_t r, const char *what)
    {
        if (first_ == ncclSuccess && r != ncclSuccess) {
            first_ = r;
            what_ = what;
        }
    }
    int end()
    {
        if (opened_) {
            opened_ = false;
            note(ncclGroupEnd(), "ncclGroupEnd");
        }
        return first_ == ncclSuccess ? VBC_OK : nccl_fail(first_, what_);
    }

  private:
    ncclResult_t first_ = ncclSuccess;
    const char *what_ = "";
    bool opened_ = false;
};

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
    if (!p) return v;
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
    if (s->stage_ev) {
        DevGuard dg(s->dev[0]);
        (void)hipEventSynchronize(s->stage_ev);
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
            if (s->stage_ev) (void)hipEventDestroy(s->stage_ev);
            if (s->hx) (void)hipFree(s->hx);
            if (s->hy) (void)hipFree(s->hy);
        }
    }
    for (vbc_handle *h : s->h)
        if (h) (void)vbc_destroy(h);
    delete s;
}

// One product on device operands of the root (devices[0]), enqueued on the root stream s0.  Sets
// *issued once a collective may have been enqueued (the caller then marks the handle failed on error).
int mul_device(vbc_sharded *s, int trans, const char *x, int64_t nx, char *y, int64_t ny, double alpha,
               double beta, hipStream_t s0, bool *issued)
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
    // 1. x to the shards: the span each one reads (disjoint output) or its slice (partial output)
    if (!s->comm.empty()) {
        *issued = true;
        NcclGroup grp;
        for (int g = 0; g < G && grp.ok(); g++) {
            if (disj) {  // the span of x shard g reads, straight from the root (shard 0 reads the root's x)
                const int64_t xl = s->xlo[g], xn = s->xhi[g] - s->xlo[g];
                if (g == 0 || xn <= 0) continue;
                grp.note(ncclSend(x + xl * esz, (size_t)xn, dt, g, s->comm[0], s0), "ncclSend(x span)");
                if (grp.ok())
                    grp.note(ncclRecv(static_cast<char *>(s->xb[g]) + xl * esz, (size_t)xn, dt, 0, s->comm[g], s->st[g]),
                             "ncclRecv(x span)");
            } else if (g > 0 && len(g) > 0) {
                grp.note(ncclSend(x + lo(g) * esz, (size_t)len(g), dt, g, s->comm[0], s0), "ncclSend(x)");
                if (grp.ok()) grp.note(ncclRecv(s->xb[g], (size_t)len(g), dt, 0, s->comm[g], s->st[g]), "ncclRecv(x)");
            }
        }
        if (int st = grp.end()) return st;
        // β y of a disjoint slice lives on the root: send it to its shard first
        if (disj && beta != 0.0) {
            NcclGroup gb;
            for (int g = 1; g < G && gb.ok(); g++) {
                if (len(g) == 0) continue;
                gb.note(ncclSend(y + lo(g) * esz, (size_t)len(g), dt, g, s->comm[0], s0), "ncclSend(y)");
                if (gb.ok()) gb.note(ncclRecv(s->yb[g], (size_t)len(g), dt, 0, s->comm[g], s->st[g]), "ncclRecv(y)");
            }
            if (int st = gb.end()) return st;
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
        NcclGroup grp;
        for (int g = 0; g < G && grp.ok(); g++) {
            if (disj) {
                if (g == 0 || len(g) == 0) continue;
                grp.note(ncclSend(s->yb[g], (size_t)len(g), dt, 0, s->comm[g], s->st[g]), "ncclSend(y)");
                if (grp.ok()) grp.note(ncclRecv(y + lo(g) * esz, (size_t)len(g), dt, g, s->comm[0], s0), "ncclRecv(y)");
            } else {
                void *buf = g == 0 ? (void *)y : s->yb[g];
                grp.note(ncclReduce(buf, buf, (size_t)ny, dt, ncclSum, 0, s->comm[g], stream(g)), "ncclReduce(y)");
            }
        }
        if (int st = grp.end()) return st;
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

// mul_device with the failed-state bookkeeping.
int mul_checked(vbc_sharded *s, int trans, const char *x, int64_t nx, char *y, int64_t ny, double alpha,
                double beta, hipStream_t s0)
{
    bool issued = false;
    const int st = mul_device(s, trans, x, nx, y, ny, alpha, beta, s0, &issued);
    if (st != VBC_OK && issued) s->failed = true;
    return st;
}

// Root staging buffers (max(m, n) compute-eltype elements each), allocated together on first use;
// `s0` waits for the previous product that used them.
int stage(vbc_sharded *s, hipStream_t s0)
{
    if (!s->hx) {
        const size_t bytes = (size_t)std::max<int64_t>(std::max(s->m, s->n), 1) * s->esz;
        void *a = nullptr, *b = nullptr;
        if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) {
            if (a) (void)hipFree(a);
            return vbc::fail(VBC_HIP_ERROR, "hipMalloc of a staging buffer failed");
        }
        s->hx = a;
        s->hy = b;
    }
    if (s->stage_used) VBC_HIPS(hipStreamWaitEvent(s0, s->stage_ev, 0));
    return VBC_OK;
}

int unstage(vbc_sharded *s, hipStream_t s0)
{
    VBC_HIPS(hipEventRecord(s->stage_ev, s0));
    s->stage_used = true;
    return VBC_OK;
}

// Common validation of a product call; also refuses a FAILED handle.
int check_product(const vbc_sharded *s, int trans, const void *x, int64_t nx, const void *y, int64_t ny, int mem)
{
    if (!s) return vbc::fail(VBC_INVALID_ARG, "NULL handle");
    if (s->failed)
        return vbc::fail(VBC_RCCL_ERROR, "sharded handle is FAILED (an earlier product failed mid-exchange); "
                                         "destroy and re-create it");
    const int64_t want_x = trans ? s->m : s->n, want_y = trans ? s->n : s->m;
    if (nx != want_x || ny != want_y) return vbc::fail(VBC_DIM_MISMATCH, "DimensionMismatch");
    if ((nx > 0 && !x) || (ny > 0 && !y)) return vbc::fail(VBC_INVALID_ARG, "NULL x or y");
    if (ny > 0 && x == y) return vbc::fail(VBC_INVALID_ARG, "x and y must not alias");
    if (mem != VBC_MEM_DEVICE && mem != VBC_MEM_HOST)
        return vbc::fail(VBC_INVALID_ARG, "mem must be VBC_MEM_DEVICE or VBC_MEM_HOST");
    return VBC_OK;
}

void quirks(unsigned flags, int trans, double &alpha, double &beta)
{
    if (flags & VBC_MUL_REFERENCE_QUIRKS) {  // applied here: the shards then run plain BLAS semantics
        alpha = 1.0;
        if (trans) beta = 0.0;
    }
}

// Host operands of the compute eltype: staged on the root, the device path on the root's internal
// stream, returns when y is final.  The caller holds s->mu.
int mul_host(vbc_sharded *s, int trans, const void *x, int64_t nx, void *y, int64_t ny, double alpha, double beta)
{
    DevGuard dg(s->dev[0]);
    if (!dg.ok) return vbc::fail(VBC_HIP_ERROR, "hipSetDevice failed");
    const int64_t esz = s->esz;
    hipStream_t s0 = s->st[0];
    if (int st = stage(s, s0)) return st;
    if (nx > 0) VBC_HIPS(hipMemcpyAsync(s->hx, x, nx * esz, hipMemcpyHostToDevice, s0));
    if (ny > 0 && beta != 0.0) VBC_HIPS(hipMemcpyAsync(s->hy, y, ny * esz, hipMemcpyHostToDevice, s0));
    if (int st = mul_checked(s, trans, static_cast<const char *>(s->hx), nx, static_cast<char *>(s->hy), ny, alpha,
                             beta, s0))
        return st;
    DevGuard dg2(s->dev[0]);
    if (ny > 0) VBC_HIPS(hipMemcpyAsync(y, s->hy, ny * esz, hipMemcpyDeviceToHost, s0));
    if (int st = unstage(s, s0)) return st;
    VBC_HIPS(hipStreamSynchronize(s0));
    return VBC_OK;
}

// The matrix of either format as the 2D format: 1DVBC = unit block rows (K = m, Π.spl = 1:m+1).
struct Fields {
    bool is2d = false;
    int64_t m = 0, n = 0, U = 1, W = 0, K = 0, L = 0;
    std::vector<int64_t> PS, S, P, I, O;  // 1-based, as the reference stores them
    const char *V = nullptr;
    int vsz = 0;
    int64_t u(int64_t k) const { return is2d ? PS[k + 1] - PS[k] : 1; }  // height of block row k (0-based)
};

int validate(const Fields &f)
{
    const int64_t L = f.L;
    if (f.S[0] != 1 || f.S[L] != f.n + 1 || f.P[0] != 1 || f.O[0] != 1) return vbc::fail(VBC_INVALID_ARG, "bad Φ.spl / pos / ofs");
    if (f.is2d) {
        if (f.PS[0] != 1 || f.PS[f.K] != f.m + 1) return vbc::fail(VBC_INVALID_ARG, "bad Π.spl");
        for (int64_t k = 0; k < f.K; k++)
            if (f.PS[k + 1] <= f.PS[k]) return vbc::fail(VBC_INVALID_ARG, "Π.spl must increase");
    }
    for (int64_t l = 0; l < L; l++)
        if (f.S[l + 1] <= f.S[l] || f.P[l + 1] < f.P[l]) return vbc::fail(VBC_INVALID_ARG, "inconsistent Φ.spl / pos");
    const int64_t lim = f.is2d ? f.K : f.m;
    for (int64_t r = 0; r < f.P[L] - 1; r++)
        if (f.I[r] < 1 || f.I[r] > lim) return vbc::fail(VBC_INVALID_ARG, f.is2d ? "idx out of range 1:K" : "idx out of range 1:m");
    for (int64_t l = 0; l < L; l++) {  // ofs steps: Σ u·w over the stripe's blocks
        int64_t want = 0;
        const int64_t w = f.S[l + 1] - f.S[l];
        for (int64_t r = f.P[l] - 1; r < f.P[l + 1] - 1; r++) want += f.u(f.I[r] - 1) * w;
        if (f.O[l + 1] - f.O[l] != want) return vbc::fail(VBC_INVALID_ARG, "inconsistent ofs");
    }
    return VBC_OK;
}

// One shard's handle from its fields (1-based Int64 arrays, raw values of val_dtype).
int create_shard(const Fields &f, vbc_handle **out, int64_t m, int64_t n, int64_t K, const int64_t *ps, int64_t L,
                 const int64_t *spl, const int64_t *pos, const int64_t *idx, const int64_t *ofs, const char *val,
                 const vbc_types *t64, int device, unsigned flags)
{
    const int64_t nv = ofs[L] - 1;
    if (f.is2d)
        return vbc2d_create_ex(out, m, n, f.U, f.W, K, ps, L, spl, pos, idx, ofs, nv > 0 ? val : nullptr, nv, t64, device,
                               flags);
    return vbc1d_create_ex(out, m, n, f.W, L, spl, pos, idx, ofs, nv > 0 ? val : nullptr, nv, t64, device, flags);
}

// The largest R in {3, 2} such that R divides m and every stripe's stored rows come in aligned runs of R
// consecutive rows (a node's dof rows); 1 otherwise (distributed.py row_runs).  Row cuts at multiples of R
// keep every row shard node-blocked (its forward lane pairs / row runs need m_local % 3 == 0).
int64_t row_runs(const Fields &f)
{
    const int64_t L = f.L;
    for (int64_t R = 3; R >= 2; R--) {
        if (f.m % R) continue;
        bool ok = true;
        for (int64_t l = 0; l < L && ok; l++) {
            const int64_t a = f.P[l] - 1, b = f.P[l + 1] - 1;
            if ((b - a) % R) { ok = false; break; }
            for (int64_t r = a; r < b && ok; r++) {
                const int64_t k = (r - a) % R, row = f.I[r] - 1;
                ok = row % R == k && (k == 0 || row == f.I[r - 1]);
            }
        }
        if (ok) return R;
    }
    return 1;
}

// The cuts of a split (byte-balanced, distributed.py stripe_split / row_split: value bytes + 4-B keys + stripe
// headers) and, per shard, the span [xlo, xhi) of x its disjoint-output product reads -- the rows its stripes
// store (stripe split, B'x) or the columns of the stripes with a stored row in its row range (row split, B x).
// The root sends each shard that span instead of broadcasting x; a mesh operator's shard reads its own share
// of x plus a halo.
struct Plan {
    std::vector<int64_t> cuts;      // stripe split: N+1 stripe cuts; row split: N+1 block-row (1D: row) cuts
    std::vector<int64_t> xlo, xhi;  // per shard, 0-based; [0, 0) when it reads none
};

Plan plan_split(const Fields &f, int csz, int N, int split)
{
    const int64_t L = f.L;
    const std::vector<int64_t> &S = f.S, &P = f.P, &I = f.I, &O = f.O;
    Plan p;
    p.xlo.assign(N, INT64_MAX);
    p.xhi.assign(N, INT64_MIN);
    if (split == VBC_SPLIT_STRIPES) {
        std::vector<double> cost(L + 1, 0.0);
        for (int64_t l = 0; l < L; l++)
            cost[l + 1] = cost[l] + (double)((O[l + 1] - O[l]) * csz + (P[l + 1] - P[l]) * 4 + 12);
        p.cuts = balanced_cuts(cost, N);
        for (int g = 0; g < N; g++)
            for (int64_t r = P[p.cuts[g]] - 1; r < P[p.cuts[g + 1]] - 1; r++) {
                const int64_t k = I[r] - 1;
                p.xlo[g] = std::min(p.xlo[g], f.is2d ? f.PS[k] - 1 : k);
                p.xhi[g] = std::max(p.xhi[g], f.is2d ? f.PS[k + 1] - 1 : k + 1);
            }
    } else {
        // cost per block row (1D: per row) = its blocks' value bytes + a 4-B key each
        const int64_t K = f.is2d ? f.K : f.m;
        std::vector<double> per(K + 1, 0.0);
        for (int64_t l = 0; l < L; l++)
            for (int64_t r = P[l] - 1; r < P[l + 1] - 1; r++)
                per[I[r]] += (double)(f.u(I[r] - 1) * (S[l + 1] - S[l]) * csz + 4);  // I is 1-based: prefix index
        for (int64_t k = 0; k < K; k++) per[k + 1] += per[k];
        std::vector<int64_t> kc = balanced_cuts(per, N);  // block-row ranges
        if (!f.is2d) {  // a 1DVBC's node runs stay whole (distributed.py row_split / row_runs)
            const int64_t a = row_runs(f);
            if (a > 1)
                for (int g = 1; g < N; g++) kc[g] = std::max(kc[g - 1], std::min(K, (kc[g] + a / 2) / a * a));
        }
        for (int64_t l = 0; l < L; l++)
            for (int64_t r = P[l] - 1; r < P[l + 1] - 1; r++) {  // shard g holds 1-based k in (kc[g], kc[g+1]]
                const int g = (int)(std::lower_bound(kc.begin() + 1, kc.end(), I[r]) - (kc.begin() + 1));
                p.xlo[g] = std::min(p.xlo[g], S[l] - 1);
                p.xhi[g] = std::max(p.xhi[g], S[l + 1] - 1);
            }
        p.cuts = std::move(kc);
    }
    for (int g = 0; g < N; g++)
        if (p.xhi[g] <= p.xlo[g]) p.xlo[g] = p.xhi[g] = 0;
    return p;
}

// VBC_SPLIT_AUTO (vbc.h): the split with the smaller predicted time of the products `flags` builds (B'x for
// VBC_CREATE_TRANSPOSED or no direction flag, B x for VBC_CREATE_FORWARD).  The model is distributed.py's
// predict_product_us for this one-process handle's exchange: the slowest shard's kernel -- a
// measured launch-and-ramp floor plus its bytes (matrix share, x reads, y writes) at the measured streaming
// rate -- plus the exchange through the root: each shard's x span sent over its own link and y slices
// gathered (disjoint output), or x slices scattered and an ncclReduce of y (partial output), at ASSUMED xGMI
// rates (7 links of 76.8 GB/s per direction, 60 % of it reached, 2 us per ring step; no multi-GPU box was
// available to measure).
constexpr double kModelT0Us = 3.1, kModelStreamGBs = 5700.0;
constexpr double kModelLinkGBs = 76.8 * 0.6, kModelCollGBs = 7 * kModelLinkGBs, kModelStepUs = 2.0;

double predict_us(const Fields &f, int csz, int N, int split, int trans, const Plan &p)
{
    const int64_t L = f.L;
    double mat = (double)csz * (double)(f.O[L] - 1) + 4.0 * (double)(f.P[L] - 1) + 4.0 * (3.0 * L + 3.0) +
                 (f.is2d ? 4.0 * (f.K + 1) : 0.0);
    mat /= N;
    if (split == VBC_SPLIT_ROWS && N > 1) mat += 12.0 * (double)L * (N - 1) / N;  // every row shard keeps the headers
    const double nx = (double)(trans ? f.m : f.n) * csz, ny = (double)(trans ? f.n : f.m) * csz;
    const bool disj = disjoint_output(split, trans);
    double span = 0.0, sent = 0.0;  // the widest x span a shard reads; the widest the root sends
    for (int g = 0; g < N; g++) {
        span = std::max(span, (double)(p.xhi[g] - p.xlo[g]) * csz);
        if (g > 0) sent = std::max(sent, (double)(p.xhi[g] - p.xlo[g]) * csz);
    }
    const double kern = kModelT0Us + (mat + (disj ? span : nx / N) + (disj ? ny / N : ny)) / (kModelStreamGBs * 1e3);
    if (N <= 1) return kern;
    // a ring reduce moves the whole vector through every hop (pipelined); the root's direct sends and receives
    // of slices move (N-1)/N of it; the x spans go out over the root's N-1 links at once
    const double part = (double)(N - 1) / N, lat = (N - 1) * kModelStepUs, bw = kModelCollGBs * 1e3;
    const double coll = disj ? (sent / (kModelLinkGBs * 1e3) + kModelStepUs) + (part * ny / bw + lat)  // x spans, y slices
                             : (part * nx / bw + lat) + (ny / bw + lat);  // scatter x slices, reduce y
    return kern + coll;
}

// Within 2 % the costs tie (a square operator: the two splits mirror each other); a tie goes to the split
// whose outputs are disjoint for the one direction built (bit-identical to the single-GPU product, no
// reduction), and to the stripe split when both are (the reference's own parallel direction,
// multiply_1DVBC.jl:169-177).
int auto_split(const Fields &f, int csz, int N, unsigned flags)
{
    const bool t = (flags & VBC_CREATE_TRANSPOSED) || !(flags & VBC_CREATE_FORWARD);
    const bool fw = (flags & VBC_CREATE_FORWARD) != 0;
    double cost[2] = {0.0, 0.0};
    for (int sp = 0; sp < 2; sp++) {
        const Plan p = plan_split(f, csz, N, sp);
        if (t) cost[sp] += predict_us(f, csz, N, sp, 1, p);
        if (fw) cost[sp] += predict_us(f, csz, N, sp, 0, p);
    }
    if (cost[VBC_SPLIT_ROWS] < 0.98 * cost[VBC_SPLIT_STRIPES]) return VBC_SPLIT_ROWS;
    if (cost[VBC_SPLIT_STRIPES] < 0.98 * cost[VBC_SPLIT_ROWS]) return VBC_SPLIT_STRIPES;
    return (fw && !t) ? VBC_SPLIT_ROWS : VBC_SPLIT_STRIPES;
}

int create_sharded(vbc_sharded **out, Fields &f, int64_t nval, const vbc_types *types, int ngpus, const int *devices,
                   int split, unsigned flags)
{
    if (!out) return vbc::fail(VBC_INVALID_ARG, "NULL out");
    *out = nullptr;
    if (!types) return vbc::fail(VBC_INVALID_ARG, "NULL vbc_types");
    if (ngpus < 1 || !devices) return vbc::fail(VBC_INVALID_ARG, "ngpus must be >= 1 with a device list");
    if (split != VBC_SPLIT_STRIPES && split != VBC_SPLIT_ROWS && split != VBC_SPLIT_AUTO)
        return vbc::fail(VBC_INVALID_ARG, "split must be VBC_SPLIT_STRIPES, VBC_SPLIT_ROWS or VBC_SPLIT_AUTO");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return vbc::fail(VBC_HIP_ERROR, "hipGetDeviceCount failed");
    bool all_same = true, distinct = true;
    for (int g = 0; g < ngpus; g++) {
        if (devices[g] < 0 || devices[g] >= count) return vbc::fail(VBC_INVALID_ARG, "device ordinal out of range");
        all_same = all_same && devices[g] == devices[0];
        for (int k = 0; k < g; k++) distinct = distinct && devices[k] != devices[g];
    }
    if (!all_same && !distinct)
        return vbc::fail(VBC_INVALID_ARG, "devices must be all distinct (RCCL) or all the same device");
    if (int st = validate(f)) return st;
    const int64_t L = f.L, m = f.m, n = f.n;
    if (f.O[L] - 1 > nval || (f.O[L] - 1 > 0 && !f.V)) return vbc::fail(VBC_INVALID_ARG, "val shorter than ofs[L+1]-1");
    f.vsz = vbc::elem_size(types->val_dtype);
    if (f.vsz == 0) return vbc::fail(VBC_UNSUPPORTED_DTYPE, "unknown val_dtype");
    const int csz = vbc::elem_size(types->compute_dtype);
    if (csz == 0) return vbc::fail(VBC_UNSUPPORTED_DTYPE, "unknown compute_dtype");
    if (split == VBC_SPLIT_AUTO) split = auto_split(f, csz, ngpus, flags);
    const char *V = f.V;
    const int vsz = f.vsz;

    vbc_sharded *s = new vbc_sharded;
    s->m = m; s->n = n; s->ngpus = ngpus; s->split = split; s->cdt = types->compute_dtype;
    s->esz = csz; s->local = all_same && ngpus > 1;
    s->dev.assign(devices, devices + ngpus);
    s->h.assign(ngpus, nullptr);
    vbc_types t64 = *types;
    t64.index_bits = 64;
    const std::vector<int64_t> &S = f.S, &P = f.P, &I = f.I, &O = f.O;

    Plan plan = plan_split(f, csz, ngpus, split);
    s->xlo = plan.xlo;
    s->xhi = plan.xhi;
    if (split == VBC_SPLIT_STRIPES) {
        const std::vector<int64_t> &lc = plan.cuts;
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
            int st = create_shard(f, &s->h[g], m, S[b] - S[a], f.K, f.PS.data(), Lg, sg.data(), pg.data(),
                                  I.data() + (P[a] - 1), og.data(), V + (O[a] - 1) * vsz, &t64, devices[g], flags);
            if (st) { destroy_all(s); return st; }
        }
    } else {
        const std::vector<int64_t> &kc = plan.cuts;  // block-row ranges
        s->cut.resize(ngpus + 1);
        for (int g = 0; g <= ngpus; g++) s->cut[g] = f.is2d ? f.PS[kc[g]] - 1 : kc[g];  // row ranges
        for (int g = 0; g < ngpus; g++) {
            const int64_t k0 = kc[g], k1 = kc[g + 1];
            std::vector<int64_t> pg(L + 1), og(L + 1), ig, psg;
            std::vector<char> vg;
            pg[0] = og[0] = 1;
            for (int64_t l = 0; l < L; l++) {
                const int64_t w = S[l + 1] - S[l];
                int64_t kept = 0, kept_vals = 0, off = O[l] - 1;  // running value offset inside the stripe
                for (int64_t r = P[l] - 1; r < P[l + 1] - 1; r++) {
                    const int64_t bsz = f.u(I[r] - 1) * w;
                    if (I[r] > k0 && I[r] <= k1) {
                        ig.push_back(I[r] - k0);
                        const char *src = V + off * vsz;
                        vg.insert(vg.end(), src, src + bsz * vsz);
                        kept++;
                        kept_vals += bsz;
                    }
                    off += bsz;
                }
                pg[l + 1] = pg[l] + kept;
                og[l + 1] = og[l] + kept_vals;
            }
            if (f.is2d) {
                psg.resize(k1 - k0 + 1);
                for (int64_t k = k0; k <= k1; k++) psg[k - k0] = f.PS[k] - (f.PS[k0] - 1);
            }
            int st = create_shard(f, &s->h[g], s->cut[g + 1] - s->cut[g], n, k1 - k0, psg.data(), L, S.data(),
                                  pg.data(), ig.empty() ? nullptr : ig.data(), og.data(),
                                  vg.empty() ? nullptr : vg.data(), &t64, devices[g], flags);
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
            return vbc::fail(VBC_HIP_ERROR, "stream / event creation failed");
        }
        if (g == 0 && (hipEventCreateWithFlags(&s->start, hipEventDisableTiming) != hipSuccess ||
                       hipEventCreateWithFlags(&s->stage_ev, hipEventDisableTiming) != hipSuccess)) {
            destroy_all(s);
            return vbc::fail(VBC_HIP_ERROR, "event creation failed");
        }
        // (x buffers zeroed once: a shard's product reads only its x span, which every product refreshes)
        if (g > 0 && !s->local &&
            (hipMalloc(&s->xb[g], big * csz) != hipSuccess || hipMalloc(&s->yb[g], big * csz) != hipSuccess ||
             hipMemset(s->xb[g], 0, big * csz) != hipSuccess)) {
            destroy_all(s);
            return vbc::fail(VBC_HIP_ERROR, "hipMalloc of an exchange buffer failed");
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

bool is_float(int dt) { return dt == VBC_F64 || dt == VBC_F32; }
bool known_dtype(int dt) { return dt >= VBC_F64 && dt <= VBC_BOOL; }

}  // namespace

extern "C" {

int vbc1d_create_sharded(vbc_sharded **out, int64_t m, int64_t n, int64_t W, int64_t L, const void *spl,
                         const void *pos, const void *idx, const void *ofs, const void *val, int64_t nval,
                         const vbc_types *types, int ngpus, const int *devices, int split, unsigned flags)
{
    if (out) *out = nullptr;
    if (!types) return fail(VBC_INVALID_ARG, "NULL vbc_types");
    if (types->index_bits != 32 && types->index_bits != 64) return fail(VBC_INVALID_ARG, "index_bits must be 32 or 64");
    if (L < 0 || m < 0 || n < 0 || !spl || !pos || !ofs) return fail(VBC_INVALID_ARG, "bad stripe arrays");
    const int bits = types->index_bits;
    Fields f;
    f.m = m; f.n = n; f.W = W; f.K = m; f.L = L;
    f.S = as64(spl, bits, L + 1);
    f.P = as64(pos, bits, L + 1);
    f.O = as64(ofs, bits, L + 1);
    const int64_t q = f.P[L] - 1;
    if (f.P[0] != 1 || q < 0 || (q > 0 && !idx)) return fail(VBC_INVALID_ARG, "bad pos");
    f.I = as64(idx, bits, q);
    f.V = static_cast<const char *>(val);
    return create_sharded(out, f, nval, types, ngpus, devices, split, flags);
}

int vbc2d_create_sharded(vbc_sharded **out, int64_t m, int64_t n, int64_t U, int64_t W, int64_t K, const void *pspl,
                         int64_t L, const void *spl, const void *pos, const void *idx, const void *ofs, const void *val,
                         int64_t nval, const vbc_types *types, int ngpus, const int *devices, int split, unsigned flags)
{
    if (out) *out = nullptr;
    if (!types) return fail(VBC_INVALID_ARG, "NULL vbc_types");
    if (types->index_bits != 32 && types->index_bits != 64) return fail(VBC_INVALID_ARG, "index_bits must be 32 or 64");
    if (K < 0 || L < 0 || m < 0 || n < 0 || !pspl || !spl || !pos || !ofs)
        return fail(VBC_INVALID_ARG, "bad partition arrays");
    const int bits = types->index_bits;
    Fields f;
    f.is2d = true;
    f.m = m; f.n = n; f.U = U; f.W = W; f.K = K; f.L = L;
    f.PS = as64(pspl, bits, K + 1);
    f.S = as64(spl, bits, L + 1);
    f.P = as64(pos, bits, L + 1);
    f.O = as64(ofs, bits, L + 1);
    const int64_t q = f.P[L] - 1;
    if (f.P[0] != 1 || q < 0 || (q > 0 && !idx)) return fail(VBC_INVALID_ARG, "bad pos");
    f.I = as64(idx, bits, q);
    f.V = static_cast<const char *>(val);
    return create_sharded(out, f, nval, types, ngpus, devices, split, flags);
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

int vbc_sharded_split(const vbc_sharded *s, int *split)
{
    if (!s || !split) return fail(VBC_INVALID_ARG, "NULL argument");
    *split = s->split;
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

int vbc_sharded_xspan(const vbc_sharded *s, int g, int64_t *lo, int64_t *hi)
{
    if (!s || g < 0 || g >= s->ngpus) return fail(VBC_INVALID_ARG, "no such shard");
    if (lo) *lo = s->xlo[g];
    if (hi) *hi = s->xhi[g];
    return VBC_OK;
}

int vbc_sharded_mul(vbc_sharded *s, int trans, const void *x, int64_t nx, void *y, int64_t ny, double alpha,
                    double beta, int mem, void *stream, unsigned flags)
{
    if (int st = check_product(s, trans, x, nx, y, ny, mem)) return st;
    quirks(flags, trans, alpha, beta);
    std::lock_guard<std::mutex> lk(s->mu);
    if (mem == VBC_MEM_DEVICE)
        return mul_checked(s, trans, static_cast<const char *>(x), nx, static_cast<char *>(y), ny, alpha, beta,
                           (hipStream_t)stream);
    return mul_host(s, trans, x, nx, y, ny, alpha, beta);
}

int vbc_sharded_mul_ex(vbc_sharded *s, int trans, const void *x, int x_dtype, int64_t incx, int64_t nx, void *y,
                       int y_dtype, int64_t incy, int64_t ny, double alpha, double beta, int mem, void *stream,
                       unsigned flags)
{
    if (int st = check_product(s, trans, x, nx, y, ny, mem)) return st;
    const int cdt = s->cdt;
    if (!known_dtype(x_dtype) || !known_dtype(y_dtype)) return fail(VBC_UNSUPPORTED_DTYPE, "unknown eltype");
    if (cdt == VBC_I64 && is_float(x_dtype))
        return fail(VBC_UNSUPPORTED_DTYPE, "floating-point x on an integer handle (InexactError)");
    if (is_float(cdt) ? y_dtype != cdt : (y_dtype != VBC_I64 && y_dtype != VBC_I32))
        return fail(VBC_UNSUPPORTED_DTYPE, "eltype(y) must be the handle's compute eltype (or Int32 on an Int64 handle)");
    if ((nx > 0 && incx == 0) || (ny > 0 && incy == 0)) return fail(VBC_INVALID_ARG, "zero stride");
    if (cdt == VBC_I64 && (alpha != std::trunc(alpha) || beta != std::trunc(beta)))
        return fail(VBC_INVALID_ARG, "alpha and beta must be integers on an integer handle (InexactError)");
    const bool direct_x = x_dtype == cdt && (incx == 1 || nx <= 1);
    const bool direct_y = y_dtype == cdt && (incy == 1 || ny <= 1);
    if (direct_x && direct_y) return vbc_sharded_mul(s, trans, x, nx, y, ny, alpha, beta, mem, stream, flags);
    quirks(flags, trans, alpha, beta);
    const int64_t esz = s->esz;
    std::lock_guard<std::mutex> lk(s->mu);
    if (mem == VBC_MEM_HOST) {  // convert on the host, then the contiguous host path
        std::vector<char> xs, ys((size_t)std::max<int64_t>(ny, 1) * esz);
        const void *xp = x;
        if (!direct_x) {
            xs.resize((size_t)std::max<int64_t>(nx, 1) * esz);
            vbc::host_convert_to(x, x_dtype, nx, incx, xs.data(), cdt);
            xp = xs.data();
        }
        if (beta != 0.0) vbc::host_convert_to(y, y_dtype, ny, incy, ys.data(), cdt);
        if (int st = mul_host(s, trans, xp, nx, ys.data(), ny, alpha, beta)) return st;
        vbc::host_store(ys.data(), cdt, ny, y, y_dtype, incy);
        return VBC_OK;
    }
    // device operands on devices[0]: conversion kernels into / out of the root staging buffers
    DevGuard dg(s->dev[0]);
    if (!dg.ok) return fail(VBC_HIP_ERROR, "hipSetDevice failed");
    hipStream_t s0 = (hipStream_t)stream;
    if (int st = stage(s, s0)) return st;
    const char *dx = static_cast<const char *>(x);
    char *dy = static_cast<char *>(y);
    if (!direct_x) {
        if (int st = vbc::convert_gather(x, x_dtype, incx, s->hx, cdt, nx, s0)) return st;
        dx = static_cast<const char *>(s->hx);
    }
    if (!direct_y) {
        if (beta != 0.0) {
            if (int st = vbc::convert_gather(y, y_dtype, incy, s->hy, cdt, ny, s0)) return st;
        }
        dy = static_cast<char *>(s->hy);
    }
    if (int st = mul_checked(s, trans, dx, nx, dy, ny, alpha, beta, s0)) return st;
    DevGuard dg2(s->dev[0]);
    if (!direct_y) {
        if (int st = vbc::convert_scatter(s->hy, cdt, y, y_dtype, incy, ny, s0)) return st;
    }
    return unstage(s, s0);
}

}  // extern "C"
