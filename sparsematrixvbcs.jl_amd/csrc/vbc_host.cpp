// libvbc host-side layout producers: partitioners and CSC -> reference-layout builders.
//
// The builders produce the exact field arrays of the reference's constructors
// (constructors_1DVBC.jl:9-92, constructors_VBC.jl:15-133) but by a different algorithm: instead of
// the reference's w-way column merge, each stripe's distinct rows (or block rows) are collected,
// sorted and deduplicated, given slots, and the stripe's entries are placed by a merge walk of each
// (sorted) column against the slots.  1DVBC stripes are independent, so count and fill run over
// stripe ranges on host threads (VBC_HOST_THREADS, default min(hardware threads, 16)).  The oracle
// (oracle/vbc_oracle.c) restates the merge line by line; tests require both to agree exactly, which
// pins this implementation.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

#include "vbc_host.h"
#include "vbc_internal.h"

using vbc::fail;

namespace {

// Host threads for the builders: VBC_HOST_THREADS, else min(hardware threads, 16).
int host_threads()
{
    if (const char *e = std::getenv("VBC_HOST_THREADS")) return std::max(1, std::atoi(e));
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc ? hc : 1u, 16u));
}

// f(lo, hi, status&) over [0, n) in contiguous chunks on host threads; the first nonzero status wins.
template <typename F>
int parallel_ranges(int64_t n, int64_t work, F f)
{
    const int nt = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, work / 200000));
    if (nt <= 1 || n < 2 * nt) {
        int st = VBC_OK;
        f((int64_t)0, n, st);
        return st;
    }
    std::vector<int> sts(nt, VBC_OK);
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
        th.emplace_back([&, t] { f(n * t / nt, n * (t + 1) / nt, sts[t]); });
    for (auto &x : th) x.join();
    for (int st : sts)
        if (st) return st;
    return VBC_OK;
}


int check_csc(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval)
{
    if (m < 0 || n < 0) return fail(VBC_INVALID_ARG, "number of rows/columns must be >= 0");
    if (!colptr) return fail(VBC_INVALID_ARG, "colptr is NULL");
    if (colptr[0] != 1) return fail(VBC_INVALID_ARG, "colptr[1] must be 1");
    for (int64_t j = 0; j < n; j++)
        if (colptr[j + 1] < colptr[j]) return fail(VBC_INVALID_ARG, "colptr must be non-decreasing");
    if (colptr[n] > 1 && !rowval) return fail(VBC_INVALID_ARG, "rowval is NULL");
    // 1: a row index out of 1:m, 2: rows not strictly increasing within a column (worst of all columns)
    const int bad = parallel_ranges(n, colptr[n] - 1, [&](int64_t j0, int64_t j1, int &st) {
        for (int64_t j = j0; j < j1; j++)
            for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; p++) {
                const int64_t i = rowval[p];
                if (i < 1 || i > m) st = std::max(st, 1);
                else if (p > colptr[j] - 1 && rowval[p - 1] >= i) st = std::max(st, 2);
            }
    });
    if (bad == 1) return fail(VBC_INVALID_ARG, "rowval out of range 1:m");
    if (bad) return fail(VBC_INVALID_ARG, "rowval must be strictly increasing within a column");
    return VBC_OK;
}

int check_spl(int64_t n, int64_t L, const int64_t *spl, int64_t W, bool assert_w)
{
    if (L < 0) return fail(VBC_INVALID_ARG, "L must be >= 0");
    if (spl[0] != 1 || spl[L] != n + 1) return fail(VBC_INVALID_ARG, "spl must run from 1 to n+1");
    for (int64_t l = 0; l < L; l++) {
        const int64_t w = spl[l + 1] - spl[l];
        if (w < 1) return fail(VBC_INVALID_ARG, "spl must be strictly increasing");
        if (assert_w && w > W) return fail(VBC_ASSERTION, "AssertionError: w <= W");
    }
    return VBC_OK;
}

// Sorted distinct 0-based rows of columns [j0, j1) (each column's rows ascending): a merge of the
// sorted columns with duplicates dropped; columns whose pattern equals the first's (every column of a
// StrictChunker stripe) are skipped.
inline void stripe_rows(const int64_t *colptr, const int64_t *rowval, int64_t j0, int64_t j1,
                        std::vector<int64_t> &rows, std::vector<int64_t> &tmp)
{
    rows.clear();
    const int64_t *a = rowval + colptr[j0] - 1;
    const int64_t na = colptr[j0 + 1] - colptr[j0];
    for (int64_t p = 0; p < na; p++) rows.push_back(a[p] - 1);
    for (int64_t j = j0 + 1; j < j1; j++) {
        const int64_t *b = rowval + colptr[j] - 1;
        const int64_t nb = colptr[j + 1] - colptr[j];
        if (nb == na && std::equal(a, a + na, b)) continue;
        tmp.clear();
        size_t s = 0;
        for (int64_t p = 0; p < nb; p++) {
            const int64_t i = b[p] - 1;
            while (s < rows.size() && rows[s] < i) tmp.push_back(rows[s++]);
            if (s < rows.size() && rows[s] == i) s++;
            tmp.push_back(i);
        }
        while (s < rows.size()) tmp.push_back(rows[s++]);
        rows.swap(tmp);
    }
}

template <typename T>
int fill_1d(int64_t m, int64_t W, const int64_t *colptr, const int64_t *rowval, const T *nzval,
            int64_t L, const int64_t *spl, const int64_t *pos, const int64_t *ofs, int64_t *idx,
            T *val, int64_t pad)
{
    (void)m;
    const int64_t nv = ofs[L] - 1;
    std::fill(val + nv, val + nv + pad, T(0));
    for (int64_t l = 0; l < L; l++)
        if (spl[l + 1] - spl[l] > W) return fail(VBC_ASSERTION, "AssertionError: w <= W");
    const int status = parallel_ranges(L, colptr[spl[L] - 1] - 1, [&](int64_t l0, int64_t l1, int &st) {
        std::vector<int64_t> rows, tmp;
        for (int64_t l = l0; l < l1 && st == VBC_OK; l++) {
            const int64_t j0 = spl[l] - 1, j1 = spl[l + 1] - 1, w = j1 - j0;
            stripe_rows(colptr, rowval, j0, j1, rows, tmp);
            if ((int64_t)rows.size() != pos[l + 1] - pos[l]) {
                st = VBC_INVALID_ARG;
                continue;
            }
            for (size_t s = 0; s < rows.size(); s++) idx[pos[l] - 1 + (int64_t)s] = rows[s] + 1;
            T *seg = val + (ofs[l] - 1);
            std::fill(seg, seg + (int64_t)rows.size() * w, T(0));
            for (int64_t j = j0; j < j1; j++) {  // merge walk: the column's rows against the slots
                size_t s = 0;
                for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; p++) {
                    const int64_t i = rowval[p] - 1;
                    while (rows[s] != i) s++;
                    seg[(int64_t)s * w + (j - j0)] = nzval[p];
                }
            }
        }
    });
    // the message is set here: the last-error string is per thread
    return status ? fail(status, "pos inconsistent with A and spl") : VBC_OK;
}

template <typename T>
int fill_2d(int64_t m, int64_t U, int64_t W, const int64_t *colptr, const int64_t *rowval,
            const T *nzval, int64_t K, const int64_t *pspl, int64_t L, const int64_t *spl,
            const int64_t *pos, const int64_t *ofs, int64_t *idx, T *val, int64_t pad)
{
    std::vector<int64_t> asg(m), stamp(K, 0), boff(K, 0), blocks;
    for (int64_t k = 0; k < K; k++) {
        if (pspl[k + 1] - pspl[k] > U) return fail(VBC_ASSERTION, "AssertionError: u <= U");
        for (int64_t i = pspl[k] - 1; i < pspl[k + 1] - 1; i++) asg[i] = k;
    }
    const int64_t nv = ofs[L] - 1;
    std::fill(val, val + nv + pad, T(0));
    for (int64_t l = 0; l < L; l++) {
        const int64_t j0 = spl[l] - 1, j1 = spl[l + 1] - 1, w = j1 - j0;
        if (w > W) return fail(VBC_ASSERTION, "AssertionError: w <= W");
        blocks.clear();
        for (int64_t j = j0; j < j1; j++)
            for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; p++) {
                const int64_t k = asg[rowval[p] - 1];
                if (stamp[k] != l + 1) { stamp[k] = l + 1; blocks.push_back(k); }
            }
        std::sort(blocks.begin(), blocks.end());
        if ((int64_t)blocks.size() != pos[l + 1] - pos[l])
            return fail(VBC_INVALID_ARG, "pos inconsistent with A, Π and Φ");
        int64_t off = 0;
        for (size_t s = 0; s < blocks.size(); s++) {
            const int64_t k = blocks[s];
            boff[k] = off;
            off += (pspl[k + 1] - pspl[k]) * w;
            idx[pos[l] - 1 + (int64_t)s] = k + 1;
        }
        if (off != ofs[l + 1] - ofs[l]) return fail(VBC_INVALID_ARG, "ofs inconsistent");
        T *seg = val + (ofs[l] - 1);
        for (int64_t j = j0; j < j1; j++)
            for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; p++) {
                const int64_t i = rowval[p] - 1, k = asg[i];
                seg[boff[k] + (i - (pspl[k] - 1)) * w + (j - j0)] = nzval[p];
            }
    }
    return VBC_OK;
}

}  // namespace

extern "C" {

int vbcx_partition_equi(int64_t n, int64_t w, int64_t *spl, int64_t *L)
{
    if (n < 0 || w < 1) return fail(VBC_INVALID_ARG, "EquiChunker: need n >= 0 and w >= 1");
    int64_t l = 0;
    for (int64_t j = 1; j <= n; j += w) spl[l++] = j;
    spl[l] = n + 1;
    *L = l;
    return VBC_OK;
}

int vbcx_partition_strict(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                          int64_t W, int64_t *spl, int64_t *L)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    if (W < 1) return fail(VBC_INVALID_ARG, "W must be > 0");
    int64_t l = 0, first = 0;
    for (int64_t j = 0; j < n; j++) {
        bool join = false;
        if (j > 0 && j - first < W) {
            const int64_t a0 = colptr[first] - 1, a1 = colptr[first + 1] - 1;
            const int64_t b0 = colptr[j] - 1, b1 = colptr[j + 1] - 1;
            join = (a1 - a0 == b1 - b0) && std::equal(rowval + a0, rowval + a1, rowval + b0);
        }
        if (!join) { spl[l++] = j + 1; first = j; }
    }
    spl[l] = n + 1;
    *L = l;
    return VBC_OK;
}

int vbcx_partition_overlap(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                           double rho, int64_t W, int64_t *spl, int64_t *L)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    if (W < 1 || !(rho >= 0.0 && rho <= 1.0)) return fail(VBC_INVALID_ARG, "need W > 0, 0 <= rho <= 1");
    std::vector<int64_t> stamp(m, -1);
    int64_t l = 0, first = 0, nfirst = 0;
    for (int64_t j = 0; j < n; j++) {
        const int64_t b0 = colptr[j] - 1, b1 = colptr[j + 1] - 1, nb = b1 - b0;
        bool join = false;
        if (j > 0 && j - first < W) {
            int64_t common = 0;
            for (int64_t p = b0; p < b1; p++) common += (stamp[rowval[p] - 1] == first);
            join = (double)common >= rho * (double)std::max(nb, nfirst);
        }
        if (!join) {
            spl[l++] = j + 1;
            first = j;
            nfirst = nb;
            for (int64_t p = b0; p < b1; p++) stamp[rowval[p] - 1] = first;
        }
    }
    spl[l] = n + 1;
    *L = l;
    return VBC_OK;
}

int vbcx_partition_dynamic(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                           int64_t W, double c_stripe, double c_col, double c_pin, double c_row,
                           double c_cell, int64_t *spl, int64_t *L)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    if (W < 1) return fail(VBC_INVALID_ARG, "W must be > 0");
    const double inf = std::numeric_limits<double>::infinity();
    std::vector<double> f(n + 1, inf);
    std::vector<int64_t> back(n + 1, 0), stamp(m, -1);
    f[0] = 0.0;
    for (int64_t e = 1; e <= n; e++) {
        int64_t rows = 0, pins = 0;
        for (int64_t w = 1; w <= W && w <= e; w++) {
            const int64_t j = e - w;  // add column j (0-based) to the stripe [j, e)
            for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; p++) {
                const int64_t i = rowval[p] - 1;
                if (stamp[i] != e) { stamp[i] = e; rows++; }
            }
            pins += colptr[j + 1] - colptr[j];
            const double c = c_stripe + c_col * w + c_pin * pins + c_row * rows + c_cell * w * rows;
            if (f[j] + c < f[e]) { f[e] = f[j] + c; back[e] = j; }  // ties keep the widest stripe
        }
    }
    std::vector<int64_t> cuts;
    for (int64_t e = n; e > 0; e = back[e]) cuts.push_back(back[e]);
    int64_t l = 0;
    for (auto it = cuts.rbegin(); it != cuts.rend(); ++it) spl[l++] = *it + 1;
    spl[l] = n + 1;
    *L = l;
    return VBC_OK;
}

int vbcx_partition_dynamic_table(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                                 int64_t W, const double *alpha, const double *beta, int64_t *spl, int64_t *L)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    if (W < 1 || !alpha || !beta) return fail(VBC_INVALID_ARG, "W must be > 0 with W alpha / beta entries");
    const double inf = std::numeric_limits<double>::infinity();
    std::vector<double> f(n + 1, inf);
    std::vector<int64_t> back(n + 1, 0), stamp(m, -1);
    f[0] = 0.0;
    for (int64_t e = 1; e <= n; e++) {
        int64_t rows = 0;
        for (int64_t w = 1; w <= W && w <= e; w++) {
            const int64_t j = e - w;  // add column j (0-based) to the stripe [j, e)
            for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; p++) {
                const int64_t i = rowval[p] - 1;
                if (stamp[i] != e) { stamp[i] = e; rows++; }
            }
            const double c = alpha[w - 1] + beta[w - 1] * (double)rows;
            if (f[j] + c < f[e]) { f[e] = f[j] + c; back[e] = j; }
        }
    }
    std::vector<int64_t> cuts;
    for (int64_t e = n; e > 0; e = back[e]) cuts.push_back(back[e]);
    int64_t l = 0;
    for (auto it = cuts.rbegin(); it != cuts.rend(); ++it) spl[l++] = *it + 1;
    spl[l] = n + 1;
    *L = l;
    return VBC_OK;
}

int vbcx_partition_block(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval, const int64_t *grp,
                         int64_t G, int64_t R, const double *gw, int64_t W, const double *alpha, const double *colw,
                         int64_t *spl, int64_t *L)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    if (W < 1 || R < 1 || R > 64 || !gw || !alpha || !colw)
        return fail(VBC_INVALID_ARG, "block cost model: need W > 0, 1 <= R <= 64 components and their tables");
    if (!grp && G != m) return fail(VBC_INVALID_ARG, "without a row grouping every row is its own group (G == m)");
    if (grp)
        for (int64_t i = 0; i < m; i++)
            if (grp[i] < 1 || grp[i] > G) return fail(VBC_INVALID_ARG, "row group id out of 1..G");
    const double inf = std::numeric_limits<double>::infinity();
    std::vector<double> f(n + 1, inf), S(R);
    std::vector<int64_t> back(n + 1, 0), stamp(std::max<int64_t>(G, 1), -1);
    f[0] = 0.0;
    for (int64_t e = 1; e <= n; e++) {
        std::fill(S.begin(), S.end(), 0.0);
        for (int64_t w = 1; w <= W && w <= e; w++) {
            const int64_t j = e - w;  // add column j (0-based) to the stripe [j, e)
            for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; p++) {
                const int64_t g = grp ? grp[rowval[p] - 1] - 1 : rowval[p] - 1;
                if (stamp[g] != e) {  // a block row the stripe did not touch yet: one more u x w block
                    stamp[g] = e;
                    for (int64_t r = 0; r < R; r++) S[r] += gw[r * G + g];
                }
            }
            double c = alpha[w - 1];
            for (int64_t r = 0; r < R; r++) c += colw[r * W + w - 1] * S[r];
            if (f[j] + c < f[e]) { f[e] = f[j] + c; back[e] = j; }
        }
    }
    std::vector<int64_t> cuts;
    for (int64_t e = n; e > 0; e = back[e]) cuts.push_back(back[e]);
    int64_t l = 0;
    for (auto it = cuts.rbegin(); it != cuts.rend(); ++it) spl[l++] = *it + 1;
    spl[l] = n + 1;
    *L = l;
    return VBC_OK;
}

int vbcx_1dvbc_count(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval, int64_t L,
                     const int64_t *spl, int64_t *pos, int64_t *ofs)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    if (int st = check_spl(n, L, spl, 0, false)) return st;
    // distinct rows per stripe (pos / ofs hold the counts until the prefix sum)
    int st = parallel_ranges(L, colptr[n] - 1, [&](int64_t l0, int64_t l1, int &) {
        std::vector<int64_t> rows, tmp;
        for (int64_t l = l0; l < l1; l++) {
            stripe_rows(colptr, rowval, spl[l] - 1, spl[l + 1] - 1, rows, tmp);
            pos[l + 1] = (int64_t)rows.size();
        }
    });
    if (st) return st;
    pos[0] = 1;
    ofs[0] = 1;
    for (int64_t l = 0; l < L; l++) {
        const int64_t rows = pos[l + 1];
        pos[l + 1] = pos[l] + rows;
        ofs[l + 1] = ofs[l] + rows * (spl[l + 1] - spl[l]);
    }
    return VBC_OK;
}

int vbcx_1dvbc_fill(int64_t m, int64_t n, int64_t W, const int64_t *colptr, const int64_t *rowval,
                    const void *nzval, int dtype, int64_t L, const int64_t *spl, const int64_t *pos,
                    const int64_t *ofs, int64_t *idx, void *val, int64_t pad)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    if (W < 1) return fail(VBC_INVALID_ARG, "W must be > 0");
    if (int st = check_spl(n, L, spl, W, true)) return st;
    if (pad < 0) return fail(VBC_INVALID_ARG, "pad must be >= 0");
    if (dtype == VBC_F64)
        return fill_1d(m, W, colptr, rowval, (const double *)nzval, L, spl, pos, ofs, idx,
                       (double *)val, pad);
    if (dtype == VBC_F32)
        return fill_1d(m, W, colptr, rowval, (const float *)nzval, L, spl, pos, ofs, idx,
                       (float *)val, pad);
    if (dtype == VBC_I64)
        return fill_1d(m, W, colptr, rowval, (const int64_t *)nzval, L, spl, pos, ofs, idx, (int64_t *)val, pad);
    if (dtype == VBC_I32)
        return fill_1d(m, W, colptr, rowval, (const int32_t *)nzval, L, spl, pos, ofs, idx, (int32_t *)val, pad);
    if (dtype == VBC_BOOL)
        return fill_1d(m, W, colptr, rowval, (const uint8_t *)nzval, L, spl, pos, ofs, idx, (uint8_t *)val, pad);
    return fail(VBC_UNSUPPORTED_DTYPE, "unknown dtype");
}

int vbcx_vbc_count(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval, int64_t K,
                   const int64_t *pspl, int64_t L, const int64_t *spl, int64_t *pos, int64_t *ofs)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    if (int st = check_spl(n, L, spl, 0, false)) return st;
    if (int st = check_spl(m, K, pspl, 0, false)) return st;
    std::vector<int64_t> asg(m), stamp(K, 0);
    for (int64_t k = 0; k < K; k++)
        for (int64_t i = pspl[k] - 1; i < pspl[k + 1] - 1; i++) asg[i] = k;
    pos[0] = 1;
    ofs[0] = 1;
    for (int64_t l = 0; l < L; l++) {
        const int64_t w = spl[l + 1] - spl[l];
        int64_t nb = 0, nv = 0;
        for (int64_t j = spl[l] - 1; j < spl[l + 1] - 1; j++)
            for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; p++) {
                const int64_t k = asg[rowval[p] - 1];
                if (stamp[k] != l + 1) {
                    stamp[k] = l + 1;
                    nb++;
                    nv += (pspl[k + 1] - pspl[k]) * w;
                }
            }
        pos[l + 1] = pos[l] + nb;
        ofs[l + 1] = ofs[l] + nv;
    }
    return VBC_OK;
}

int vbcx_vbc_fill(int64_t m, int64_t n, int64_t U, int64_t W, const int64_t *colptr,
                  const int64_t *rowval, const void *nzval, int dtype, int64_t K,
                  const int64_t *pspl, int64_t L, const int64_t *spl, const int64_t *pos,
                  const int64_t *ofs, int64_t *idx, void *val, int64_t pad)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    if (U < 1 || W < 1) return fail(VBC_INVALID_ARG, "U and W must be > 0");
    if (int st = check_spl(n, L, spl, W, true)) return st;
    if (int st = check_spl(m, K, pspl, U, true)) return st;
    if (pad < 0) return fail(VBC_INVALID_ARG, "pad must be >= 0");
    if (dtype == VBC_F64)
        return fill_2d(m, U, W, colptr, rowval, (const double *)nzval, K, pspl, L, spl, pos, ofs,
                       idx, (double *)val, pad);
    if (dtype == VBC_F32)
        return fill_2d(m, U, W, colptr, rowval, (const float *)nzval, K, pspl, L, spl, pos, ofs,
                       idx, (float *)val, pad);
    if (dtype == VBC_I64)
        return fill_2d(m, U, W, colptr, rowval, (const int64_t *)nzval, K, pspl, L, spl, pos, ofs, idx,
                       (int64_t *)val, pad);
    if (dtype == VBC_I32)
        return fill_2d(m, U, W, colptr, rowval, (const int32_t *)nzval, K, pspl, L, spl, pos, ofs, idx,
                       (int32_t *)val, pad);
    if (dtype == VBC_BOOL)
        return fill_2d(m, U, W, colptr, rowval, (const uint8_t *)nzval, K, pspl, L, spl, pos, ofs, idx,
                       (uint8_t *)val, pad);
    return fail(VBC_UNSUPPORTED_DTYPE, "unknown dtype");
}

int vbcx_transpose_pattern(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowval,
                           int64_t *rowptr, int64_t *colval)
{
    if (int st = check_csc(m, n, colptr, rowval)) return st;
    std::fill(rowptr, rowptr + m + 1, 0);
    for (int64_t p = 0; p < colptr[n] - 1; p++) rowptr[rowval[p]]++;
    rowptr[0] = 1;
    for (int64_t i = 0; i < m; i++) rowptr[i + 1] += rowptr[i];
    std::vector<int64_t> next(rowptr, rowptr + m);
    for (int64_t j = 0; j < n; j++)
        for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; p++)
            colval[(next[rowval[p] - 1]++) - 1] = j + 1;
    return VBC_OK;
}

}  // extern "C"
