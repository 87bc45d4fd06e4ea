// libvbc generic-eltype paths: exact integer products and eltype / stride conversions.
//
// The reference's kernels are generic in Tv and compute in eltype(y) (multiply_1DVBC.jl:27,34,102:
// `convert(Vec{$w, eltype(y)}, vload(Vec{$w, Tv}, A_val, q)) * convert(eltype(y), x[...])`), and its
// tests run Bool and Int32 matrices (runtests.jl:15-16).  Integer eltypes are computed here in 64-bit
// two's-complement wrapping arithmetic: Julia's Int64 arithmetic exactly, and -- after truncation --
// Julia's Int32 arithmetic exactly too (wrapping mod 2^64 then mod 2^32 equals wrapping mod 2^32).
// Wrapping addition is associative, so the forward product's atomic accumulation is bit-exact and
// run-to-run deterministic.  These kernels are not bandwidth-tuned: floating-point eltypes (the
// benchmarked path) run the slotted / swept / merge kernels.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "vbc_handle.h"

namespace vbc {

// mul!(y, B', x): one lane per output column j (of stripe l = col2stripe[j]), rows in stored order.
__global__ __launch_bounds__(256) void int_spmv_t(IntLayout lay, const int64_t *__restrict__ x,
                                                  int64_t *__restrict__ y, int64_t n, uint64_t alpha,
                                                  uint64_t beta, int rd)
{
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int32_t l = lay.col2stripe[j];
    const int64_t w = lay.w[l], c = j - lay.col0[l];
    const int64_t r0 = lay.rbeg[l], r1 = lay.rbeg[l + 1];
    const int64_t *v = lay.val + lay.voff[l] + c;
    uint64_t acc = 0;
    for (int64_t r = r0; r < r1; r++) acc += (uint64_t)v[(r - r0) * w] * (uint64_t)x[lay.rows[r]];
    uint64_t out = alpha * acc;
    if (rd) out += beta * (uint64_t)y[j];
    y[j] = (int64_t)out;
}

__global__ __launch_bounds__(256) void int_scale(int64_t *__restrict__ y, int64_t m, uint64_t beta, int rd)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) y[i] = rd ? (int64_t)(beta * (uint64_t)y[i]) : 0;
}

// mul!(y, B, x): one lane per stored row, dot with the stripe's x slice, wrapping atomic add.
__global__ __launch_bounds__(256) void int_spmv_f(IntLayout lay, const int64_t *__restrict__ x,
                                                  int64_t *__restrict__ y, uint64_t alpha)
{
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= lay.nrows) return;
    const int32_t l = lay.row2stripe[r];
    const int64_t w = lay.w[l];
    const int64_t *v = lay.val + lay.voff[l] + (r - lay.rbeg[l]) * w;
    const int64_t *xs = x + lay.col0[l];
    uint64_t dot = 0;
    for (int64_t c = 0; c < w; c++) dot += (uint64_t)v[c] * (uint64_t)xs[c];
    atomicAdd(reinterpret_cast<unsigned long long *>(y + lay.rows[r]), (unsigned long long)(alpha * dot));
}

int mul_int(const vbc_handle *h, int trans, const void *x, void *y, double alpha, double beta, hipStream_t s)
{
    const uint64_t a = (uint64_t)(int64_t)alpha, b = (uint64_t)(int64_t)beta;
    const IntLayout &lay = h->li;
    const int64_t *xs = static_cast<const int64_t *>(x);
    int64_t *ys = static_cast<int64_t *>(y);
    if (trans) {
        if (h->n == 0) return VBC_OK;
        hipLaunchKernelGGL(int_spmv_t, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, s, lay, xs, ys, h->n, a, b,
                           (int)(beta != 0.0));
    } else {
        if (h->m == 0) return VBC_OK;
        hipLaunchKernelGGL(int_scale, dim3((unsigned)((h->m + 255) / 256)), dim3(256), 0, s, ys, h->m, b,
                           (int)(beta != 0.0));
        if (lay.nrows > 0)
            hipLaunchKernelGGL(int_spmv_f, dim3((unsigned)((lay.nrows + 255) / 256)), dim3(256), 0, s, lay, xs, ys, a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("integer product launch failed: %s", hipGetErrorString(e));
        return VBC_HIP_ERROR;
    }
    return VBC_OK;
}

// ---------------------------------------------------------------------------------------------
// Eltype / stride conversion between a caller's StridedVector and a contiguous compute-eltype
// buffer (x: convert(eltype(y), x[i]); y: the result stored back, Int64 -> Int32 by truncation).
// ---------------------------------------------------------------------------------------------
template <typename Ti, typename To>
__global__ __launch_bounds__(256) void cvt_gather(const Ti *__restrict__ src, int64_t inc, To *__restrict__ dst, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = (To)src[i * inc];
}

template <typename Ti, typename To>
__global__ __launch_bounds__(256) void cvt_scatter(const Ti *__restrict__ src, To *__restrict__ dst, int64_t inc, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i * inc] = (To)src[i];
}

template <typename Ti>
static hipError_t gather_to(const void *src, int64_t inc, int out_dtype, void *dst, int64_t n, hipStream_t s)
{
    const dim3 g((unsigned)((n + 255) / 256)), b(256);
    const Ti *p = static_cast<const Ti *>(src);
    switch (out_dtype) {
    case VBC_F64: hipLaunchKernelGGL((cvt_gather<Ti, double>), g, b, 0, s, p, inc, static_cast<double *>(dst), n); break;
    case VBC_F32: hipLaunchKernelGGL((cvt_gather<Ti, float>), g, b, 0, s, p, inc, static_cast<float *>(dst), n); break;
    case VBC_I64: hipLaunchKernelGGL((cvt_gather<Ti, int64_t>), g, b, 0, s, p, inc, static_cast<int64_t *>(dst), n); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int convert_gather(const void *src, int src_dtype, int64_t inc, void *dst, int dst_dtype, int64_t n, hipStream_t s)
{
    if (n <= 0) return VBC_OK;
    hipError_t e;
    switch (src_dtype) {
    case VBC_F64: e = gather_to<double>(src, inc, dst_dtype, dst, n, s); break;
    case VBC_F32: e = gather_to<float>(src, inc, dst_dtype, dst, n, s); break;
    case VBC_I64: e = gather_to<int64_t>(src, inc, dst_dtype, dst, n, s); break;
    case VBC_I32: e = gather_to<int32_t>(src, inc, dst_dtype, dst, n, s); break;
    case VBC_BOOL: e = gather_to<uint8_t>(src, inc, dst_dtype, dst, n, s); break;
    default: return fail(VBC_UNSUPPORTED_DTYPE, "unknown eltype");
    }
    if (e != hipSuccess) {
        set_error("eltype conversion failed: %s", hipGetErrorString(e));
        return VBC_HIP_ERROR;
    }
    return VBC_OK;
}

int convert_scatter(const void *src, int src_dtype, void *dst, int dst_dtype, int64_t inc, int64_t n, hipStream_t s)
{
    if (n <= 0) return VBC_OK;
    const dim3 g((unsigned)((n + 255) / 256)), b(256);
    if (src_dtype == VBC_F64 && dst_dtype == VBC_F64)
        hipLaunchKernelGGL((cvt_scatter<double, double>), g, b, 0, s, static_cast<const double *>(src), static_cast<double *>(dst), inc, n);
    else if (src_dtype == VBC_F32 && dst_dtype == VBC_F32)
        hipLaunchKernelGGL((cvt_scatter<float, float>), g, b, 0, s, static_cast<const float *>(src), static_cast<float *>(dst), inc, n);
    else if (src_dtype == VBC_I64 && dst_dtype == VBC_I64)
        hipLaunchKernelGGL((cvt_scatter<int64_t, int64_t>), g, b, 0, s, static_cast<const int64_t *>(src), static_cast<int64_t *>(dst), inc, n);
    else if (src_dtype == VBC_I64 && dst_dtype == VBC_I32)
        hipLaunchKernelGGL((cvt_scatter<int64_t, int32_t>), g, b, 0, s, static_cast<const int64_t *>(src), static_cast<int32_t *>(dst), inc, n);
    else
        return fail(VBC_UNSUPPORTED_DTYPE, "no conversion for this y eltype");
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("eltype conversion failed: %s", hipGetErrorString(e));
        return VBC_HIP_ERROR;
    }
    return VBC_OK;
}

}  // namespace vbc
