// Probe 2: random-gather throughput vs memory-level parallelism (U independent gathers per lane in
// flight) and x size; plus the full stream+gather body at the same U.  Not part of the library.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void init_idx(int *idx, long n, unsigned m, unsigned long long seed)
{
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        unsigned long long z = i * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        idx[i] = (int)(z % m);
    }
}
__global__ void init_val(double *v, long n)
{
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) v[i] = 1.0 + (i & 7);
}

typedef double d2 __attribute__((ext_vector_type(2)));

// one lane per row (MODE 0: gather only, x[idx[r]]), or two lanes per w=4 row (MODE 1: full body)
template <int MODE, int U>
__global__ __launch_bounds__(256) void probe(const d2 *val, const int *idx, const double *x, long rows, double *out)
{
    double acc0 = 0, acc1 = 0;
    const long lanes = MODE == 0 ? rows : rows * 2;
    const long T = (long)gridDim.x * 256;
    for (long base = blockIdx.x * 256L + threadIdx.x; base < lanes; base += T * U) {
        int ii[U];
        d2 vv[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long t = base + u * T;
            const long r = MODE == 0 ? t : (t >> 1);
            ii[u] = t < lanes ? __builtin_nontemporal_load(idx + r) : 0;
            if (MODE == 1) vv[u] = t < lanes ? __builtin_nontemporal_load(val + t) : d2{0, 0};
        }
        double xx[U];
#pragma unroll
        for (int u = 0; u < U; u++) xx[u] = x[ii[u]];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (MODE == 0) acc0 += xx[u];
            else { acc0 = __builtin_fma(vv[u].x, xx[u], acc0); acc1 = __builtin_fma(vv[u].y, xx[u], acc1); }
        }
    }
    if (acc0 + acc1 == 12345.678) out[0] = acc0;
}

int main()
{
    const long rows = 25000000;
    d2 *val;
    int *idx;
    double *x, *out;
    const long xmax = 10000000;
    CK(hipMalloc(&val, rows * 32));
    CK(hipMalloc(&idx, rows * 4));
    CK(hipMalloc(&x, xmax * 8));
    CK(hipMalloc(&out, 8));
    init_val<<<4096, 256>>>((double *)val, rows * 4);
    init_val<<<4096, 256>>>(x, xmax);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto kern, int grid, const char *name, long m, double bytes) {
        for (int i = 0; i < 3; i++) kern<<<grid, 256>>>(val, idx, x, rows, out);
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; i++) kern<<<grid, 256>>>(val, idx, x, rows, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-22s m=%-9ld grid=%-6d %8.1f us  %6.1f Ggather/s  %7.0f GB/s alg\n", name, m, grid, ms * 1e3,
               rows / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e9);
    };
    for (long m : {10000000L, 4000000L, 1000000L, 250000L}) {
        init_idx<<<4096, 256>>>(idx, rows, (unsigned)m, 12345);
        CK(hipDeviceSynchronize());
        printf("--- m=%ld (%.0f MB)\n", m, m * 8 / 1e6);
        const double gb = rows * 4.0 + m * 8.0, fb = rows * 36.0 + m * 8.0;
        for (int g : {2048, 8192}) {
            timeit(probe<0, 1>, g, "gather U1", m, gb);
            timeit(probe<0, 4>, g, "gather U4", m, gb);
            timeit(probe<0, 8>, g, "gather U8", m, gb);
            timeit(probe<0, 16>, g, "gather U16", m, gb);
            timeit(probe<1, 1>, g, "full U1", m, fb);
            timeit(probe<1, 4>, g, "full U4", m, fb);
            timeit(probe<1, 8>, g, "full U8", m, fb);
        }
    }
    return 0;
}
