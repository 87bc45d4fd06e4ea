// Memory-system probe for the NS-1DVBC transposed product (not part of the library).
// Times, on synthetic data shaped like the NS workload (q = 2.5e7 rows of w = 4 fp64, random x rows):
//   stream   : val (16 B/lane) + idx only, no x gather
//   gather   : idx + x[idx] only
//   full     : acc += val * x[idx]  (element-level SpMV body, no segments)
// for several x sizes and load policies.  hipcc --offload-arch=gfx950 -O3 gather_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void init_idx(int *idx, long n, unsigned m, unsigned long long seed, int sorted_runs)
{
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        unsigned long long z = (i / (sorted_runs ? sorted_runs : 1)) * 0x9E3779B97F4A7C15ull + seed;
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
template <int NT>
__device__ __forceinline__ double2 ldv(const double2 *p)
{
    d2 t = NT ? __builtin_nontemporal_load((const d2 *)p) : *(const d2 *)p;
    return double2(t.x, t.y);
}
template <int NT>
__device__ __forceinline__ int ldi(const int *p)
{
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// rows of w=4 doubles: 2 lanes per row, lane holds 2 doubles.
template <int MODE, int NT>
__global__ __launch_bounds__(256) void probe(const double2 *val, const int *idx, const double *x, long rows, double *out)
{
    double a0 = 0, a1 = 0;
    const long nlanes = rows * 2;
    for (long t = blockIdx.x * 256L + threadIdx.x; t < nlanes; t += (long)gridDim.x * 256) {
        const long r = t >> 1;
        if (MODE == 0) {  // stream
            const double2 v = ldv<NT>(val + t);
            const int i = ldi<NT>(idx + r);
            a0 += v.x + (double)i;
            a1 += v.y;
        } else if (MODE == 1) {  // gather only
            const int i = ldi<NT>(idx + r);
            a0 += x[i];
        } else {  // full
            const double2 v = ldv<NT>(val + t);
            const int i = ldi<NT>(idx + r);
            const double xv = x[i];
            a0 = __builtin_fma(v.x, xv, a0);
            a1 = __builtin_fma(v.y, xv, a1);
        }
    }
    if (a0 + a1 == 12345.678) out[0] = a0;  // keep live
}

int main()
{
    const long rows = 25000000;  // q
    const long nval = rows * 4;
    double2 *val;
    int *idx;
    double *x, *out;
    const long xmax = 10000000;
    CK(hipMalloc(&val, nval * 8));
    CK(hipMalloc(&idx, rows * 4));
    CK(hipMalloc(&x, xmax * 8));
    CK(hipMalloc(&out, 8));
    init_val<<<4096, 256>>>((double *)val, nval);
    init_val<<<4096, 256>>>(x, xmax);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const double bytes_stream = nval * 8.0 + rows * 4.0;
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
        printf("%-28s m=%-9ld grid=%-6d %8.1f us  %7.0f GB/s (alg bytes %.0f MB)\n", name, m, grid, ms * 1e3,
               bytes / (ms * 1e-3) / 1e9, bytes / 1e6);
    };
    const long ms_[] = {10000000, 1000000, 100000};
    const int grids[] = {prop.multiProcessorCount * 8, prop.multiProcessorCount * 32};
    for (int runs : {0, 10}) {
        for (long m : ms_) {
            init_idx<<<4096, 256>>>(idx, rows, (unsigned)m, 12345, runs);
            CK(hipDeviceSynchronize());
            printf("--- x rows m=%ld (%.0f MB), idx %s\n", m, m * 8 / 1e6, runs ? "runs of 10 equal" : "uniform");
            for (int g : grids) {
                timeit(probe<0, 1>, g, "stream nt", m, bytes_stream);
                timeit(probe<0, 0>, g, "stream plain", m, bytes_stream);
                timeit(probe<1, 1>, g, "gather (idx nt)", m, rows * 4.0 + m * 8.0);
                timeit(probe<2, 1>, g, "full nt", m, bytes_stream + m * 8.0);
                timeit(probe<2, 0>, g, "full plain", m, bytes_stream + m * 8.0);
            }
        }
    }
    return 0;
}
