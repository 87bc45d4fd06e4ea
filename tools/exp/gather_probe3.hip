// Probe 3 (round 4): where do NS's x-gather misses come from?  Random 8-B gathers
// (indices hashed on the fly, so the only memory traffic is the gathers themselves) from tables of
// 2 MB (L2-resident), 80 MB (NS's fp64 x: Infinity-Cache-resident), 1 GB and 4 GB (far beyond the
// 256 MB Infinity Cache: every miss goes to HBM).  If the gather rate from the 80 MB table equals
// the HBM-resident ones, the NS kernel is bound by the L2 miss request rate whatever serves it; if
// it is well above, NS's misses are served by the Infinity Cache and its HBM bytes are ~algorithmic.
// Also: the same gathers interleaved with a 1 GB non-temporal stream (NS's mix).  Not library code.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void init_val(double *v, long n)
{
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) v[i] = 1.0 + (i & 7);
}

typedef double d2 __attribute__((ext_vector_type(2)));

// G gathers per lane, U in flight; STREAM: each lane also streams 32 B per gather (NS: 4 values per row)
template <int U, bool STREAM>
__global__ __launch_bounds__(256) void probe(const double *x, unsigned long long m, long gathers, const d2 *s,
                                             long srows, double *out, unsigned long long seed)
{
    double acc = 0;
    const long T = (long)gridDim.x * 256;
    for (long base = blockIdx.x * 256L + threadIdx.x; base < gathers; base += T * U) {
        double xx[U];
        d2 vv[U][2];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long t = base + u * T;
            const unsigned long long i = mix((unsigned long long)t * 0x9E3779B97F4A7C15ull + seed) % m;
            xx[u] = x[i];
            if (STREAM) {
                const long r = (t % srows) * 2;
                vv[u][0] = __builtin_nontemporal_load(s + r);
                vv[u][1] = __builtin_nontemporal_load(s + r + 1);
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            acc += xx[u];
            if (STREAM) acc += vv[u][0].x * vv[u][1].y;
        }
    }
    if (acc == 12345.678) out[0] = acc;
}

int main(int argc, char **argv)
{
    // gather_probe3 [table_elems grid stream]: one configuration only (for rocprofv3 --pmc passes)
    const bool one = argc >= 4;
    const long gathers = 25000000;  // NS: 2.5e7 stored rows -> 2.5e7 x gathers per product
    const long tmax = 4L << 30;     // 4 GB table
    const long srows = 31250000;    // 1 GB stream (32 B per row)
    double *x, *out;
    d2 *s;
    CK(hipMalloc(&x, tmax));
    CK(hipMalloc(&s, srows * 32));
    CK(hipMalloc(&out, 8));
    init_val<<<8192, 256>>>(x, tmax / 8);
    init_val<<<8192, 256>>>((double *)s, srows * 4);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto kern, int grid, const char *name, unsigned long long m) {
        for (int i = 0; i < 3; i++) kern<<<grid, 256>>>(x, m, gathers, s, srows, out, 7 + i);
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; i++) kern<<<grid, 256>>>(x, m, gathers, s, srows, out, 100 + i);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-16s table %8.1f MB grid %-6d %8.1f us  %6.1f G gathers/s\n", name, m * 8 / 1e6, grid, ms * 1e3,
               gathers / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    if (one) {
        const unsigned long long m = strtoull(argv[1], nullptr, 10);
        const int g = atoi(argv[2]);
        if (atoi(argv[3])) timeit(probe<8, true>, g, "gather+stream U8", m);
        else timeit(probe<8, false>, g, "gather U8", m);
        return 0;
    }
    for (unsigned long long m : {262144ull, 10000000ull, 125000000ull, 500000000ull}) {
        for (int g : {4096, 16384}) {
            timeit(probe<8, false>, g, "gather U8", m);
            timeit(probe<16, false>, g, "gather U16", m);
            timeit(probe<8, true>, g, "gather+stream U8", m);
        }
    }
    return 0;
}
