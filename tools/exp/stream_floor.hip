// Floor of a small streaming product in a graph replay: how long does one launch that reads B bytes
// (16 B per lane per load, all loads of a wave issued together) take, against an empty launch, with
// and without kernel-argument preloading (scalar args only are preloaded on gfx950).
// Build: hipcc --offload-arch=gfx950 -O3 [-mllvm -amdgpu-kernarg-preload-count=16] stream_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_empty(float *y) {}
__global__ void k_one(const float *a, float *y) { if (threadIdx.x == 0 && blockIdx.x == 0) y[0] = a[0] + 1.f; }

// Each wave reads NL consecutive 1 KB blocks (16 B per lane) starting at its own offset, folds, stores one float4.
typedef float f4v __attribute__((ext_vector_type(4)));
template <int NL, bool NT = false>
__global__ __launch_bounds__(64) void k_stream(const float4 *__restrict__ a, float4 *__restrict__ y, int nw) {
    int w = blockIdx.x;
    if (w >= nw) return;
    const float4 *p = a + (size_t)w * NL * 64 + threadIdx.x;
    float4 v[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        if constexpr (NT) {
            f4v t = __builtin_nontemporal_load((const f4v *)(p + i * 64));
            v[i] = make_float4(t.x, t.y, t.z, t.w);
        } else v[i] = p[i * 64];
    }
    float4 s = v[0];
#pragma unroll
    for (int i = 1; i < NL; ++i) { s.x += v[i].x; s.y += v[i].y; s.z += v[i].z; s.w += v[i].w; }
    y[(size_t)w * 64 + threadIdx.x] = s;
}

// Same with a dependent second round (an index loaded first, then the data): the planar product's
// keys -> gathers chain.
template <int NL>
__global__ __launch_bounds__(64) void k_stream2(const float4 *__restrict__ a, const int *__restrict__ idx, float4 *__restrict__ y, int nw) {
    int w = blockIdx.x;
    if (w >= nw) return;
    const float4 *p = a + (size_t)w * NL * 64 + threadIdx.x;
    float4 v[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) v[i] = p[i * 64];
    int j = idx[(size_t)w * 64 + threadIdx.x];
    float4 g = a[j];
    float4 s = g;
#pragma unroll
    for (int i = 0; i < NL; ++i) { s.x += v[i].x; s.y += v[i].y; s.z += v[i].z; s.w += v[i].w; }
    y[(size_t)w * 64 + threadIdx.x] = s;
}

template <class F>
static double replay(F launch, hipStream_t st, int reps) {
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
    double best = 1e30;
    for (int t = 0; t < 5; ++t) {
        CK(hipEventRecord(e0, st)); CK(hipGraphLaunch(ge, st)); CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms * 1e3 / reps);
    }
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    return best;
}

int main() {
    hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    size_t big = 256ull << 20;
    float4 *a, *y; int *idx;
    CK(hipMalloc(&a, big)); CK(hipMalloc(&y, big)); CK(hipMalloc(&idx, big / 4));
    CK(hipMemset(a, 0, big)); CK(hipMemset(y, 0, big));
    std::vector<int> h(big / 16 / 4);
    srand(1); for (auto &v : h) v = rand() % (int)(big / 16 / 8);
    CK(hipMemcpy(idx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    const int R = 200;
    printf("empty   %.2f us\n", replay([&] { k_empty<<<1, 64, 0, st>>>((float *)y); }, st, R));
    printf("one     %.2f us\n", replay([&] { k_one<<<1, 64, 0, st>>>((float *)a, (float *)y); }, st, R));
    for (double mb : {6.0, 12.0, 25.0, 40.0, 52.0, 100.0}) {
        size_t bytes = (size_t)(mb * 1e6);
#define RUN(NL) do { int nw = (int)(bytes / (NL * 1024)); \
        double t1 = replay([&] { k_stream<NL><<<nw, 64, 0, st>>>(a, y, nw); }, st, R); \
        double t2 = replay([&] { k_stream2<NL><<<nw, 64, 0, st>>>(a, idx, y, nw); }, st, R); \
        double t3 = replay([&] { k_stream<NL, true><<<nw, 64, 0, st>>>(a, y, nw); }, st, R); \
        printf("%5.0f MB  NL=%2d waves=%6d  stream %.2f us (%.0f GB/s)  nontemporal %.2f us  +dependent gather %.2f us\n", mb, NL, nw, t1, bytes / t1 / 1e3, t3, t2); } while (0)
        RUN(2); RUN(4); RUN(6); RUN(8); RUN(12); RUN(16); RUN(32);
    }
    return 0;
}
