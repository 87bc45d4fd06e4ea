// Vector-memory issue cost by access shape (gfx950): each wave issues N loads of one shape from an
// L2-resident table (4 MB), so time measures the CU's address / data path, not HBM.  Shapes:
//   0 dword, 64 lanes contiguous (256 B)            1 dword, 4 groups of 16 lanes, 64 B each at random lines
//   2 dwordx4, 64 lanes contiguous (1 KB)           3 dwordx4, 4 groups of 4 lanes (64 B) at random lines,
//                                                     other lanes idle (16 lanes active)
//   4 dwordx3, 4 groups of 16 lanes (192 B each) at random 192-B blocks
//   5 dwordx4, 4 groups of 12 lanes (192 B each) at random blocks, 16 lanes idle
//   6 dword, every lane the same address in its group of 16 (broadcast), 4 groups
//   7 dwordx3 broadcast (16 lanes same 12 B), 4 groups
//   8 dwordx4, 16 groups of 4 lanes (64 B each) at random lines (all 64 lanes: a planar tile row's X rows)
//   9 dwordx3, 48 lanes, 576 B contiguous (16 tiles' 3 x 3 values, lanes q < 3 of each group of 4)
//  10 dword, 16 groups of 4 lanes reading the same 4 B, 64 B contiguous (16 keys, each read by 4 lanes)
//  11 dwordx4, 64 lanes contiguous 1 KB STORE (16 stripes' outputs)
//  12 16 B per lane at its own random 24-B run (8-B aligned: x0, x1 of a fp64 3-dof gather)
//  13 8 B per lane at its own random 24-B run + 16 (x2 of the same gather)
//  14 16 B per lane, lane pairs on one random 24-B run (offsets 0 and 8: a cooperative 3-dof gather)
// Prints ns per load instruction per CU (all waves of the chip together).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hash(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

template <int SHAPE>
__global__ __launch_bounds__(256) void probe(const float *__restrict__ t, uint32_t nlines, int iters, float *out)
{
    const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
    const uint32_t wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    float acc = 0.f;
    typedef float f3 __attribute__((ext_vector_type(3)));
    typedef float f4 __attribute__((ext_vector_type(4)));
    const uint32_t base = hash(wid * 7919u + g * 31u), base0 = hash(wid * 7919u);
    for (int it = 0; it < iters; it += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t h = base + (uint32_t)(it + u) * 40503u;  // line index (masked below: nlines is 2^k)
            if constexpr (SHAPE == 0) {
                acc += t[(size_t)(((base0 + (uint32_t)(it + u) * 40503u) & (nlines / 4 - 1))) * 64 + lane];
            } else if constexpr (SHAPE == 1) {
                acc += t[(size_t)(h & (nlines - 1)) * 16 + j];
            } else if constexpr (SHAPE == 2) {
                const f4 v = *(const f4 *)(t + (size_t)(((base0 + (uint32_t)(it + u) * 40503u) & (nlines / 16 - 1))) * 256 + lane * 4);
                acc += v.x + v.w;
            } else if constexpr (SHAPE == 3) {
                if (j < 4) {
                    const f4 v = *(const f4 *)(t + (size_t)(h & (nlines - 1)) * 16 + j * 4);
                    acc += v.x + v.w;
                }
            } else if constexpr (SHAPE == 4) {
                const f3 v = *(const f3 *)(t + (size_t)(h & (nlines / 4 - 1)) * 48 + j * 3);
                acc += v.x + v.z;
            } else if constexpr (SHAPE == 5) {
                if (j < 12) {
                    const f4 v = *(const f4 *)(t + (size_t)(h & (nlines / 4 - 1)) * 48 + j * 4);
                    acc += v.x + v.w;
                }
            } else if constexpr (SHAPE == 6) {
                acc += t[(size_t)(h & (nlines - 1)) * 16];
            } else if constexpr (SHAPE == 7) {
                const f3 v = *(const f3 *)(t + (size_t)(h & (nlines - 1)) * 16);
                acc += v.x + v.z;
            } else if constexpr (SHAPE == 8) {
                const uint32_t h16 = hash(wid * 7919u + (lane >> 2) * 31u) + (uint32_t)(it + u) * 40503u;
                const f4 v = *(const f4 *)(t + (size_t)(h16 & (nlines - 1)) * 16 + (lane & 3) * 4);
                acc += v.x + v.w;
            } else if constexpr (SHAPE == 9) {
                if ((lane & 3) < 3) {
                    const f3 v = *(const f3 *)(t + (size_t)(((base0 + (uint32_t)(it + u) * 40503u) & (nlines / 16 - 1))) * 256 +
                                               (lane >> 2) * 9 + (lane & 3) * 3);
                    acc += v.x + v.z;
                }
            } else if constexpr (SHAPE == 10) {
                acc += t[(size_t)(((base0 + (uint32_t)(it + u) * 40503u) & (nlines - 1))) * 16 + (lane >> 2)];
            } else if constexpr (SHAPE == 12 || SHAPE == 13 || SHAPE == 14) {
                struct __attribute__((packed, aligned(8))) d2 { double a, b; };
                const uint32_t hr = SHAPE == 14 ? hash(wid * 7919u + (lane >> 1) * 31u) + (uint32_t)(it + u) * 40503u
                                                : hash(wid * 7919u + lane * 31u) + (uint32_t)(it + u) * 40503u;
                const char *run = (const char *)t + (size_t)(hr & 0x1FFFFu) * 24;
                if constexpr (SHAPE == 13) {
                    acc += (float)*(const double *)(run + 16);
                } else {
                    const d2 v = *(const d2 *)(run + (SHAPE == 14 ? (lane & 1) * 8 : 0));
                    acc += (float)(v.a + v.b);
                }
            } else {
                f4 *o = (f4 *)(out + 64 + (size_t)(((base0 + (uint32_t)(it + u) * 40503u) & (1023u))) * 256) + lane;
                *o = f4{acc, acc, acc, acc};
            }
        }
    }
    if (acc == 123.456f) out[0] = acc;
}

template <int S>
static float run(const float *t, uint32_t nlines, int iters, float *out, int grid)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(probe<S>, dim3(grid), dim3(256), 0, 0, t, nlines, iters, out);
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(probe<S>, dim3(grid), dim3(256), 0, 0, t, nlines, iters, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

int main()
{
    const size_t bytes = 4 << 20;  // L2-resident
    float *t, *out;
    CHECK(hipMalloc(&t, bytes + 4096));
    CHECK(hipMalloc(&out, 64 * 4 + 1024 * 1024 + 4096));
    CHECK(hipMemset(t, 0, bytes + 4096));
    const uint32_t nlines = bytes / 64;
    int cus = 256;
    const int grid = cus * 8;  // 32 waves per CU
    const int iters = 512;
    const char *names[] = {"dword contiguous 256 B", "dword 4 x 64 B random", "dwordx4 contiguous 1 KB",
                           "dwordx4 4 x 64 B (16 lanes)", "dwordx3 4 x 192 B", "dwordx4 4 x 192 B (48 lanes)",
                           "dword broadcast x4 groups", "dwordx3 broadcast x4 groups", "dwordx4 16 x 64 B random",
                           "dwordx3 48 lanes 576 B contiguous", "dword 16 x 4 B, 4 lanes each", "dwordx4 store 1 KB",
                           "16 B, 64 random 24-B runs", "8 B, 64 random 24-B runs + 16", "16 B, 32 runs, lane pairs"};
    float ms[15];
    ms[0] = run<0>(t, nlines, iters, out, grid);
    ms[1] = run<1>(t, nlines, iters, out, grid);
    ms[2] = run<2>(t, nlines, iters, out, grid);
    ms[3] = run<3>(t, nlines, iters, out, grid);
    ms[4] = run<4>(t, nlines, iters, out, grid);
    ms[5] = run<5>(t, nlines, iters, out, grid);
    ms[6] = run<6>(t, nlines, iters, out, grid);
    ms[7] = run<7>(t, nlines, iters, out, grid);
    ms[8] = run<8>(t, nlines, iters, out, grid);
    ms[9] = run<9>(t, nlines, iters, out, grid);
    ms[10] = run<10>(t, nlines, iters, out, grid);
    ms[11] = run<11>(t, nlines, iters, out, grid);
    ms[12] = run<12>(t, nlines, iters, out, grid);
    ms[13] = run<13>(t, nlines, iters, out, grid);
    ms[14] = run<14>(t, nlines, iters, out, grid);
    const double per_cu = (double)grid * 4 * iters / cus;  // wave-instructions per CU
    for (int s = 0; s < 15; s++)
        printf("shape %d %-32s %8.3f ms  %6.2f cycles/instr/CU at 2.4 GHz\n", s, names[s], ms[s],
               ms[s] * 1e-3 * 2.4e9 / per_cu);
    return 0;
}
