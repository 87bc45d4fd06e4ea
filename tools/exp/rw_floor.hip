// Floor of the FE headline's traffic mix on one MI355X: 1.0e9 B of streamed reads (16 B per lane, U
// loads of 1 KB per wave in flight, two stages as the slotted kernel) with and without the product's
// 8 % of contiguous writes, written every NB KB-rows as one burst per wave (the LDS-staged y runs of
// spmv_slots).  Build: hipcc --offload-arch=gfx950 -O3 -o rw_floor rw_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

// Each wave streams rows [r0, r1) of 1 KB (64 lanes x 16 B); every WR rows (WR = 0: never) it writes
// one 1 KB row of y (write ratio 1 / WR), in bursts of NB rows.
template <int U, int WR, int NB, bool NT>
__global__ __launch_bounds__(256) void k_rw(const d2 *__restrict__ a, d2 *__restrict__ y, int rows_per_wave, int nw)
{
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nw) return;
    const int lane = threadIdx.x & 63;
    const d2 *p = a + (size_t)w * rows_per_wave * 64 + lane;
    d2 *q = y + (size_t)w * (WR ? rows_per_wave / WR + NB : 1) * 64 + lane;
    d2 acc = {0, 0}, buf[NB > 0 ? NB : 1];
    int nb = 0, since = 0;
    d2 vA[U], vB[U];
#pragma unroll
    for (int u = 0; u < U; u++) vA[u] = NT ? __builtin_nontemporal_load(p + u * 64) : p[u * 64];
    for (int r = 0; r < rows_per_wave; r += 2 * U) {
#pragma unroll
        for (int u = 0; u < U; u++) vB[u] = NT ? __builtin_nontemporal_load(p + (r + U + u) * 64) : p[(r + U + u) * 64];
#pragma unroll
        for (int u = 0; u < U; u++) acc = acc * vA[u] + vA[u];
        if (WR) {
            since += U;
            if (since >= WR) {
                since -= WR;
                buf[nb++ % (NB > 0 ? NB : 1)] = acc;
                if (nb % NB == 0) {
#pragma unroll
                    for (int i = 0; i < NB; i++) q[i * 64] = buf[i];
                    q += NB * 64;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) vA[u] = NT ? __builtin_nontemporal_load(p + (r + 2 * U + u) * 64) : p[(r + 2 * U + u) * 64];
#pragma unroll
        for (int u = 0; u < U; u++) acc = acc * vB[u] + vB[u];
        if (WR) {
            since += U;
            if (since >= WR) {
                since -= WR;
                buf[nb++ % (NB > 0 ? NB : 1)] = acc;
                if (nb % NB == 0) {
#pragma unroll
                    for (int i = 0; i < NB; i++) q[i * 64] = buf[i];
                    q += NB * 64;
                }
            }
        }
    }
    if (!WR) q[0] = acc;
}

template <int U, int WR, int NB, bool NT>
static void run(const char *name, const d2 *a, d2 *y, size_t bytes, int rows_per_wave)
{
    const size_t rows = bytes / 1024;
    const int nw = (int)(rows / rows_per_wave);
    const int blocks = (nw + 3) / 4;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) k_rw<U, WR, NB, NT><<<blocks, 256>>>(a, y, rows_per_wave, nw);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; i++) k_rw<U, WR, NB, NT><<<blocks, 256>>>(a, y, rows_per_wave, nw);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    const double rb = (double)nw * rows_per_wave * 1024, wb = WR ? rb / WR : 0;
    printf("%-34s rows/wave %5d waves %7d  %7.1f us  read %6.0f GB/s  read+write %6.0f GB/s\n", name, rows_per_wave,
           nw, us, rb / us / 1e3, (rb + wb) / us / 1e3);
}

int main()
{
    const size_t bytes = 1006ull << 20;  // the FE product's read bytes (PMC: 1.006e9 of 1.086e9)
    d2 *a, *y;
    CK(hipMalloc(&a, bytes + (1 << 20)));
    CK(hipMalloc(&y, bytes / 4));
    CK(hipMemset(a, 0, bytes + (1 << 20)));
    for (int rpw : {384, 768, 1536}) {
        run<8, 0, 1, true>("read only, nt", a, y, bytes, rpw);
        run<8, 0, 1, false>("read only, cached", a, y, bytes, rpw);
        run<8, 12, 8, true>("read + 1/12 writes, bursts of 8", a, y, bytes, rpw);
        run<8, 12, 1, true>("read + 1/12 writes, single rows", a, y, bytes, rpw);
        run<8, 12, 16, true>("read + 1/12 writes, bursts of 16", a, y, bytes, rpw);
        run<4, 12, 8, true>("U=4 read + 1/12 writes, bursts 8", a, y, bytes, rpw);
        run<16, 12, 8, true>("U=16 read + 1/12 writes, bursts 8", a, y, bytes, rpw);
    }
    return 0;
}
