// gather_probe.hip -- calibration micro-benchmark (not part of the library).
//
// Random gathers of G contiguous bytes (G = 16, 32, 64, 128) from a table far
// larger than the 256 MB Infinity Cache, one gather per lane per iteration,
// XOR-accumulated so nothing is dead.  Reported: gathers/s and bytes/s under
// the "each miss fills 128 B" and "fills only the touched 64-B sectors"
// readings; whichever exceeds the HBM peak is impossible.
//
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/gather_probe scripts/gather_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

template <int G>
__global__ void probe(const ulonglong2 *__restrict__ t, uint64_t n_units, int iters, uint64_t *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t acc = 0;
    constexpr int U = G / 16;
    for (int it = 0; it < iters; ++it) {
        uint64_t u = mix(tid * 1315423911ull + it) % (n_units / 8) * 8;   // 128-B aligned line
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const ulonglong2 v = t[u + k];
            acc ^= v.x + v.y;
        }
    }
    out[tid] = acc;
}

template <int G>
double run(const ulonglong2 *t, uint64_t n_units, uint64_t *out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    probe<G><<<blocks, 256>>>(t, n_units, iters, out);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) probe<G><<<blocks, 256>>>(t, n_units, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const uint64_t bytes = 8ull << 30;
    const uint64_t n_units = bytes / 16;
    ulonglong2 *t;
    uint64_t *out;
    const int blocks = 256 * 32, iters = 64;
    if (hipMalloc(&t, bytes) != hipSuccess || hipMalloc(&out, (size_t)blocks * 256 * 8) != hipSuccess) return 1;
    hipMemset(t, 1, bytes);
    const double gathers = (double)blocks * 256 * iters;
    double ms[4] = {run<16>(t, n_units, out, blocks, iters), run<32>(t, n_units, out, blocks, iters),
                    run<64>(t, n_units, out, blocks, iters), run<128>(t, n_units, out, blocks, iters)};
    const int G[4] = {16, 32, 64, 128};
    printf("[");
    for (int k = 0; k < 4; ++k) {
        const double gps = gathers / (ms[k] * 1e-3);
        const double sectors = G[k] <= 64 ? 1 : 2;
        printf("%s{\"gather_bytes\": %d, \"ms\": %.4f, \"Ggathers_per_s\": %.2f, \"TBps_if_128B_lines\": %.3f, "
               "\"TBps_if_64B_sectors\": %.3f}", k ? ", " : "", G[k], ms[k], gps / 1e9, gps * 128 / 1e12,
               gps * 64 * sectors / 1e12);
    }
    printf("]\n");
    return 0;
}
