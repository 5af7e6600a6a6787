// pattern_probe.hip -- speed-of-light calibration for the read-order scan (not part of the library).
//
// Reproduces bp_scan32's memory pattern for one 50M-pair batch with no compute:
//   streaming: 16-B pair record + rw x 8-B read-row words (column-major) read, 8-B result written
//   gathers  : G random 16-B loads per lane from a genome-sized table (the A / B windows),
//              line-aligned or at random 16-B offsets
// Variants: streaming only, gathers only, both.  The kernel cannot beat "both".
//
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/pattern_probe scripts/pattern_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error %s\n", #x); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

template <int G, bool STREAM, bool PAIRED = false>
__global__ __launch_bounds__(256) void pattern(const ulonglong2 *__restrict__ pairs, const uint64_t *__restrict__ words,
                                               int rw, const ulonglong2 *__restrict__ table, uint64_t n_units,
                                               uint64_t n, uint64_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t acc = 0, seed = 0;
    if (STREAM) {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        const u64x2 p = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(pairs) + i);
        acc = p.x ^ p.y;
        seed = p.x;
        for (int j = 0; j < rw; ++j) acc += __builtin_nontemporal_load(words + (uint64_t)j * n + i);
    }
#pragma unroll
    for (int k = 0; k < G; ++k) {
        // PAIRED: lanes 2m, 2m+1 read the two adjacent 16-B units of ONE random 32-B span
        // (one line), i.e. per lane one 16-B load but half the distinct lines
        const uint64_t key = PAIRED ? (i >> 1) : i;
        uint64_t u = mix(key * 0x9E37ull + k + (seed & 1)) % n_units;
        if (PAIRED) u = (u & ~1ull) + (i & 1);
        const ulonglong2 v = table[u];
        acc ^= v.x + v.y;
    }
    if (STREAM) __builtin_nontemporal_store(acc, out + i);
    else if (acc == 0x123456789ull) out[i] = acc;     // keeps the gathers live without a store stream
}

template <int G, bool S, bool PR = false>
float run(const ulonglong2 *pairs, const uint64_t *words, int rw, const ulonglong2 *t, uint64_t nu, uint64_t n,
          uint64_t *out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const unsigned grid = (unsigned)((n + 255) / 256);
    pattern<G, S, PR><<<grid, 256>>>(pairs, words, rw, t, nu, n, out);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < 10; ++r) pattern<G, S, PR><<<grid, 256>>>(pairs, words, rw, t, nu, n, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}

int main() {
    const uint64_t n = 50000000ull;
    const int rw = 3;
    const uint64_t table_bytes = 800ull << 20;   // ~hg19 code planes (0.78 GB)
    const uint64_t nu = table_bytes / 16;
    ulonglong2 *pairs, *t;
    uint64_t *words, *out;
    CK(hipMalloc(&pairs, n * 16));
    CK(hipMalloc(&words, n * 8 * rw));
    CK(hipMalloc(&out, n * 8));
    CK(hipMalloc(&t, table_bytes));
    CK(hipMemset(pairs, 1, n * 16));
    CK(hipMemset(words, 2, n * 8 * rw));
    CK(hipMemset(t, 3, table_bytes));
    const float s0 = run<0, true>(pairs, words, rw, t, nu, n, out);
    const float g1 = run<1, false>(pairs, words, rw, t, nu, n, out);
    const float g2 = run<2, false>(pairs, words, rw, t, nu, n, out);
    const float b1 = run<1, true>(pairs, words, rw, t, nu, n, out);
    const float b2 = run<2, true>(pairs, words, rw, t, nu, n, out);
    const float b3 = run<3, true>(pairs, words, rw, t, nu, n, out);
    const float p4 = run<4, true, true>(pairs, words, rw, t, nu, n, out);
    const float b4 = run<4, true>(pairs, words, rw, t, nu, n, out);
    printf("{\"pairs\": %llu, \"stream_only_ms\": %.4f, \"gather1_only_ms\": %.4f, \"gather2_only_ms\": %.4f, "
           "\"stream_gather1_ms\": %.4f, \"stream_gather2_ms\": %.4f, \"stream_gather3_ms\": %.4f, "
           "\"gathers_per_s_2only\": %.4g, \"stream_gather4_ms\": %.4f, \"stream_gather4_paired_ms\": %.4f}\n",
           (unsigned long long)n, s0, g1, g2, b1, b2, b3, 2.0 * n / (g2 * 1e-3), b4, p4);
    return 0;
}
