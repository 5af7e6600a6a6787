// policy_probe.hip -- calibration micro-benchmark (not part of the library).
//
// Question: can a random 32-B window gather cost less than one 128-B line fill?
// The read-order scan is bound by ~2 random window lines per pair
// (profiles/r01/pattern_probe.json).  This probe gathers 16 B per lane (one
// load) or 32 B per lane pair (lanes 2m / 2m+1 load the two halves of one
// 32-B window in one instruction, as the kernel does) from an 8 GiB table,
// under every combination of
//   allocation : hipMalloc (coarse grained) | hipDeviceMallocFinegrained | hipDeviceMallocUncached
//   cache bits : none | nt | sc0 | sc1 | sc0+sc1 | sc0+sc1+nt   (buffer_load aux field, gfx950 CPol)
// and reports gathers/s.  A rate well above ~50 G gathers/s (the coarse-grained
// 128-B-line rate) would mean smaller memory-side requests.
//
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/policy_probe scripts/policy_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// PAIR: lanes 2m, 2m+1 share one random 32-B window (each loads 16 B of it).
template <int AUX, bool PAIR>
__global__ void probe(const uint8_t *__restrict__ t, uint32_t n_lines, int iters, uint32_t *out) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)t, 0, 0x7fffffff, 0x00020000);
    uint32_t acc = 0;
    const uint64_t lane_key = PAIR ? (tid >> 1) : tid;
    for (int it = 0; it < iters; ++it) {
        // one 2 GiB window of the table per iteration quarter keeps offsets in 31 bits
        const uint64_t r = mix(lane_key * 1315423911ull + it);
        const uint32_t line = (uint32_t)(r % n_lines);
        const uint32_t sub = (uint32_t)(r >> 40) & 3;          // 32-B window at a random 32-B slot
        uint32_t off = line * 128u + sub * 32u + (PAIR ? (tid & 1) * 16u : 0u);
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX);
        acc ^= v.x + v.y + v.z + v.w;
    }
    out[tid] = acc;
}

template <int AUX, bool PAIR>
double run(const uint8_t *t, uint32_t n_lines, uint32_t *out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    probe<AUX, PAIR><<<blocks, 256>>>(t, n_lines, iters, out);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) probe<AUX, PAIR><<<blocks, 256>>>(t, n_lines, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms / 5;
}

int main() {
    const uint64_t bytes = 2ull << 30;                 // 2 GiB: 8x the Infinity Cache, 31-bit offsets
    const uint32_t n_lines = (uint32_t)(bytes / 128);
    const int blocks = 256 * 32, iters = 64;
    uint32_t *out;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    const char *alloc_name[3] = {"coarse", "finegrained", "uncached"};
    const unsigned flags[3] = {0, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
    printf("[");
    bool first = true;
    for (int a = 0; a < 3; ++a) {
        uint8_t *t = nullptr;
        hipError_t e = a == 0 ? hipMalloc((void **)&t, bytes) : hipExtMallocWithFlags((void **)&t, bytes, flags[a]);
        if (e != hipSuccess) {
            fprintf(stderr, "alloc %s failed: %s\n", alloc_name[a], hipGetErrorString(e));
            continue;
        }
        hipMemset(t, 1, bytes);
        hipDeviceSynchronize();
        const double lanes = (double)blocks * 256 * iters;
        struct R { const char *pol; bool pair; double ms; } rs[12] = {
            {"none", false, run<0, false>(t, n_lines, out, blocks, iters)},
            {"nt", false, run<2, false>(t, n_lines, out, blocks, iters)},
            {"sc0", false, run<1, false>(t, n_lines, out, blocks, iters)},
            {"sc1", false, run<16, false>(t, n_lines, out, blocks, iters)},
            {"sc0sc1", false, run<17, false>(t, n_lines, out, blocks, iters)},
            {"sc0sc1nt", false, run<19, false>(t, n_lines, out, blocks, iters)},
            {"none", true, run<0, true>(t, n_lines, out, blocks, iters)},
            {"nt", true, run<2, true>(t, n_lines, out, blocks, iters)},
            {"sc0", true, run<1, true>(t, n_lines, out, blocks, iters)},
            {"sc1", true, run<16, true>(t, n_lines, out, blocks, iters)},
            {"sc0sc1", true, run<17, true>(t, n_lines, out, blocks, iters)},
            {"sc0sc1nt", true, run<19, true>(t, n_lines, out, blocks, iters)},
        };
        for (auto &r : rs) {
            const double gathers = r.pair ? lanes / 2 : lanes;
            printf("%s{\"alloc\": \"%s\", \"policy\": \"%s\", \"gather_bytes\": %d, \"ms\": %.4f, "
                   "\"Ggathers_per_s\": %.2f, \"TBps_if_128B_lines\": %.3f}",
                   first ? "" : ",\n ", alloc_name[a], r.pol, r.pair ? 32 : 16, r.ms, gathers / (r.ms * 1e-3) / 1e9,
                   gathers / (r.ms * 1e-3) * 128 / 1e12);
            first = false;
        }
        hipFree(t);
    }
    printf("]\n");
    return 0;
}
