// size_probe.hip -- calibration micro-benchmark (not part of the library).
//
// Random-line gather rate versus table size: lanes 2m / 2m+1 load the two 16-B halves of one
// random 32-B window (one L2 request per window, as the scan does) from tables of 8 MiB .. 2 GiB.
// Below 32 MiB (8 x 4 MiB L2) windows are mostly L2 hits, below 256 MiB Infinity-Cache hits,
// above it HBM line fills.  Question answered: would a batch bucketed by genome region
// (each bucket's slice of the 1.6 GB word-pair table <= ~200 MB) gather faster than the
// read-order batch's ~54 G lines/s from HBM?
//
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/size_probe scripts/size_probe.hip
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

__global__ void probe(const uint8_t *__restrict__ t, uint32_t n_lines, int iters, uint32_t *out) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)t, 0, 0x7fffffff, 0x00020000);
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        const uint64_t r = mix((uint64_t)(tid >> 1) * 1315423911ull + it);
        const uint32_t line = (uint32_t)(r % n_lines);
        const uint32_t sub = (uint32_t)(r >> 40) & 3;
        const uint32_t off = line * 128u + sub * 32u + (tid & 1) * 16u;
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
        acc ^= v.x + v.y + v.z + v.w;
    }
    out[tid] = acc;
}

int main() {
    const uint64_t max_bytes = 2ull << 30;
    const int blocks = 256 * 32, iters = 64;
    uint8_t *t;
    uint32_t *out;
    if (hipMalloc((void **)&t, max_bytes) != hipSuccess || hipMalloc((void **)&out, (size_t)blocks * 256 * 4) != hipSuccess)
        return 1;
    (void)hipMemset(t, 1, max_bytes);
    const uint64_t sizes_mb[] = {8, 32, 64, 128, 192, 256, 384, 512, 1024, 2047};
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    printf("[");
    for (int k = 0; k < 10; ++k) {
        const uint32_t n_lines = (uint32_t)((sizes_mb[k] << 20) / 128);
        probe<<<blocks, 256>>>(t, n_lines, iters, out);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a);
        for (int r = 0; r < 5; ++r) probe<<<blocks, 256>>>(t, n_lines, iters, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        const double windows = (double)blocks * 256 * iters / 2;
        printf("%s{\"table_MiB\": %llu, \"ms\": %.4f, \"Gwindows_per_s\": %.2f}", k ? ",\n " : "",
               (unsigned long long)sizes_mb[k], ms, windows / (ms * 1e-3) / 1e9);
    }
    printf("]\n");
    return 0;
}
