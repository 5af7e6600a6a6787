// sort_probe.hip -- calibration micro-benchmark for VERDICT r02 item 2 (not part of the library).
//
// Question: can a read-order batch be put into genome order on the device cheaply enough that the
// scan's windows come from L2 (one random line per pair for its row instead of two for its
// windows)?  The design under test ("keysort"): an 8-B (bucket, pair index) sort by a block-local
// LDS counting scatter, then a scan in bucket order that gathers each pair's 64-B AoS row through
// the permutation, reads both windows from an L2-local genome slice and scatters its 8-B result
// back to input order.  This probe times every memory pattern of that design separately and the
// whole pattern end to end, with no search arithmetic (a lower bound on any kernel doing it), next
// to the read-order pattern the shipped scan has (streamed rows, two random windows):
//
//   stream_rows      rows[i] (64 B) read, out[i] written: the streamed part of a scan
//   scatter8         out[perm(i)] = v: random 8-B writes (results back to input order)
//   gather8          out[i] = src[perm(i)]: random 8-B reads (the same by gather)
//   gather_rows      rows[perm(i)]: random 64-B AoS rows, one request per row
//   gather_scatter   rows[perm(i)] read, out[perm(i)] written: the sorted scan minus windows
//   keysort          K1 bucket histogram (LDS) + K2 block-local LDS rank + scatter of 4-B pair indices
//   sorted_scan      gather_scatter + both windows of each pair from the bucket's genome slice (bucket
//                    order, blocks mapped so one XCD walks a contiguous range of buckets)
//   readorder_scan   rows streamed + both windows at random (what the shipped kernel moves)
//
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/sort_probe scripts/sort_probe.hip
// run:   scripts/sort_probe [n_pairs]     (prints one JSON line per pattern)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__host__ __device__ inline uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// a bijection of [0, n): i -> (i * A + B) mod n with A odd and coprime to n (n is a multiple of 2^k
// times an odd part; A is a large prime not dividing it)
__device__ __forceinline__ uint32_t perm_of(uint64_t i, uint64_t n) {
    return (uint32_t)((i * 2654435761ull + 40503ull) % n);
}

// genome model: G bases, 2 bits each in a word-pair table (8 B per 32 bases), one copy
constexpr uint64_t kGenome = 3137161264ull;
__device__ __forceinline__ uint64_t locus_of(uint64_t i) { return mix(i ^ 0x5EEDull) % (kGenome - 30000); }
__device__ __forceinline__ uint32_t span_of(uint64_t i) { return 150u + (uint32_t)(mix(i ^ 0xABCull) % 19851u); }

__device__ __forceinline__ uint64_t xcd_block(uint32_t b, uint32_t nwg) {
    const uint32_t x = b & 7u, j = b >> 3, q = nwg >> 3, r = nwg & 7u;
    return (uint64_t)x * q + (x < r ? x : r) + j;
}

__global__ __launch_bounds__(256) void stream_rows(const u32x4 *__restrict__ rows, uint64_t *__restrict__ out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    u32x4 a = __builtin_nontemporal_load(rows + 4 * i), b = __builtin_nontemporal_load(rows + 4 * i + 1),
          c = __builtin_nontemporal_load(rows + 4 * i + 2);
    __builtin_nontemporal_store((uint64_t)(a.x ^ b.y ^ c.z) | ((uint64_t)(a.w + b.z + c.x) << 32), out + i);
}

__global__ __launch_bounds__(256) void scatter8(uint64_t *__restrict__ out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    out[perm_of(i, n)] = i * 0x9E37ull;
}

__global__ __launch_bounds__(256) void gather8(const uint64_t *__restrict__ src, uint64_t *__restrict__ out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    __builtin_nontemporal_store(src[perm_of(i, n)], out + i);
}

// one row = 64 B; lanes 4m..4m+3 load the four 16-B pieces of pair m's row in ONE instruction (one
// request per row), then the owner lane gets its three pieces (48 B used: record + 3 read words)
template <bool SCATTER>
__global__ __launch_bounds__(256) void gather_rows(const u32x4 *__restrict__ rows, uint64_t *__restrict__ out, uint64_t n) {
    const uint64_t base = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u);
    const int lane = threadIdx.x & 63;
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint64_t m = base + 16 * c + (lane >> 2);
        if (m < n) {
            const u32x4 v = rows[4 * (uint64_t)perm_of(m, n) + (lane & 3)];
            acc ^= v.x + v.y + v.z + v.w;
        }
    }
    const uint64_t i = base + lane;
    if (i >= n) return;
    if (SCATTER) out[perm_of(i, n)] = acc;
    else __builtin_nontemporal_store((uint64_t)acc, out + i);
}

// ---- keysort: buckets of the A-window locus ---------------------------------------------------
constexpr int kSortT = 4096;          // pairs per block (16 per thread)
__global__ __launch_bounds__(256) void bucket_keys(uint32_t *__restrict__ key, uint64_t n, int shift) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) key[i] = (uint32_t)(locus_of(i) >> shift);
}

__global__ __launch_bounds__(256) void k1_hist(const uint32_t *__restrict__ key, uint64_t n, uint32_t nb,
                                               uint32_t *__restrict__ count) {
    extern __shared__ uint32_t h[];
    for (uint32_t b = threadIdx.x; b < nb; b += 256) h[b] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * kSortT;
    for (int k = 0; k < kSortT / 256; ++k) {
        const uint64_t i = b0 + k * 256 + threadIdx.x;
        if (i < n) atomicAdd(&h[key[i]], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += 256)
        if (h[b]) atomicAdd(&count[b], h[b]);
}

__global__ void k_prefix(const uint32_t *__restrict__ count, uint32_t nb, uint32_t *__restrict__ cursor) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        uint32_t s = 0;
        for (uint32_t b = 0; b < nb; ++b) { cursor[b] = s; s += count[b]; }
    }
}

// LDS counting sort of the block's keys, then each bucket's run written contiguously at a slot
// reserved with one atomic per (block, bucket)
__global__ __launch_bounds__(256) void k2_scatter(const uint32_t *__restrict__ key, uint64_t n, uint32_t nb,
                                                  uint32_t *__restrict__ cursor, uint32_t *__restrict__ perm) {
    extern __shared__ uint32_t sm[];
    uint32_t *h = sm, *start = sm + nb, *idx = sm + 2 * nb;   // idx: kSortT sorted pair indices
    for (uint32_t b = threadIdx.x; b < nb; b += 256) h[b] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * kSortT;
    uint32_t myk[kSortT / 256], myr[kSortT / 256];
    for (int k = 0; k < kSortT / 256; ++k) {
        const uint64_t i = b0 + k * 256 + threadIdx.x;
        myk[k] = i < n ? key[i] : 0xFFFFFFFFu;
        myr[k] = i < n ? atomicAdd(&h[myk[k]], 1u) : 0u;
    }
    __syncthreads();
    // block-local exclusive prefix over buckets: each thread sums a chunk, a scan over the 256
    // chunk sums, then each thread writes its chunk's starts
    __shared__ uint32_t part[256];
    const uint32_t C = (nb + 255) / 256, lo = threadIdx.x * C, hi = min(nb, lo + C);
    uint32_t s = 0;
    for (uint32_t b = lo; b < hi; ++b) s += h[b];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {
        const uint32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    s = part[threadIdx.x] - s;                  // exclusive
    for (uint32_t b = lo; b < hi; ++b) { start[b] = s; s += h[b]; }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += 256) {
        const uint32_t c = h[b];
        h[b] = c ? atomicAdd(&cursor[b], c) : 0u;    // global base of this block's run of bucket b
    }
    __syncthreads();
    for (int k = 0; k < kSortT / 256; ++k)
        if (myk[k] != 0xFFFFFFFFu) idx[start[myk[k]] + myr[k]] = (uint32_t)(b0 + k * 256 + threadIdx.x);
    __syncthreads();
    // write the runs: position j of the block's sorted order goes to h[bucket] + (j - start[bucket])
    for (int k = 0; k < kSortT / 256; ++k) {
        const uint32_t j = k * 256 + threadIdx.x;
        if (b0 + j >= n) continue;
        const uint32_t pi = idx[j];
        const uint32_t b = key[pi];                  // L2 hit (read by this block just before)
        perm[h[b] + (j - start[b])] = pi;
    }
}

// ---- the two scan patterns (no search arithmetic) -----------------------------------------------
__device__ __forceinline__ u32x4 window_load(__amdgpu_buffer_rsrc_t rs, uint64_t g0) {
    // 32 B of word pairs from q0 = g0 >> 5: lanes 2m, 2m+1 would split it; here one lane loads 16 B
    return __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((g0 >> 5) * 8u), 0, 0);
}

__global__ __launch_bounds__(256) void sorted_scan(const u32x4 *__restrict__ rows, const uint32_t *__restrict__ perm,
                                                   const uint32_t *__restrict__ wt, uint32_t wt_bytes,
                                                   uint64_t *__restrict__ out, uint64_t n) {
    const uint64_t blk = xcd_block(blockIdx.x, gridDim.x);
    const uint64_t base = blk * 256 + (threadIdx.x & ~63u);
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)wt, 0, (int)wt_bytes, 0x00020000);
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint64_t m = base + 16 * c + (lane >> 2);
        if (m < n) {
            const u32x4 v = rows[4 * (uint64_t)perm[m] + (lane & 3)];
            acc ^= v.x + v.y + v.z + v.w;
        }
    }
    const uint64_t i = base + lane;
    if (i >= n) return;
    const uint32_t p = perm[i];
    const uint64_t a = locus_of(p), b = a + span_of(p);
    const u32x4 wa = window_load(rs, a), wb = window_load(rs, b);
    const u32x4 wa2 = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((a >> 5) * 8u) + 16u, 0, 0);
    const u32x4 wb2 = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((b >> 5) * 8u) + 16u, 0, 0);
    acc ^= wa.x + wb.y + wa2.z + wb2.w;
    out[p] = acc;
}

__global__ __launch_bounds__(256) void readorder_scan(const u32x4 *__restrict__ rows, const uint32_t *__restrict__ wt,
                                                      uint32_t wt_bytes, uint64_t *__restrict__ out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)wt, 0, (int)wt_bytes, 0x00020000);
    u32x4 r0 = __builtin_nontemporal_load(rows + 4 * i), r1 = __builtin_nontemporal_load(rows + 4 * i + 1),
          r2 = __builtin_nontemporal_load(rows + 4 * i + 2);
    const uint64_t a = locus_of(i), b = a + span_of(i);
    const u32x4 wa = window_load(rs, a), wb = window_load(rs, b);
    const u32x4 wa2 = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((a >> 5) * 8u) + 16u, 0, 0);
    const u32x4 wb2 = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((b >> 5) * 8u) + 16u, 0, 0);
    __builtin_nontemporal_store((uint64_t)(r0.x ^ r1.y ^ r2.z ^ wa.x ^ wb.y ^ wa2.z ^ wb2.w), out + i);
}

template <class F>
static float timed(F f, int reps = 5) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 50000000ull;
    const uint32_t grid = (uint32_t)((n + 255) / 256);
    const uint64_t wt_bytes = (kGenome / 32 + 64) * 8;     // one copy of the word-pair table (0.78 GB)
    u32x4 *rows;
    uint64_t *out, *src;
    uint32_t *wt, *key, *perm, *count, *cursor;
    CK(hipMalloc((void **)&rows, n * 64));
    CK(hipMalloc((void **)&out, n * 8));
    CK(hipMalloc((void **)&src, n * 8));
    CK(hipMalloc((void **)&wt, wt_bytes));
    CK(hipMalloc((void **)&key, n * 4));
    CK(hipMalloc((void **)&perm, n * 4));
    constexpr uint32_t kMaxBuckets = 1u << 16;      // count / cursor capacity; every nb below is checked
    CK(hipMalloc((void **)&count, kMaxBuckets * 4));
    CK(hipMalloc((void **)&cursor, kMaxBuckets * 4));
    CK(hipMemset(rows, 1, n * 64));
    CK(hipMemset(src, 2, n * 8));
    CK(hipMemset(wt, 3, wt_bytes));
    auto line = [&](const char *name, float ms, double bytes_per_pair, const char *extra) {
        printf("{\"pattern\": \"%s\", \"n\": %llu, \"ms\": %.4f, \"pairs_per_s\": %.4g, \"moved_GBs\": %.1f%s}\n", name,
               (unsigned long long)n, ms, n / (ms * 1e-3), bytes_per_pair * n / (ms * 1e-3) / 1e9, extra);
        fflush(stdout);
    };
    line("stream_rows", timed([&] { stream_rows<<<grid, 256>>>(rows, out, n); }), 56, "");
    line("scatter8", timed([&] { scatter8<<<grid, 256>>>(out, n); }), 8, "");
    line("gather8", timed([&] { gather8<<<grid, 256>>>(src, out, n); }), 16, "");
    line("gather_rows", timed([&] { gather_rows<false><<<grid, 256>>>(rows, out, n); }), 72, "");
    line("gather_scatter", timed([&] { gather_rows<true><<<grid, 256>>>(rows, out, n); }), 72, "");
    line("readorder_scan", timed([&] { readorder_scan<<<grid, 256>>>(rows, wt, (uint32_t)wt_bytes, out, n); }), 56 + 64 + 8,
         "");
    for (int shift : {22, 20, 18}) {               // 748 / 2992 / 11968 buckets of 4 / 1 / 0.25 Mbp
        const uint32_t nb = (uint32_t)((kGenome >> shift) + 1);
        if (nb > kMaxBuckets) continue;
        bucket_keys<<<grid, 256>>>(key, n, shift);
        const uint32_t sgrid = (uint32_t)((n + kSortT - 1) / kSortT);
        const size_t lds1 = nb * 4, lds2 = (2 * (size_t)nb + kSortT) * 4;
        if (lds2 + 1024 > 160 * 1024) continue;
        CK(hipFuncSetAttribute((const void *)k1_hist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1));
        CK(hipFuncSetAttribute((const void *)k2_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
        const float ms_sort = timed([&] {
                CK(hipMemsetAsync(count, 0, nb * 4));
            k1_hist<<<sgrid, 256, lds1>>>(key, n, nb, count);
            k_prefix<<<1, 64>>>(count, nb, cursor);
            k2_scatter<<<sgrid, 256, lds2>>>(key, n, nb, cursor, perm);
        });
        const float ms_scan = timed([&] { sorted_scan<<<grid, 256>>>(rows, perm, wt, (uint32_t)wt_bytes, out, n); });
        char ex[160];
        snprintf(ex, sizeof ex, ", \"buckets\": %u, \"sort_ms\": %.4f, \"scan_ms\": %.4f", nb, ms_sort, ms_scan);
        line("keysort+sorted_scan", ms_sort + ms_scan, 4 + 8 + 8 + 64 + 8, ex);
    }
    // validate the permutation of the last sort: every pair exactly once, buckets ascending
    std::vector<uint32_t> hp(n), hk(n);
    CK(hipMemcpy(hp.data(), perm, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hk.data(), key, n * 4, hipMemcpyDeviceToHost));
    std::vector<uint8_t> seen(n, 0);
    bool ok = true;
    for (uint64_t j = 0; j < n && ok; ++j) {
        if (hp[j] >= n || seen[hp[j]]++) ok = false;
        if (j && hk[hp[j]] < hk[hp[j - 1]]) ok = false;
    }
    printf("{\"pattern\": \"keysort_check\", \"permutation_valid_and_bucket_sorted\": %s}\n", ok ? "true" : "false");
    return ok ? 0 : 1;
}
