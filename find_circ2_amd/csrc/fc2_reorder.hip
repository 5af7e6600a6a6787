// fc2_reorder.hip -- device locality reorder of a pair batch (stable counting sort
// by genome bucket of the A window).
//
// Why: a batch in read order (the order bwa mem emits fragments, find_circ.py
// iterates them at :1376-1395) sends every lane of a wave to an unrelated
// genome locus; each window then costs a whole 128-B line fill from HBM for the
// ~20 bytes it uses (profiles/traffic_r01.json: 346 B/pair moved vs 81 B/pair
// algorithmic).  Sorting the batch by locus first makes the waves that run
// together on one XCD read the same few MB of the genome planes, which then
// stay in that XCD's L2 (84 B/pair moved for a locus-ordered batch).
//
// The sort is a single-pass stable counting sort with one digit of <= 1024 buckets
// of 2^shift genome bases (bucket = (chrom_start + a_pos) >> shift):
//   K1 reorder_hist    : per chunk of kChunk pairs, bucket histogram (LDS atomics)
//   K2 reorder_gsum    : per group of kGroup chunks, per-bucket sums
//   K3 reorder_base    : per bucket, exclusive prefix over groups + bucket bases
//   K4 reorder_offsets : per chunk, per bucket, first destination slot
//   K5 reorder_scatter : move pair records + read rows to their slot (stable:
//                        ranks inside a chunk follow batch order, via wave
//                        ballots and an LDS per-wave count table)
// Chunks are dealt to XCDs in contiguous ranges (as bp_scan32 does for ordered
// batches) so that the partial 128-B lines of one bucket's destination run are
// completed inside one L2 before they are written back.
// Results of a scan over the reordered batch are in reordered order; slot[i]
// is the input position of reordered pair i.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fc2_common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxBuckets = 1024;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ uint32_t bucket_of(const fc2_pair &pr, const fc2_genome_view &g, uint32_t shift,
                                              uint32_t nb) {
    if (g.dummy || pr.chrom >= g.n_chrom) return 0;
    const int64_t pos = pr.a_pos < 0 ? 0 : (int64_t)pr.a_pos;
    const uint64_t gb = g.chrom_start[pr.chrom] + (uint64_t)pos;
    const uint64_t b = gb >> shift;
    return b >= nb ? nb - 1 : (uint32_t)b;
}

__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b, uint32_t nwg) {   // see bp_scan32 xcd_block
    const uint32_t x = b & 7u, j = b >> 3, q = nwg >> 3, r = nwg & 7u;
    return x * q + (x < r ? x : r) + j;
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ fc2_pair load_pair(const fc2_pair *p) {
    const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
    fc2_pair r;
    __builtin_memcpy(&r, &v, sizeof r);
    return r;
}

__global__ __launch_bounds__(kThreads) void reorder_hist(fc2_genome_view g, const fc2_pair *__restrict__ pairs,
                                                         uint64_t n, uint32_t shift, uint32_t nb, int rounds,
                                                         uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[kMaxBuckets];
    for (uint32_t k = threadIdx.x; k < nb; k += kThreads) h[k] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kThreads * rounds;
#pragma unroll 4
    for (int r = 0; r < rounds; ++r) {
        const uint64_t i = base + (uint64_t)r * kThreads + threadIdx.x;
        if (i < n) atomicAdd(&h[bucket_of(load_pair(pairs + i), g, shift, nb)], 1u);
    }
    __syncthreads();
    uint32_t *row = hist + (uint64_t)blockIdx.x * nb;
    for (uint32_t k = threadIdx.x; k < nb; k += kThreads) row[k] = h[k];
}

// gsum[grp][b] = sum over the group's chunks of hist[c][b]
__global__ __launch_bounds__(kMaxBuckets) void reorder_gsum(const uint32_t *__restrict__ hist, uint32_t nchunks,
                                                            uint32_t nb, uint32_t group, uint32_t *__restrict__ gsum) {
    const uint32_t b = threadIdx.x;
    if (b >= nb) return;
    const uint32_t c0 = blockIdx.x * group, c1 = min(nchunks, c0 + group);
    uint32_t s = 0;
#pragma unroll 8
    for (uint32_t c = c0; c < c1; ++c) s += hist[(uint64_t)c * nb + b];
    gsum[(uint64_t)blockIdx.x * nb + b] = s;
}

// One block: gsum[grp][b] <- bucket base + exclusive prefix over groups.
__global__ __launch_bounds__(kMaxBuckets) void reorder_base(uint32_t *__restrict__ gsum, uint32_t ngroups,
                                                            uint32_t nb) {
    __shared__ uint32_t tot[kMaxBuckets];
    const uint32_t b = threadIdx.x;
    uint32_t run = 0;
    if (b < nb) {
        for (uint32_t g0 = 0; g0 < ngroups; g0 += 16) {
            uint32_t v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = (g0 + k < ngroups) ? gsum[(uint64_t)(g0 + k) * nb + b] : 0u;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (g0 + k < ngroups) { gsum[(uint64_t)(g0 + k) * nb + b] = run; run += v[k]; }
        }
    }
    tot[b] = b < nb ? run : 0u;
    __syncthreads();
    // inclusive Hillis-Steele scan over the bucket totals
    for (uint32_t d = 1; d < kMaxBuckets; d <<= 1) {
        const uint32_t add = b >= d ? tot[b - d] : 0u;
        __syncthreads();
        tot[b] += add;
        __syncthreads();
    }
    if (b >= nb) return;
    const uint32_t base = tot[b] - run;          // exclusive
    for (uint32_t gi = 0; gi < ngroups; ++gi) gsum[(uint64_t)gi * nb + b] += base;
}

// hist[c][b] <- first destination slot of chunk c's pairs in bucket b
__global__ __launch_bounds__(kMaxBuckets) void reorder_offsets(uint32_t *__restrict__ hist,
                                                               const uint32_t *__restrict__ gsum, uint32_t nchunks,
                                                               uint32_t nb, uint32_t group) {
    const uint32_t b = threadIdx.x;
    if (b >= nb) return;
    const uint32_t c0 = blockIdx.x * group, c1 = min(nchunks, c0 + group);
    uint32_t run = gsum[(uint64_t)blockIdx.x * nb + b];
    for (uint32_t c = c0; c < c1; c += 16) {
        uint32_t v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = (c + k < c1) ? hist[(uint64_t)(c + k) * nb + b] : 0u;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (c + k < c1) { hist[(uint64_t)(c + k) * nb + b] = run; run += v[k]; }
    }
}

template <int RW>
__global__ __launch_bounds__(kThreads) void reorder_scatter(fc2_genome_view g, fc2_batch_view in, uint32_t shift,
                                                            uint32_t nb, uint32_t nbits, const uint32_t *__restrict__ offs,
                                                            fc2_pair *__restrict__ pairs_out,
                                                            uint64_t *__restrict__ words_out,
                                                            uint64_t *__restrict__ nwords_out,
                                                            uint32_t *__restrict__ slot_out, uint32_t rw_rt,
                                                            int rounds, int nt_store) {
    __shared__ uint32_t run[kMaxBuckets];
    __shared__ uint32_t wcnt[kWaves][kMaxBuckets];
    const uint32_t chunk = xcd_chunk(blockIdx.x, gridDim.x);
    const uint32_t *row = offs + (uint64_t)chunk * nb;
    for (uint32_t k = threadIdx.x; k < nb; k += kThreads) {
        run[k] = row[k];
#pragma unroll
        for (int w = 0; w < kWaves; ++w) wcnt[w][k] = 0;
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t base = (uint64_t)chunk * kThreads * rounds;
    const uint32_t rw = RW > 0 ? (uint32_t)RW : rw_rt;
    for (int r = 0; r < rounds; ++r) {
        const uint64_t i = base + (uint64_t)r * kThreads + threadIdx.x;
        const bool valid = i < in.n;
        fc2_pair pr{};
        if (valid) pr = load_pair(in.pairs + i);
        uint64_t w[RW > 0 ? RW : 1];
        if constexpr (RW > 0) {
#pragma unroll
            for (int j = 0; j < RW; ++j)
                w[j] = valid ? __builtin_nontemporal_load(in.read_words + (uint64_t)j * in.stride + i) : 0ull;
        }
        const uint32_t bk = valid ? bucket_of(pr, g, shift, nb) : 0u;
        uint64_t peers = __ballot(valid);
        for (uint32_t bit = 0; bit < nbits; ++bit) {
            const bool on = (bk >> bit) & 1u;
            const uint64_t bal = __ballot(on);
            peers &= on ? bal : ~bal;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        const uint32_t cnt = (uint32_t)__popcll(peers);
        const bool leader = valid && rank == 0;
        if (leader) wcnt[wave][bk] = cnt;
        __syncthreads();
        uint32_t dst = 0;
        if (valid) {
            dst = run[bk] + rank;
            for (int w2 = 0; w2 < wave; ++w2) dst += wcnt[w2][bk];
        }
        __syncthreads();
        if (leader) { atomicAdd(&run[bk], cnt); wcnt[wave][bk] = 0; }
        if (valid) {
            u64x2 pv;
            __builtin_memcpy(&pv, &pr, sizeof pv);
            if (nt_store) __builtin_nontemporal_store(pv, reinterpret_cast<u64x2 *>(pairs_out + dst));
            else *reinterpret_cast<u64x2 *>(pairs_out + dst) = pv;
            if constexpr (RW > 0) {
#pragma unroll
                for (int j = 0; j < RW; ++j) words_out[(uint64_t)j * in.stride + dst] = w[j];
            } else {
                for (uint32_t j = 0; j < rw; ++j)
                    words_out[(uint64_t)j * in.stride + dst] = in.read_words[(uint64_t)j * in.stride + i];
            }
            slot_out[dst] = (uint32_t)i;
            if ((pr.flags & FC2_PAIR_READ_N) && nwords_out)
                for (uint32_t j = 0; j < in.nw; ++j)
                    nwords_out[(uint64_t)j * in.stride + dst] = in.read_nwords[(uint64_t)j * in.stride + i];
        }
    }
}

// chunks per group of K2-K4: >= 64, and at most 128 groups (K3 walks them serially)
uint32_t group_size(uint32_t nchunks) {
    const uint32_t g = (nchunks + 127) / 128;
    return g < 64 ? 64 : g;
}

unsigned ceil_log2(uint64_t x) {
    unsigned s = 0;
    while ((1ull << s) < x) ++s;
    return s;
}

}  // namespace

namespace fc2 {
int g_reorder_rounds = 4;      // pairs per thread per chunk (FC2_TUNE_REORDER_ROUNDS; r01 sweep: 32 -> 4.4 ms,
                               // 8/4 -> 3.3 ms, 2 -> 2.9 ms per 50M pairs)
int g_reorder_nt = 0;          // non-temporal scatter stores (FC2_TUNE_REORDER_NT)
int g_reorder_shift = 0;       // bucket = 2^shift bases; 0: ~1024 buckets over the genome (FC2_TUNE_REORDER_SHIFT)
}  // namespace fc2

extern "C" int fc2_reorder_plan(const fc2_genome_view *g, uint64_t n, fc2_reorder_info *info) {
    if (!g || !info) return fc2::fail(FC2_E_PARAM, "fc2_reorder_plan: null argument");
    if (n > 0xFFFFFFFFull) return fc2::fail(FC2_E_RANGE, "fc2_reorder_plan: batch larger than 2^32 pairs");
    const uint64_t bases = g->dummy ? 1 : (g->n_units ? g->n_units * 64 : 1);
    unsigned shift = ceil_log2(bases);
    shift = shift > 10 ? shift - 10 : 0;
    if (shift < 16) shift = 16;                    // >= 64 kbp per bucket
    if (fc2::g_reorder_shift) {                    // FC2_TUNE_REORDER_SHIFT: coarser buckets (fewer fronts)
        shift = (unsigned)fc2::g_reorder_shift;
        while (((bases - 1) >> shift) + 1 > (uint64_t)kMaxBuckets) ++shift;
    }
    const uint64_t nb = ((bases - 1) >> shift) + 1;
    info->n = n;
    info->shift = shift;
    info->n_buckets = (uint32_t)nb;
    const uint64_t chunk = (uint64_t)kThreads * fc2::g_reorder_rounds;
    info->chunk = (uint32_t)chunk;
    info->n_chunks = (uint32_t)((n + chunk - 1) / chunk);
    info->n_groups = (info->n_chunks + group_size(info->n_chunks) - 1) / group_size(info->n_chunks);
    info->bucket_bits = ceil_log2(nb);
    info->workspace_bytes = ((uint64_t)info->n_chunks + info->n_groups) * nb * sizeof(uint32_t) + 256;
    return FC2_OK;
}

extern "C" int fc2_reorder_launch(const fc2_reorder_info *info, const fc2_genome_view *g, const fc2_batch_view *in,
                                  fc2_pair *pairs_out, uint64_t *read_words_out, uint64_t *read_nwords_out,
                                  uint32_t *slot_out, void *workspace, void *stream) {
    if (!info || !g || !in) return fc2::fail(FC2_E_PARAM, "fc2_reorder_launch: null argument");
    if (info->n != in->n) return fc2::fail(FC2_E_PARAM, "fc2_reorder_launch: plan was made for another batch size");
    if (in->n == 0) return FC2_OK;
    if (!in->pairs || !in->read_words || in->stride < in->n || !pairs_out || !read_words_out || !slot_out ||
        !workspace)
        return fc2::fail(FC2_E_PARAM, "fc2_reorder_launch: bad buffers");
    if (in->nw && in->read_nwords && !read_nwords_out)
        return fc2::fail(FC2_E_PARAM, "fc2_reorder_launch: read_nwords_out needed");
    if (!g->dummy && !g->chrom_start) return fc2::fail(FC2_E_PARAM, "fc2_reorder_launch: bad genome view");
    fc2_reorder_info chk;
    int rc = fc2_reorder_plan(g, in->n, &chk);
    if (rc) return rc;
    if (chk.n_buckets != info->n_buckets || chk.shift != info->shift || chk.n_chunks != info->n_chunks ||
        chk.chunk != info->chunk)
        return fc2::fail(FC2_E_PARAM, "fc2_reorder_launch: plan does not match the genome");
    hipStream_t s = (hipStream_t)stream;
    const uint32_t nb = info->n_buckets, nc = info->n_chunks, ng = info->n_groups;
    uint32_t *hist = static_cast<uint32_t *>(workspace);
    uint32_t *gsum = hist + (uint64_t)nc * nb;
    const int rounds = (int)(info->chunk / kThreads);
    hipLaunchKernelGGL(reorder_hist, dim3(nc), dim3(kThreads), 0, s, *g, in->pairs, in->n, info->shift, nb, rounds,
                       hist);
    const uint32_t grp = group_size(nc);
    hipLaunchKernelGGL(reorder_gsum, dim3(ng), dim3(kMaxBuckets), 0, s, hist, nc, nb, grp, gsum);
    hipLaunchKernelGGL(reorder_base, dim3(1), dim3(kMaxBuckets), 0, s, gsum, ng, nb);
    hipLaunchKernelGGL(reorder_offsets, dim3(ng), dim3(kMaxBuckets), 0, s, hist, gsum, nc, nb, grp);
    uint64_t *nwo = in->read_nwords ? read_nwords_out : nullptr;
#define FC2_RS(RWV)                                                                                              \
    hipLaunchKernelGGL((reorder_scatter<RWV>), dim3(nc), dim3(kThreads), 0, s, *g, *in, info->shift, nb,        \
                       info->bucket_bits, hist, pairs_out, read_words_out, nwo, slot_out, in->rw, rounds,   \
                       fc2::g_reorder_nt)
    switch (in->rw) {
        case 2: FC2_RS(2); break;
        case 3: FC2_RS(3); break;
        case 4: FC2_RS(4); break;
        default: FC2_RS(0); break;
    }
#undef FC2_RS
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fc2::fail(FC2_E_HIP, std::string("reorder launch: ") + hipGetErrorString(e));
    return FC2_OK;
}
