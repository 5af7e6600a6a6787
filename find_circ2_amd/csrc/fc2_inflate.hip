// fc2_inflate.hip -- BGZF blocks inflated on the GPU: the BAM input of the read loop
// (fc2_ingest.cpp bgzf_batch; the reference reads it through pysam/htslib, find_circ.py:461-469).
//
// A BGZF block (SAM/BAM spec 4.1) is a gzip member of at most 64 KiB holding at most 64 KiB of
// output, independent of every other block: one wavefront per block.  The DEFLATE stream (RFC 1951)
// is serial, so it is decoded wave-uniformly and kept in scalar registers: the payload is read 64
// words at a time, one word per lane (a refill is a v_readlane, the next 64 words already in flight),
// and every table entry read from LDS is made scalar (readfirstlane), so the decode's control flow is
// scalar branches.  The lanes work side by side where the work is parallel: building a Huffman
// code's tables (a ballot ranks the symbols of each length; each lane fills its own codes' entries),
// the bytes of a match (every source byte precedes the match -- p - dist + j mod dist -- so one
// iteration moves 64 bytes even for overlapping copies), stored blocks, and the stores to HBM.
// The output goes through a 16 KiB ring in LDS flushed to HBM 4 KiB at a time; a match reaching
// farther back (DEFLATE's window is 32 KiB) reads the stored output.  Fast tables of 9 and 7 bits
// (longer codes: the canonical test from there on) keep a workgroup at 20 KB of LDS: eight a CU,
// two waves a SIMD, one decoding while the other waits.  A table entry carries the symbol's
// meaning (literal / length or distance base and its extra-bit count / end of block), so a length
// or a distance is one lookup and one shift.  Every access is bounds-checked: a malformed block sets
// its status word, and the host, which checks each block's CRC-32 and ISIZE on the bytes it copies
// back, inflates any block the GPU refused on the CPU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/fc2_ingest.h"
#include "fc2_common.h"
#include "fc2_inflate.h"

namespace {

constexpr uint32_t kOutMax = 65536;            // BGZF ISIZE limit
constexpr uint32_t kRing = 16384;              // the LDS ring: half DEFLATE's window (farther: HBM)
constexpr uint32_t kRingMask = kRing - 1;
constexpr uint32_t kFlush = 4096;              // ring -> HBM granule
constexpr int kLitBits = 9;                    // fast-table bits: literal/length code
constexpr int kDistBits = 7;                   // distance code, and the code-length code

enum : uint32_t { INF_OK = 0, INF_BAD_TYPE = 1, INF_BAD_STORED = 2, INF_BAD_COUNTS = 3, INF_BAD_CODE = 4,
                  INF_BAD_DIST = 5, INF_OVERFLOW = 6, INF_OVERRUN = 7, INF_SHORT = 8, INF_TOO_BIG = 9,
                  INF_BAD_CLCODE = 10, INF_BAD_CLSYM = 11, INF_BAD_REPEAT = 12, INF_NO_EOB = 13,
                  INF_BAD_LITCODE = 14, INF_BAD_DISTCODE = 15, INF_BAD_CRC = 16 };

// a table entry: codeword length (0: not in the fast table), extra-bit count, kind, value
enum : uint32_t { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_BAD = 3 };
enum Table { T_LIT, T_DIST, T_CL };

__device__ __forceinline__ uint32_t entry(uint32_t len, uint32_t extra, uint32_t kind, uint32_t value) {
    return len | (extra << 4) | (kind << 8) | (value << 16);
}

struct Lds {                                   // 19968 B: eight workgroups a CU, two waves a SIMD
    uint8_t ring[kRing];
    uint32_t lfast[1 << kLitBits];
    uint32_t dfast[1 << kDistBits];            // (also the code-length code's table)
    uint32_t cnt[16];                          // codes per length, while a code is built
    uint16_t lsym[288], dsym[32];              // symbols in canonical order (codes past the fast tables)
    uint8_t lens[320];
};

__constant__ uint16_t kLBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59,
                                    67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                    1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDExt[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11,
                                  12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// what symbol s of a table means (len: its codeword length)
__device__ __forceinline__ uint32_t meaning(Table t, uint32_t s, uint32_t len) {
    if (t == T_CL) return entry(len, 0, K_LIT, s);
    if (t == T_DIST) return s < 30 ? entry(len, kDExt[s], K_LEN, kDBase[s]) : entry(len, 0, K_BAD, 0);
    if (s < 256) return entry(len, 0, K_LIT, s);
    if (s == 256) return entry(len, 0, K_EOB, 0);
    return s < 286 ? entry(len, kLExt[s - 257], K_LEN, kLBase[s - 257]) : entry(len, 0, K_BAD, 0);
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// the bit reader: wave-uniform, over a window of 64 payload words held one per lane (`win`: lane
// i holds word base + i) -- a refill is a v_readlane, not a dependent global load -- with the next
// window (`nxt`) loaded while this one is read.  `w` = the 32-bit words holding the block's payload,
// bit 0 of `pos` = bit 0 of w[0]; words past `last` read as 0 (no load past the payload)
struct Bits {
    const uint32_t *w;
    uint32_t pos, end;                         // bit positions
    uint64_t bb;                               // the bits at pos.. (nb of them)
    int nb;
    uint32_t wi;                               // next word to load into bb
    uint32_t base, last;                       // word index of lane 0's word in win; the last word
    uint32_t win, nxt;                         // this lane's word of the window, and of the next one
    int lane;
};

__device__ __forceinline__ uint32_t load_word(const Bits &b, uint32_t k) { return k <= b.last ? b.w[k] : 0u; }
__device__ __forceinline__ void window(Bits &b, uint32_t base) {
    b.base = base;
    b.win = load_word(b, base + (uint32_t)b.lane);
    b.nxt = load_word(b, base + 64u + (uint32_t)b.lane);
}
__device__ __forceinline__ uint32_t word(Bits &b, uint32_t k) {
    if (k - b.base >= 64u) {                   // (a k below base -- a seek back into bb -- reloads)
        if (k - b.base < 128u) {
            b.base += 64u;
            b.win = b.nxt;
            b.nxt = load_word(b, b.base + 64u + (uint32_t)b.lane);
        } else {
            window(b, k & ~63u);
        }
    }
    return (uint32_t)__builtin_amdgcn_readlane((int)b.win, (int)(k - b.base));
}
__device__ __forceinline__ void seek(Bits &b, uint32_t bitpos) {
    b.pos = bitpos;
    b.wi = bitpos >> 5;
    const uint32_t sh = bitpos & 31u;
    const uint32_t lo = word(b, b.wi);
    const uint32_t hi = word(b, b.wi + 1);
    b.bb = ((uint64_t)lo | ((uint64_t)hi << 32)) >> sh;
    b.nb = 64 - (int)sh;
    b.wi += 2;
}
__device__ __forceinline__ uint32_t peek(Bits &b) {  // afterwards >= 33 valid bits
    if (b.nb <= 32) {
        b.bb |= (uint64_t)word(b, b.wi++) << b.nb;
        b.nb += 32;
    }
    return (uint32_t)b.bb;
}
__device__ __forceinline__ void drop(Bits &b, int n) {
    b.bb >>= n;
    b.nb -= n;
    b.pos += (uint32_t)n;
}
__device__ __forceinline__ uint32_t bits(Bits &b, int n) {  // n <= 16
    const uint32_t v = peek(b) & ((1u << n) - 1u);
    drop(b, n);
    return v;
}

// a canonical code's per-length numbers, lane l holding those of length l: the count, the first
// code (MSB-first) and the index in sym[] of the first symbol
struct CodeV {
    uint32_t cnt, first, index;
};

// the entry of the next symbol (0: no such code); consumes its codeword and extra bits and puts the
// decoded value (base + extra bits, or the literal / code-length symbol) into `val`.  A code longer
// than the fast table is found by the canonical test from length F + 1 on (RFC 1951 3.2.2)
template <int F>
__device__ __forceinline__ uint32_t decode(Bits &b, const uint32_t *fast, const CodeV &cv, const uint16_t *sym, Table t,
                                           uint32_t &val) {
    const uint32_t v = peek(b);
    uint32_t e = uni(fast[v & ((1u << F) - 1u)]);
    if (!(e & 15u)) {
        e = 0;
        const uint32_t rv = __builtin_bitreverse32(v);
        for (int l = F + 1; l <= 15; ++l) {
            const uint32_t code = rv >> (32 - l);
            const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)cv.first, l);
            if (code - f < (uint32_t)__builtin_amdgcn_readlane((int)cv.cnt, l)) {
                const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)cv.index, l) + code - f;
                e = meaning(t, uni(sym[k]), (uint32_t)l);
                break;
            }
        }
        if (!e) return 0;
    }
    const int cl = (int)(e & 15u), ex = (int)((e >> 4) & 15u);
    val = (e >> 16) + ((uint32_t)(b.bb >> cl) & ((1u << ex) - 1u));
    drop(b, cl + ex);
    return e;
}

// the canonical code of lens[0, n) (RFC 1951 3.2.2): the fast table's entries for codes of up to F
// bits (each lane fills its own symbols'), codes per length (cnt, and in cnt_v: lane l holds the
// count of length l), the symbols in canonical order (sym); false if over-subscribed
template <int F>
__device__ bool build(const uint8_t *lens, int n, uint32_t *fast, uint32_t *cnt, uint16_t *sym, Table t, int lane,
                      CodeV &cv) {
    if (lane < 16) cnt[lane] = 0;
    for (int i = lane; i < (1 << F); i += 64) fast[i] = 0;
    __syncthreads();
    for (int s = lane; s < n; s += 64) {
        const uint32_t l = lens[s];
        if (l) atomicAdd(&cnt[l], 1u);
    }
    __syncthreads();
    uint32_t cnt_v = lane < 16 ? cnt[lane] : 0u;
    cnt_v = lane == 0 ? 0u : cnt_v;
    cv.cnt = cnt_v;
    uint32_t start[16], next[16];              // scalar: the next sym[] slot and the next code per length
    int left = 1;
    uint32_t idx = 0, code = 0;
#pragma unroll
    for (int l = 1; l < 16; ++l) {
        const uint32_t nl = (uint32_t)__builtin_amdgcn_readlane((int)cnt_v, l);
        const uint32_t np = (uint32_t)__builtin_amdgcn_readlane((int)cnt_v, l - 1);
        left = (left << 1) - (int)nl;
        code = (code + np) << 1;               // RFC 1951 3.2.2 step 2
        start[l] = idx;
        next[l] = code;
        if (lane == l) {
            cv.first = code;
            cv.index = idx;
        }
        idx += nl;
    }
    if (left < 0) {                            // over-subscribed (once negative, left only falls)
        __syncthreads();
        return false;
    }
    for (int base = 0; base < n; base += 64) {
        const int s = base + lane;
        const uint32_t l = s < n ? lens[s] : 0u;
#pragma unroll
        for (int ll = 1; ll < 16; ++ll) {
            const uint64_t m = __ballot(l == (uint32_t)ll);
            if (!m) continue;
            if (l == (uint32_t)ll) {
                const uint32_t r = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                sym[start[ll] + r] = (uint16_t)s;
                if (ll <= F) {
                    const uint32_t c = next[ll] + r;
                    const uint32_t rev = __builtin_bitreverse32(c) >> (32 - ll);
                    const uint32_t e = meaning(t, (uint32_t)s, (uint32_t)ll);
                    for (uint32_t k = rev; k < (1u << F); k += 1u << ll) fast[k] = e;
                }
            }
            const uint32_t c = (uint32_t)__popcll(m);
            start[ll] += c;
            next[ll] += c;
        }
    }
    __syncthreads();
    return true;
}

// ---- CRC-32 of the output, as it is stored (gzip's CRC, RFC 1952; zlib's crc32_combine algebra) --
// raw(D) = the CRC register after D from 0 (linear in D); raw(A B) = x^(8|B|) raw(A) + raw(B) mod p,
// and the gzip CRC = raw(D) + x^(8|D|) 0xFFFFFFFF + 0xFFFFFFFF.  The output is stored in rows of
// 1024 bytes, 16 a lane: each lane's raw CRC of its 16 bytes, folded pairwise over the wave (lanes
// l and l + 2^s: x^(8 16 2^s) left + right), is the row's raw CRC, and the running one becomes
// R = x^8192 R + row.  The last, short row is folded in byte by byte.
constexpr uint32_t kPoly = 0xEDB88320u;        // reflected CRC-32 polynomial
__constant__ uint32_t kX2n[32] = {              // x^(2^k) mod p
    0x40000000, 0x20000000, 0x08000000, 0x00800000, 0x00008000, 0xedb88320, 0xb1e6b092, 0xa06a2517,
    0xed627dae, 0x88d14467, 0xd7bbfe6a, 0xec447f11, 0x8e7ea170, 0x6427800e, 0x4d47bae0, 0x09fe548f,
    0x83852d0f, 0x30362f1a, 0x7b5a9cc3, 0x31fec169, 0x9fec022a, 0x6c8dedc4, 0x15d6874d, 0x5fde7a4e,
    0xbad90e37, 0x2e4e5eef, 0x4eaba214, 0xa8a472c0, 0x429a969e, 0x148d302a, 0xc40ba6d0, 0xc4e22c3c};

__device__ __forceinline__ uint32_t mulx(uint32_t b) { return (b >> 1) ^ (kPoly & (0u - (b & 1u))); }
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {   // a b mod p
    uint32_t p = 0;
#pragma unroll
    for (int k = 31; k >= 0; --k) {
        p ^= b & (0u - ((a >> k) & 1u));
        b = mulx(b);
    }
    return p;
}
__device__ uint32_t x8n(uint32_t n) {                     // x^(8 n) mod p: n zero bytes' shift (uniform n)
    uint32_t p = 1u << 31;
    for (int k = 3; n; n >>= 1, ++k)
        if (n & 1u) p = multmodp(kX2n[k & 31], p);
    return p;
}
__device__ __forceinline__ uint32_t crc_word(uint32_t c, uint32_t w) {   // 4 bytes, little-endian
    c ^= w;
#pragma unroll
    for (int i = 0; i < 32; ++i) c = mulx(c);
    return c;
}
// the raw CRC of the wave's 64 consecutive 16-byte pieces (lane l: piece l's raw CRC), uniform
__device__ __forceinline__ uint32_t wave_fold(uint32_t v) {
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const uint32_t right = (uint32_t)__shfl_down((int)v, 1u << s);
        v = multmodp(kX2n[7 + s], v) ^ right;  // x^(8 16 2^s): the right half's length
    }
    return uni(v);                             // (lane 0's: all 64 pieces)
}

// ring bytes [flushed, upto) -> dst, in rows of 1024: whole 4 KiB granules, and with `all` the tail
// too (16 bytes a lane: the slot is 64 KiB, the bytes past isize are not read); every stored byte
// goes into the running raw CRC R
__device__ void flush(const Lds &L, uint8_t *dst, uint32_t &flushed, uint32_t upto, bool all, int lane, uint32_t &R) {
    __syncthreads();
    const uint32_t limit = all ? upto : flushed + (upto - flushed) / kFlush * kFlush;
    const uint32_t o = 16u * (uint32_t)lane;
    while (limit - flushed >= 1024u) {
        const uint4 v = *reinterpret_cast<const uint4 *>(L.ring + (flushed & kRingMask) + o);
        *reinterpret_cast<uint4 *>(dst + flushed + o) = v;
        const uint32_t c = crc_word(crc_word(crc_word(crc_word(0u, v.x), v.y), v.z), v.w);
        R = multmodp(kX2n[13], R) ^ wave_fold(c);   // x^8192: one row
        flushed += 1024u;
    }
    if (all && upto > flushed) {                  // the last row, t < 1024 bytes
        const uint32_t t = upto - flushed, r = flushed & kRingMask;
        if (o < t) *reinterpret_cast<uint4 *>(dst + flushed + o) = *reinterpret_cast<const uint4 *>(L.ring + r + o);
        for (uint32_t i = 0; i < t; ++i) {        // byte by byte, on every lane alike (once a block)
            R ^= uni(L.ring[r + i]);
#pragma unroll
            for (int b = 0; b < 8; ++b) R = mulx(R);
        }
        flushed = upto;
    }
    __threadfence_block();                     // the stored rows visible to the wave's far-match loads
}

// block i: payload src + off[i] (len[i] bytes of raw DEFLATE), output into dst + i * 64 KiB
// (isize[i] bytes) and checked against crc[i] (when crc is given), status[i] = INF_OK or the failure
__global__ __launch_bounds__(64) void inflate_kernel(const uint8_t *__restrict__ src, const uint32_t *__restrict__ off,
                                                     const uint32_t *__restrict__ len,
                                                     const uint32_t *__restrict__ isize,
                                                     const uint32_t *__restrict__ crc, uint8_t *__restrict__ dst,
                                                     uint32_t *__restrict__ status) {
    extern __shared__ __align__(16) uint8_t smem[];
    Lds &L = *reinterpret_cast<Lds *>(smem);
    const uint32_t blk = blockIdx.x;
    const int lane = (int)threadIdx.x;
    const uint32_t o = off[blk], want = isize[blk];
    uint8_t *out = dst + (uint64_t)blk * kOutMax;
    uint32_t st = INF_OK;
    if (want > kOutMax || len[blk] >= (1u << 28)) st = INF_TOO_BIG;
    const uint32_t n = st == INF_OK ? len[blk] : 0u;   // (nothing is read of a refused block)
    Bits b;
    b.w = reinterpret_cast<const uint32_t *>(src + (o & ~3u));
    b.end = (o & 3u) * 8u + n * 8u;
    b.last = ((o & 3u) + n) >> 2;               // the word holding the first byte past the payload
    b.lane = lane;
    window(b, 0);
    seek(b, (o & 3u) * 8u);
    uint32_t p = 0, flushed = 0;                // output bytes so far; of them, stored to HBM
    uint32_t R = 0;                             // raw CRC of the stored bytes
    CodeV lcv = {0, 0, 0}, dcv = {0, 0, 0};
    bool last = false;
    while (st == INF_OK && !last) {
        if (b.pos + 3 > b.end) { st = INF_OVERRUN; break; }
        last = bits(b, 1) != 0;
        const uint32_t type = bits(b, 2);
        if (type == 0) {                        // stored: LEN, NLEN, then LEN bytes
            seek(b, (b.pos + 7u) & ~7u);
            if (b.pos + 32 > b.end) { st = INF_OVERRUN; break; }
            const uint32_t sl = bits(b, 16), nl = bits(b, 16);
            if (sl != (~nl & 0xFFFFu)) { st = INF_BAD_STORED; break; }
            if (b.pos + sl * 8u > b.end) { st = INF_OVERRUN; break; }
            if (p + sl > want) { st = INF_OVERFLOW; break; }
            const uint8_t *s = reinterpret_cast<const uint8_t *>(b.w) + (b.pos >> 3);
            for (uint32_t done = 0; done < sl;) {   // pieces of 4 KiB: the ring's unflushed bytes stay < 8 KiB
                const uint32_t k = min(sl - done, kFlush);
                for (uint32_t j = (uint32_t)lane; j < k; j += 64) L.ring[(p + j) & kRingMask] = s[done + j];
                p += k;
                done += k;
                if (p - flushed >= kFlush) flush(L, out, flushed, p, false, lane, R);
            }
            seek(b, b.pos + sl * 8u);
            continue;
        }
        if (type == 3) { st = INF_BAD_TYPE; break; }
        if (type == 1) {                        // fixed codes (RFC 1951 3.2.6)
            for (int s = lane; s < 288 + 30; s += 64)
                L.lens[s] = (uint8_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5);
            __syncthreads();
            if (!build<kLitBits>(L.lens, 288, L.lfast, L.cnt, L.lsym, T_LIT, lane, lcv) ||
                !build<kDistBits>(L.lens + 288, 30, L.dfast, L.cnt, L.dsym, T_DIST, lane, dcv)) {
                st = INF_BAD_LITCODE;
                break;
            }
        } else {                                // dynamic codes (3.2.7)
            if (b.pos + 14 > b.end) { st = INF_OVERRUN; break; }
            const int nlen = (int)bits(b, 5) + 257, ndist = (int)bits(b, 5) + 1, ncode = (int)bits(b, 4) + 4;
            if (nlen > 286 || ndist > 30) { st = INF_BAD_COUNTS; break; }
            if (lane < 19) L.lens[lane] = 0;
            __syncthreads();
            for (int k = 0; k < ncode; ++k) {   // the code-length code's lengths, 3 bits each
                const uint32_t v = bits(b, 3);
                if (lane == 0) L.lens[kClOrder[k]] = (uint8_t)v;
            }
            __syncthreads();
            if (!build<7>(L.lens, 19, L.dfast, L.cnt, L.dsym, T_CL, lane, dcv)) { st = INF_BAD_CLCODE; break; }
            const int total = nlen + ndist;
            int k = 0;
            while (k < total) {
                if (b.pos > b.end) { st = INF_OVERRUN; break; }
                uint32_t sym;
                if (!decode<7>(b, L.dfast, dcv, L.dsym, T_CL, sym)) { st = INF_BAD_CLSYM; break; }
                if (sym < 16) {
                    if (lane == 0) L.lens[k] = (uint8_t)sym;
                    ++k;
                    continue;
                }
                uint32_t val = 0;
                int rep;
                if (sym == 16) {
                    if (k == 0) { st = INF_BAD_REPEAT; break; }
                    __syncthreads();
                    val = uni(L.lens[k - 1]);
                    rep = 3 + (int)bits(b, 2);
                } else if (sym == 17) {
                    rep = 3 + (int)bits(b, 3);
                } else {
                    rep = 11 + (int)bits(b, 7);
                }
                if (k + rep > total) { st = INF_BAD_REPEAT; break; }
                for (int r = lane; r < rep; r += 64) L.lens[k + r] = (uint8_t)val;
                k += rep;
            }
            if (st != INF_OK) break;
            if (b.pos > b.end) { st = INF_OVERRUN; break; }
            __syncthreads();
            if (uni(L.lens[256]) == 0) { st = INF_NO_EOB; break; }
            if (!build<kLitBits>(L.lens, nlen, L.lfast, L.cnt, L.lsym, T_LIT, lane, lcv)) {
                st = INF_BAD_LITCODE;
                break;
            }
            if (!build<kDistBits>(L.lens + nlen, ndist, L.dfast, L.cnt, L.dsym, T_DIST, lane, dcv)) {
                st = INF_BAD_DISTCODE;
                break;
            }
        }
        // the compressed data of this block
        for (;;) {
            if (b.pos > b.end) { st = INF_OVERRUN; break; }
            uint32_t val;
            const uint32_t e = decode<kLitBits>(b, L.lfast, lcv, L.lsym, T_LIT, val);
            const uint32_t kind = (e >> 8) & 0xFFu;
            if (!e || kind == K_BAD) { st = INF_BAD_CODE; break; }
            if (kind == K_LIT) {
                if (p >= want) { st = INF_OVERFLOW; break; }
                if (lane == 0) L.ring[p & kRingMask] = (uint8_t)val;
                ++p;
            } else if (kind == K_EOB) {
                break;
            } else {
                const uint32_t mlen = val;
                uint32_t dist;
                const uint32_t de = decode<kDistBits>(b, L.dfast, dcv, L.dsym, T_DIST, dist);
                if (!de || ((de >> 8) & 0xFFu) == K_BAD || dist > p) { st = INF_BAD_DIST; break; }
                if (p + mlen > want) { st = INF_OVERFLOW; break; }
                // every source byte precedes p: one iteration moves 64 bytes, overlapping copies too.
                // A source the ring no longer holds (dist + mlen > 16 KiB: it is more than 16 KiB
                // - 258 back, past the unflushed 4 KiB + 258) is read from the stored output
                if (dist + mlen <= kRing) {
                    for (uint32_t j = (uint32_t)lane; j < mlen; j += 64)
                        L.ring[(p + j) & kRingMask] = L.ring[(p - dist + (j < dist ? j : j % dist)) & kRingMask];
                } else {
                    for (uint32_t j = (uint32_t)lane; j < mlen; j += 64)
                        L.ring[(p + j) & kRingMask] = out[p - dist + (j < dist ? j : j % dist)];
                }
                p += mlen;
            }
            if (p - flushed >= kFlush) flush(L, out, flushed, p, false, lane, R);
        }
    }
    if (st == INF_OK && p != want) st = INF_SHORT;
    if (st == INF_OK && b.pos > b.end) st = INF_OVERRUN;
    if (st == INF_OK) {
        flush(L, out, flushed, p, true, lane, R);
        if (crc && (R ^ multmodp(x8n(want), 0xFFFFFFFFu) ^ 0xFFFFFFFFu) != crc[blk]) st = INF_BAD_CRC;
    }
    if (lane == 0) status[blk] = st;
}

// block i's bytes (slot i of `slots`, isize[i] of them) to out + ooff[i], for the blocks inflated
// (status 0): 16 bytes a thread, whole uint4 stores where the destination is aligned
__global__ __launch_bounds__(256) void compact_kernel(const uint8_t *__restrict__ slots, const uint32_t *__restrict__ isize,
                                                      const uint32_t *__restrict__ ooff,
                                                      const uint32_t *__restrict__ status, uint8_t *__restrict__ out) {
    const uint32_t blk = blockIdx.y;
    const uint32_t b0 = 16u * (blockIdx.x * 256u + threadIdx.x);
    const uint32_t n = isize[blk];
    if (status[blk] != INF_OK || b0 >= n) return;
    const uint4 v = *reinterpret_cast<const uint4 *>(slots + (uint64_t)blk * kOutMax + b0);
    uint8_t *d = out + ooff[blk] + b0;
    if (b0 + 16u <= n && ((uintptr_t)d & 15u) == 0) {
        *reinterpret_cast<uint4 *>(d) = v;
        return;
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const uint32_t k = min(16u, n - b0);
    for (uint32_t i = 0; i < k; ++i) d[i] = (uint8_t)(w[i >> 2] >> (8u * (i & 3u)));
}

}  // namespace

// C ABI (include/fc2_ingest.h): n blocks; src must be readable 8 bytes past every payload
extern "C" int fc2_bgzf_inflate_launch(const uint8_t *src, const uint32_t *off, const uint32_t *len,
                                       const uint32_t *isize, const uint32_t *crc, uint8_t *dst, uint32_t *status,
                                       uint32_t n, void *stream) {
    if (!n) return FC2_OK;
    if (!src || !off || !len || !isize || !dst || !status) return fc2::fail(FC2_E_PARAM, "fc2_bgzf_inflate_launch: null argument");
    static bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void *>(inflate_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(Lds)) == hipSuccess;
    }();
    if (!attr) return fc2::fail(FC2_E_HIP, "fc2_bgzf_inflate_launch: cannot reserve the kernel's LDS");
    hipLaunchKernelGGL(inflate_kernel, dim3(n), dim3(64), sizeof(Lds), (hipStream_t)stream, src, off, len, isize, crc,
                       dst, status);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? FC2_OK : fc2::fail(FC2_E_HIP, std::string("fc2_bgzf_inflate_launch: ") + hipGetErrorString(e));
}

// ---- host side: the ingest's batches (fc2_inflate.h) -------------------------------------------
namespace fc2 {
namespace inf {

// the pinned pool: batch buffers the inflated bytes are downloaded into directly (fc2_ingest.cpp's
// batch allocator asks for them), made on first use, kept while a Gpu is open
namespace {
struct Pool {
    struct Buf {
        void *p;
        size_t size;
    };
    std::mutex mu;
    size_t cap = 0;                            // bytes of a new buffer: the largest asked of the pool
    int users = 0, max_buffers = 0;
    std::vector<Buf> idle, all;                // (a buffer keeps the size it was made with)
};
Pool &pool() {
    static Pool *p = new Pool();               // (never destroyed: outlives the static destructors)
    return *p;
}
std::atomic<bool> pool_on{false};

void pool_open(size_t cap, int max_buffers) {
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    ++P.users;
    P.cap = std::max(P.cap, cap);
    P.max_buffers = std::max(P.max_buffers, max_buffers);
    pool_on = true;
}
void pool_drop(Pool &P, void *b) {             // (P.mu held)
    (void)hipHostFree(b);
    for (size_t k = 0; k < P.all.size(); ++k)
        if (P.all[k].p == b) {
            P.all.erase(P.all.begin() + (ptrdiff_t)k);
            break;
        }
}
void pool_close() {
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    if (--P.users > 0) return;
    pool_on = false;
    for (const Pool::Buf &b : P.idle) pool_drop(P, b.p);
    P.idle.clear();                            // (buffers still in use are freed when given back)
    P.cap = 0;
    P.max_buffers = 0;
}
}  // namespace

void *pinned_take(size_t n) {
    if (!pool_on.load(std::memory_order_relaxed)) return nullptr;
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    if (!P.users || n > P.cap) return nullptr;
    for (size_t k = 0; k < P.idle.size(); ++k)
        if (P.idle[k].size >= n) {
            void *b = P.idle[k].p;
            P.idle.erase(P.idle.begin() + (ptrdiff_t)k);
            return b;
        }
    if ((int)P.all.size() >= P.max_buffers) return nullptr;
    void *b = nullptr;
    if (hipHostMalloc(&b, P.cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    P.all.push_back({b, P.cap});
    return b;
}

bool pinned_owns(const void *b) {
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    for (const Pool::Buf &x : P.all)
        if (x.p == b) return true;
    return false;
}

bool pinned_give(void *b) {
    Pool &P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    for (const Pool::Buf &x : P.all)
        if (x.p == b) {
            if (P.users) P.idle.push_back(x);
            else pool_drop(P, b);
            return true;
        }
    return false;
}

// chunks of a batch in flight at once: four chunks of 256 blocks hold half the GPU's 2048 wave slots
// for this kernel (eight 20 KB workgroups a CU), so the breakpoint search's kernels find room
constexpr int kStreams = 4;

struct Gpu {
    int device = 0;
    uint32_t max_blocks = 0;
    size_t src_cap = 0;
    hipStream_t stream[kStreams] = {};
    hipEvent_t done[kStreams] = {};            // blocking-sync: the reader thread sleeps, not spins
    uint8_t *h_src = nullptr, *d_src = nullptr, *d_slots = nullptr, *d_out = nullptr;
    uint32_t *h_meta = nullptr, *d_meta = nullptr;      // off | len | isize | crc | ooff | status
    bool pooled = false;
    // the batch under way (gpu_begin .. gpu_finish)
    char *dest = nullptr;
    uint32_t n = 0;                            // blocks submitted
    uint64_t out = 0;                          // their inflated bytes
    int chunks = 0;
    bool ok = true;
    std::string err;
};

static bool hip_ok(Gpu *g, hipError_t e, const char *what) {
    if (e == hipSuccess) return true;
    if (g->ok) g->err = std::string("GPU inflate: ") + what + ": " + hipGetErrorString(e);
    g->ok = false;
    return false;
}

Gpu *gpu_open(int device, uint32_t max_blocks, size_t pool_cap, std::string &err) {
    Gpu *g = new Gpu();
    g->device = device;
    g->max_blocks = max_blocks;
    g->src_cap = (size_t)max_blocks * kOutMax + 64;      // a BGZF block is at most 64 KiB
    const size_t out = (size_t)max_blocks * kOutMax, meta = (size_t)max_blocks * 6 * sizeof(uint32_t);
    bool ok = hip_ok(g, hipSetDevice(device), "hipSetDevice");
    for (int k = 0; k < kStreams && ok; ++k)
        ok = hip_ok(g, hipStreamCreateWithFlags(&g->stream[k], hipStreamNonBlocking), "stream") &&
             hip_ok(g, hipEventCreateWithFlags(&g->done[k], hipEventBlockingSync | hipEventDisableTiming), "event");
    ok = ok && hip_ok(g, hipHostMalloc((void **)&g->h_src, g->src_cap, hipHostMallocDefault), "pinned input") &&
         hip_ok(g, hipHostMalloc((void **)&g->h_meta, meta, hipHostMallocDefault), "pinned table") &&
         hip_ok(g, hipMalloc((void **)&g->d_src, g->src_cap), "device input") &&
         hip_ok(g, hipMalloc((void **)&g->d_slots, out), "device slots") &&
         hip_ok(g, hipMalloc((void **)&g->d_out, out), "device output") &&
         hip_ok(g, hipMalloc((void **)&g->d_meta, meta), "device table");
    if (!ok) {
        err = g->err;
        gpu_close(g);
        return nullptr;
    }
    if (pool_cap) {              // the batches the parse blocks and the read loop's chunks still hold, and one in flight
        pool_open(pool_cap, 16);
        g->pooled = true;
        void *first[3];                        // the first few made now (pinning takes ~10 ms each)
        for (void *&b : first) b = pinned_take(pool_cap);
        for (void *b : first)
            if (b) pinned_give(b);
    }
    return g;
}

void gpu_close(Gpu *g) {
    if (!g) return;
    if (hipSetDevice(g->device) == hipSuccess) {
        for (int k = 0; k < kStreams; ++k)
            if (g->stream[k]) (void)hipStreamSynchronize(g->stream[k]);
        if (g->d_meta) (void)hipFree(g->d_meta);
        if (g->d_out) (void)hipFree(g->d_out);
        if (g->d_slots) (void)hipFree(g->d_slots);
        if (g->d_src) (void)hipFree(g->d_src);
        if (g->h_meta) (void)hipHostFree(g->h_meta);
        if (g->h_src) (void)hipHostFree(g->h_src);
        for (int k = 0; k < kStreams; ++k) {
            if (g->done[k]) (void)hipEventDestroy(g->done[k]);
            if (g->stream[k]) (void)hipStreamDestroy(g->stream[k]);
        }
    }
    if (g->pooled) pool_close();
    delete g;
}

uint32_t gpu_max_blocks(const Gpu *g) { return g->max_blocks; }

void gpu_begin(Gpu *g, char *dest) {
    g->dest = dest;
    g->n = 0;
    g->out = 0;
    g->chunks = 0;
    g->ok = hipSetDevice(g->device) == hipSuccess;
    g->err = g->ok ? "" : "GPU inflate: hipSetDevice failed";
}

bool gpu_add(Gpu *g, const uint8_t *raw, const size_t *boff, const size_t *bsz, size_t i0, size_t i1) {
    if (!g->ok) return false;
    if (i1 <= i0) return true;
    if (i0 != g->n || i1 > g->max_blocks || boff[i1 - 1] + bsz[i1 - 1] + 8 > g->src_cap) {
        g->ok = false;
        g->err = "GPU inflate: chunk out of order or larger than the buffers";
        return false;
    }
    const uint32_t M = g->max_blocks;
    uint32_t *off = g->h_meta, *len = off + M, *isz = len + M, *crc = isz + M, *ooff = crc + M, *st = ooff + M;
    // the chunk's bytes into the pinned input (at their offsets in the batch), 8 zero bytes behind
    const size_t b0 = boff[i0], b1 = boff[i1 - 1] + bsz[i1 - 1];
    memcpy(g->h_src + b0, raw + b0, b1 - b0);
    memset(g->h_src + b1, 0, 8);
    bool fits = true;
    for (size_t i = i0; i < i1; ++i) {
        const uint8_t *b = raw + boff[i];
        const size_t xl = b[10] | (b[11] << 8);
        off[i] = (uint32_t)(boff[i] + 12 + xl);
        len[i] = (uint32_t)(bsz[i] - 12 - xl - 8);
        const uint8_t *t = b + bsz[i] - 8;
        crc[i] = t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24);
        isz[i] = t[4] | (t[5] << 8) | (t[6] << 16) | ((uint32_t)t[7] << 24);
        ooff[i] = (uint32_t)g->out;
        if (isz[i] > kOutMax) fits = false;
        g->out += std::min<uint32_t>(isz[i], kOutMax);
    }
    g->n = (uint32_t)i1;
    const uint32_t c = (uint32_t)(i1 - i0);
    if (!fits) {                               // not BGZF: the CPU inflates (and reports) these blocks
        for (size_t i = i0; i < i1; ++i) st[i] = INF_TOO_BIG;
        return true;
    }
    hipStream_t s = g->stream[g->chunks++ % kStreams];
    uint32_t *d_off = g->d_meta, *d_len = d_off + M, *d_isz = d_len + M, *d_crc = d_isz + M, *d_ooff = d_crc + M,
             *d_st = d_ooff + M;
    const size_t w = sizeof(uint32_t);
    bool ok = hip_ok(g, hipMemcpyAsync(g->d_src + b0, g->h_src + b0, b1 + 8 - b0, hipMemcpyHostToDevice, s), "upload");
    for (int a = 0; a < 5 && ok; ++a)
        ok = hip_ok(g, hipMemcpyAsync(g->d_meta + (size_t)a * M + i0, g->h_meta + (size_t)a * M + i0, c * w,
                                      hipMemcpyHostToDevice, s), "upload");
    ok = ok && fc2_bgzf_inflate_launch(g->d_src, d_off + i0, d_len + i0, d_isz + i0, d_crc + i0,
                                       g->d_slots + (size_t)i0 * kOutMax, d_st + i0, c, s) == FC2_OK;
    if (!ok) {
        if (g->ok) g->err = "GPU inflate: launch failed";
        g->ok = false;
        return false;
    }
    hipLaunchKernelGGL(compact_kernel, dim3(kOutMax / 16 / 256, c), dim3(256), 0, s, g->d_slots + (size_t)i0 * kOutMax,
                       d_isz + i0, d_ooff + i0, d_st + i0, g->d_out);
    const uint64_t o0 = ooff[i0];
    return hip_ok(g, hipGetLastError(), "compact") &&
           hip_ok(g, hipMemcpyAsync(g->dest + o0, g->d_out + o0, g->out - o0, hipMemcpyDeviceToHost, s), "download") &&
           hip_ok(g, hipMemcpyAsync(st + i0, d_st + i0, c * w, hipMemcpyDeviceToHost, s), "download");
}

bool gpu_finish(Gpu *g, std::string &err) {
    for (int k = 0; k < kStreams; ++k)
        if (hip_ok(g, hipEventRecord(g->done[k], g->stream[k]), "event")) hip_ok(g, hipEventSynchronize(g->done[k]), "kernel");
    if (!g->ok) err = g->err;
    return g->ok;
}

uint32_t gpu_status(const Gpu *g, size_t i) { return g->h_meta[5 * (size_t)g->max_blocks + i]; }

}  // namespace inf
}  // namespace fc2
