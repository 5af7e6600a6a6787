// fc2_kernels.hip -- CDNA4 (gfx950) kernels for find_circ2's breakpoint search.
//
// Hot path: JunctionSpan.find_breakpoints (find_circ.py:854-974) with its
// genome window fetch (indexed_fasta.get_data, find_circ.py:189-215) for a
// whole batch of anchor pairs, one pair per lane.
//
// Per pair the reference tries every breakpoint x in [0, l] and counts
//     dist(x) = #{i < x : A[i] != I[i]} + #{x <= i < l : B[i+2] != I[i]}
// (A/B = upper-cased genome windows of l+2 bases, I = internal read part),
// keeps x with dist <= maxdist whose dinucleotides A[x:x+2]+B[x:x+2] are GTAG
// ('+') or CTAC ('-') (every x with --non-canonical), scores them
// 20*canonical - 10*dist - ov (+100 strand match with --strand-pref) and
// returns the best-score ties in (x ascending, '+' before '-') order.
//
// Here every sequence is held bit-sliced (one bit per base per plane: low code
// bit, high code bit, N), so one 64-bit VALU op compares 64 bases:
//   mismatch(i) = (loA^loI | hiA^hiI | nA^nI)(i)        ('N'=='N' is a match)
//   dist(x)     = popc(mA & below(x)) + popc(mB) - popc(mB & below(x))
//   GTAG mask   = G_A & T_A>>1 & A_B & G_B>>1  (bitwise, all x at once)
// so the O(l^2) byte loop of find_circ.py:906-908 becomes ~NW word ops plus
// a popcount per signal candidate.  The work is integer and HBM-bound (no
// MFMA); see DESIGN.md for the roofline.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fc2_common.h"
#include "fc2_compact.h"
#include "fc2_scan32.h"

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint64_t lowbits(int n) {  // n in any range; bits [0, n)
    return n >= 64 ? ~0ull : (n <= 0 ? 0ull : ((1ull << n) - 1ull));
}

// bits [s, s+64) of the 128-bit value hi:lo, s in [0, 63]
[[maybe_unused]] __device__ __forceinline__ uint64_t fsh(uint64_t lo, uint64_t hi, unsigned s) {
    return s ? ((lo >> s) | (hi << (64u - s))) : lo;
}

// positions [a, b) restricted to word k (positions 64k .. 64k+63)
[[maybe_unused]] __device__ __forceinline__ uint64_t rmask(int a, int b, int k) {
    const int lo = a - 64 * k, hi = b - 64 * k;
    if (hi <= 0 || lo >= 64 || hi <= lo) return 0ull;
    return lowbits(hi) & ~lowbits(lo);
}

template <int NW>
struct Planes {
    uint64_t lo[NW + 1], hi[NW + 1], n[NW + 1];
};

// Streaming (read-once) traffic: optionally non-temporal so it does not evict
// genome lines from L2 / the Infinity Cache.
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ uint64_t ld_stream(const uint64_t *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st_stream(uint64_t *p, uint64_t v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <bool NT>
__device__ __forceinline__ fc2_pair ld_pair(const fc2_pair *p) {
    u64x2 v;
    if constexpr (NT) v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
    else v = *reinterpret_cast<const u64x2 *>(p);
    fc2_pair r;
    __builtin_memcpy(&r, &v, sizeof r);
    return r;
}

// One genome window of W bases starting at chromosome position ws, as three
// bit planes.  Positions outside [0, csize) read as 'N' (get_data's padding,
// find_circ.py:194-211).
template <int NW>
__device__ __forceinline__ void load_window(const fc2_genome_view &g, uint64_t cstart, int64_t csize,
                                            int64_t ws, int W, Planes<NW> &P) {
    if (g.dummy) {
#pragma unroll
        for (int k = 0; k <= NW; ++k) { P.lo[k] = 0; P.hi[k] = 0; P.n[k] = ~0ull; }
        return;
    }
    const int64_t g0 = (int64_t)cstart + ws;
    const int64_t u0 = g0 >> 6;  // floor division
    const unsigned sh = (unsigned)(g0 & 63);
    const ulonglong2 *U = reinterpret_cast<const ulonglong2 *>(g.units);
    uint64_t ul[NW + 2], uh[NW + 2];
#pragma unroll
    for (int j = 0; j <= NW; ++j) {
        const int64_t u = u0 + j;
        const bool need = j <= (((int)sh + W - 1) >> 6);   // units the W window actually spans
        if (need && u >= 0 && (uint64_t)u < g.n_units) {
            const ulonglong2 v = U[u];
            ul[j] = v.x; uh[j] = v.y;
        } else {
            ul[j] = 0; uh[j] = 0;
        }
    }
    ul[NW + 1] = 0; uh[NW + 1] = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        P.lo[k] = fsh(ul[k], ul[k + 1], sh);
        P.hi[k] = fsh(uh[k], uh[k + 1], sh);
    }
    P.lo[NW] = 0; P.hi[NW] = 0;

    // N plane: only touched when the coarse map says a 1024-base block has an N.
    bool anyN = false;
    {
        const int64_t nb = (int64_t)((g.n_units + 15) >> 4);
        const int64_t b0 = u0 >> 4, b1 = (u0 + NW) >> 4;
        if (b0 >= 0 && b0 < nb) anyN |= (g.ncoarse[b0 >> 5] >> (b0 & 31)) & 1u;
        if (b1 != b0 && b1 >= 0 && b1 < nb) anyN |= (g.ncoarse[b1 >> 5] >> (b1 & 31)) & 1u;
    }
    if (anyN) {
        uint64_t un[NW + 2];
#pragma unroll
        for (int j = 0; j <= NW; ++j) {
            const int64_t u = u0 + j;
            un[j] = (u >= 0 && (uint64_t)u < g.n_units) ? g.nplane[u] : 0ull;
        }
        un[NW + 1] = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) P.n[k] = fsh(un[k], un[k + 1], sh);
    } else {
#pragma unroll
        for (int k = 0; k < NW; ++k) P.n[k] = 0;
    }
    P.n[NW] = 0;

    // chromosome bounds -> 'N'
    int64_t vlo = -ws, vhi = csize - ws;
    vlo = vlo < 0 ? 0 : (vlo > W ? W : vlo);
    vhi = vhi < 0 ? 0 : (vhi > W ? W : vhi);
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint64_t v = rmask((int)vlo, (int)vhi, k);
        P.lo[k] &= v; P.hi[k] &= v; P.n[k] = (P.n[k] & v) | ~v;
    }
}

// base code (A0 C1 G2 T3 N4) at runtime position pos < 64*NW
template <int NW>
__device__ __forceinline__ unsigned code_at(const Planes<NW> &P, int pos) {
    const int k = pos >> 6, b = pos & 63;
    unsigned c = 0;
#pragma unroll
    for (int kk = 0; kk < NW; ++kk) {
        if (kk == k) {
            c = ((P.n[kk] >> b) & 1ull) ? 4u
                                        : (unsigned)(((P.lo[kk] >> b) & 1ull) | (((P.hi[kk] >> b) & 1ull) << 1));
        }
    }
    return c;
}

struct Best {
    int n_hits = 0;        // number of Splices appended (find_circ.py:947-954)
    int best_score = 0;
    int best_x = -1;
    int best_minus = 0;
    int best_dist = 0;
    int best_ov = 0;
    int n_ties = 0;
};

__device__ __forceinline__ int ov_of(int x, int l, int margin) {  // find_circ.py:917-922
    int ov = 0;
    if (margin) {
        if (x < margin) ov = margin - x;
        if (l - x < margin) ov = margin - (l - x);
    }
    return ov;
}

__device__ __forceinline__ void add_hit(Best &B, int x, int minus, int dist, int ov, int score) {
    if (B.n_hits == 0 || score > B.best_score) {
        B.best_score = score; B.best_x = x; B.best_minus = minus; B.best_dist = dist; B.best_ov = ov;
        B.n_ties = 1;
    } else if (score == B.best_score) {
        B.n_ties += 1;
    }
    B.n_hits += 1;
}

__device__ __forceinline__ uint64_t pack_result(const Best &B, unsigned gtag12, unsigned err) {
    uint64_t r;
    if (B.n_hits == 0) {
        r = (uint64_t)(uint16_t)(int16_t)-1;
        r |= (uint64_t)(FC2_RES_DONE | err) << 48;
        return r;
    }
    const unsigned nt = B.n_hits >= 2 ? (unsigned)B.n_ties : 1u;   // find_circ.py:961-972
    const unsigned dist = B.best_dist > 255 ? 255u : (unsigned)B.best_dist;
    const unsigned info = FC2_RES_DONE | err | (B.best_minus ? FC2_RES_MINUS : 0u) |
                          ((gtag12 << FC2_RES_GTAG_SHIFT) & FC2_RES_GTAG_MASK);
    r = (uint64_t)(uint16_t)(int16_t)B.best_x;
    r |= (uint64_t)(dist & 0xFF) << 16;
    r |= (uint64_t)(B.best_ov & 0xFF) << 24;
    r |= (uint64_t)(nt > 0xFFFF ? 0xFFFFu : nt) << 32;
    r |= (uint64_t)info << 48;
    return r;
}

__device__ __forceinline__ uint64_t nohit_result(unsigned err) {
    Best B;
    return pack_result(B, 0, err);
}

// ---------------------------------------------------------------------------
// register kernel: one pair per lane, NW 64-bit words per bit plane
// ---------------------------------------------------------------------------
template <int NW, bool NT>
__global__ __launch_bounds__(kBlock) void bp_scan_kernel(fc2_params p, fc2_genome_view g, fc2_batch_view bv,
                                                         uint64_t *__restrict__ out, uint64_t *__restrict__ tiemask,
                                                         uint32_t tw) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= bv.n) return;
    const fc2_pair pr = ld_pair<NT>(bv.pairs + i);
    if (pr.flags & FC2_PAIR_BYTEPATH) return;  // left for the byte-exact kernel

    const int e = p.asize - p.margin;
    const int L = (int)pr.read_len;
    const int l = L - 2 * e;
    const bool want_ties = p.allhits != 0;

    if ((pr.flags & FC2_PAIR_SKIP) || l < 0 || l > 64 * NW - 2 || pr.chrom >= g.n_chrom) {
        unsigned err = 0;
        if (!(pr.flags & FC2_PAIR_SKIP) && l >= 0 && (l > 64 * NW - 2 || pr.chrom >= g.n_chrom)) err = FC2_RES_ERR_WIN;
        st_stream<NT>(out + i, nohit_result(err));
        if (want_ties)
            for (uint32_t k = 0; k < tw; ++k) tiemask[(uint64_t)k * bv.stride + i] = 0;
        return;
    }
    const int W = l + 2;  // flank, find_circ.py:900

    // --- internal read part I[0..l): three bit planes --------------------------
    uint64_t Ilo[NW], Ihi[NW], In[NW];
    {
        uint64_t r[2 * NW + 1];
#pragma unroll
        for (int j = 0; j < 2 * NW; ++j)
            r[j] = ((uint32_t)j < bv.rw) ? ld_stream<NT>(bv.read_words + (uint64_t)j * bv.stride + i) : 0ull;
        r[2 * NW] = 0;
        const int base = l >> 6;
        const unsigned s = (unsigned)(l & 63);
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const uint64_t m = rmask(0, l, k);
            Ilo[k] = r[k] & m;
            uint64_t v = 0;
#pragma unroll
            for (int bb = 0; bb < NW; ++bb)
                if (bb == base) v = fsh(r[bb + k], r[bb + k + 1], s);
            Ihi[k] = v & m;
        }
        if (pr.flags & FC2_PAIR_READ_N) {
#pragma unroll
            for (int k = 0; k < NW; ++k)
                In[k] = ((uint32_t)k < bv.nw ? ld_stream<NT>(bv.read_nwords + (uint64_t)k * bv.stride + i) : 0ull) & rmask(0, l, k);
        } else {
#pragma unroll
            for (int k = 0; k < NW; ++k) In[k] = 0;
        }
    }

    // --- the two genome windows (find_circ.py:900-902) -------------------------
    const uint64_t cstart = g.dummy ? 0ull : g.chrom_start[pr.chrom];
    const int64_t csize = g.dummy ? (int64_t)1 << 62 : g.chrom_size[pr.chrom];
    const int64_t wsA = (int64_t)pr.a_pos + e;
    const int64_t wsB = (int64_t)pr.b_aend - e - W;
    // get_data is only length-preserving for start <= size and end >= 0; the host
    // routes anything else to the byte kernel -- flag defensively here.  The dummy
    // genome's "N"*(end-start) (find_circ.py:370-371) has the requested length anywhere.
    if (!g.dummy && (wsA > csize || wsA + W < 0 || wsB > csize || wsB + W < 0)) {
        st_stream<NT>(out + i, nohit_result(FC2_RES_ERR_WIN));
        if (want_ties)
            for (uint32_t k = 0; k < tw; ++k) tiemask[(uint64_t)k * bv.stride + i] = 0;
        return;
    }
    Planes<NW> A, B;
    load_window<NW>(g, cstart, csize, wsA, W, A);
    load_window<NW>(g, cstart, csize, wsB, W, B);

    // --- mismatch planes ------------------------------------------------------
    uint64_t mA[NW], mB[NW];
    int cA[NW], cB[NW];
    int totB = 0, accA = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint64_t m = rmask(0, l, k);
        mA[k] = ((A.lo[k] ^ Ilo[k]) | (A.hi[k] ^ Ihi[k]) | (A.n[k] ^ In[k])) & m;
        const uint64_t blo = fsh(B.lo[k], B.lo[k + 1], 2), bhi = fsh(B.hi[k], B.hi[k + 1], 2),
                       bn = fsh(B.n[k], B.n[k + 1], 2);
        mB[k] = ((blo ^ Ilo[k]) | (bhi ^ Ihi[k]) | (bn ^ In[k])) & m;
        cA[k] = accA; cB[k] = totB;
        accA += __popcll(mA[k]);
        totB += __popcll(mB[k]);
    }

    // --- splice-signal masks: GTAG -> '+', CTAC -> '-' (find_circ.py:924-954) --
    uint64_t plus[NW], minus[NW];
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint64_t xm = rmask(0, l + 1, k);
        const uint64_t aLo1 = fsh(A.lo[k], A.lo[k + 1], 1), aHi1 = fsh(A.hi[k], A.hi[k + 1], 1);
        const uint64_t bLo1 = fsh(B.lo[k], B.lo[k + 1], 1), bHi1 = fsh(B.hi[k], B.hi[k + 1], 1);
        const uint64_t A_T1 = aHi1 & aLo1;                             // A[x+1] == 'T'
        const uint64_t B_A0 = ~(B.lo[k] | B.hi[k] | B.n[k]);           // B[x]   == 'A'
        const uint64_t A_G0 = A.hi[k] & ~A.lo[k];                      // A[x]   == 'G'
        const uint64_t A_C0 = A.lo[k] & ~A.hi[k];                      // A[x]   == 'C'
        const uint64_t B_G1 = bHi1 & ~bLo1;                            // B[x+1] == 'G'
        const uint64_t B_C1 = bLo1 & ~bHi1;                            // B[x+1] == 'C'
        plus[k] = A_G0 & A_T1 & B_A0 & B_G1 & xm;
        minus[k] = A_C0 & A_T1 & B_A0 & B_C1 & xm;
    }

    const int prim_minus = (pr.flags & FC2_PAIR_PRIMARY_REV) ? 1 : 0;
    const int sp_plus = p.strandpref ? (prim_minus ? 0 : 100) : 0;   // find_circ.py:796-797
    const int sp_minus = p.strandpref ? (prim_minus ? 100 : 0) : 0;
    Best Bst;

    if (!p.noncanonical) {
        // only signal positions can produce hits: iterate their set bits in x order
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            uint64_t w = plus[k] | minus[k];
            while (w) {
                const int b = __ffsll((long long)w) - 1;
                w &= w - 1;
                const int x = 64 * k + b;
                const uint64_t below = lowbits(b);
                const int dist = cA[k] + __popcll(mA[k] & below) + totB - (cB[k] + __popcll(mB[k] & below));
                if (dist <= p.maxdist) {
                    const int ov = ov_of(x, l, p.margin);
                    const int isminus = (int)((minus[k] >> b) & 1ull);
                    const int score = 20 - 10 * dist - ov + (isminus ? sp_minus : sp_plus);
                    add_hit(Bst, x, isminus, dist, ov, score);
                }
            }
        }
    } else {
        // every x with dist <= maxdist yields a '+' and a '-' Splice (find_circ.py:947-949)
        int d = totB;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            for (int b = 0; b < 64; ++b) {
                const int x = 64 * k + b;
                if (x > l) break;
                if (d <= p.maxdist) {
                    const int ov = ov_of(x, l, p.margin);
                    const int cp = (int)((plus[k] >> b) & 1ull), cm = (int)((minus[k] >> b) & 1ull);
                    add_hit(Bst, x, 0, d, ov, 20 * cp - 10 * d - ov + sp_plus);
                    add_hit(Bst, x, 1, d, ov, 20 * cm - 10 * d - ov + sp_minus);
                }
                d += (int)((mA[k] >> b) & 1ull) - (int)((mB[k] >> b) & 1ull);
            }
        }
    }

    unsigned gtag12 = 0;
    if (Bst.n_hits) {
        const int x = Bst.best_x;
        gtag12 = code_at<NW>(A, x) | (code_at<NW>(A, x + 1) << 3) | (code_at<NW>(B, x) << 6) |
                 (code_at<NW>(B, x + 1) << 9);
    }
    st_stream<NT>(out + i, pack_result(Bst, gtag12, 0));

    if (want_ties) {
        // --all-hits: mark every tie (find_circ.py:966-974), second pass over the same hits
        uint64_t tp[NW], tm[NW];
#pragma unroll
        for (int k = 0; k < NW; ++k) { tp[k] = 0; tm[k] = 0; }
        if (Bst.n_hits) {
            const int best = Bst.best_score;
            if (!p.noncanonical) {
#pragma unroll
                for (int k = 0; k < NW; ++k) {
                    uint64_t w = plus[k] | minus[k];
                    while (w) {
                        const int b = __ffsll((long long)w) - 1;
                        w &= w - 1;
                        const int x = 64 * k + b;
                        const uint64_t below = lowbits(b);
                        const int dist = cA[k] + __popcll(mA[k] & below) + totB - (cB[k] + __popcll(mB[k] & below));
                        if (dist <= p.maxdist) {
                            const int isminus = (int)((minus[k] >> b) & 1ull);
                            const int score = 20 - 10 * dist - ov_of(x, l, p.margin) + (isminus ? sp_minus : sp_plus);
                            if (score == best) {
                                if (isminus) tm[k] |= 1ull << b; else tp[k] |= 1ull << b;
                            }
                        }
                    }
                }
            } else {
                int d = totB;
#pragma unroll
                for (int k = 0; k < NW; ++k) {
                    for (int b = 0; b < 64; ++b) {
                        const int x = 64 * k + b;
                        if (x > l) break;
                        if (d <= p.maxdist) {
                            const int ov = ov_of(x, l, p.margin);
                            const int cp = (int)((plus[k] >> b) & 1ull), cm = (int)((minus[k] >> b) & 1ull);
                            if (20 * cp - 10 * d - ov + sp_plus == best) tp[k] |= 1ull << b;
                            if (20 * cm - 10 * d - ov + sp_minus == best) tm[k] |= 1ull << b;
                        }
                        d += (int)((mA[k] >> b) & 1ull) - (int)((mB[k] >> b) & 1ull);
                    }
                }
            }
        }
        const uint32_t half = tw / 2;
        for (uint32_t k = 0; k < half; ++k) {
            uint64_t vp = 0, vm = 0;
#pragma unroll
            for (int kk = 0; kk < NW; ++kk)
                if ((uint32_t)kk == k) { vp = tp[kk]; vm = tm[kk]; }
            tiemask[(uint64_t)k * bv.stride + i] = vp;
            tiemask[(uint64_t)(half + k) * bv.stride + i] = vm;
        }
    }
}

// ---------------------------------------------------------------------------
// byte-exact kernel: any bytes, any read length (rare pairs)
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool is_acgtn(uint8_t c) {
    return c == 'A' || c == 'C' || c == 'G' || c == 'T' || c == 'N';
}
__device__ __forceinline__ unsigned code_of(uint8_t c) {
    return c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
}

// find_breakpoints (find_circ.py:854-974) of one pair on the bytes of its arena block (fc2_bytes_view
// layout): the best hit and its tie count into Bst, a reference error into err, the best hit's
// 4-mer into gtag12; with --all-hits every tie of the best score goes to tie(strand, x) in a second
// pass (x ascending, as the stable sort keeps them).  L = len(read_part) (< 2^31).
template <class Tie>
__device__ __forceinline__ void bytes_eval(const fc2_params &p, int L, uint8_t flags, const uint8_t *blk, Best &Bst,
                                           unsigned &err, unsigned &gtag12, Tie tie) {
    err = 0;
    gtag12 = 0;
    const int e = p.asize - p.margin;
    const int l = L - 2 * e;
    if ((flags & FC2_PAIR_SKIP) || l < 0) return;
    const int lenI = ((const int32_t *)blk)[0], lenA = ((const int32_t *)blk)[1], lenB = ((const int32_t *)blk)[2];
    const int tailB = ((const int32_t *)blk)[3];      // lenI == 1: B's bytes past its slot that differ from I[0]
    const int64_t lc = l;
    const int64_t slotA = lc + 3, slotB = 2 * lc + 3;   // stored bytes per window (fc2_bytepath_fill)
    const uint8_t *I = blk + 16;
    const uint8_t *Af = I + lenI;
    const uint8_t *Bf = Af + slotA;
    const int64_t sB = lenB < slotB ? lenB : slotB;     // A is only read below x + 2 <= l + 2 < slotA
    const bool want_ties = p.allhits != 0;

    // Windows normally have l+2 bytes.  Outside get_data's defined range they can
    // come back shorter or longer (find_circ.py:194-211), and with asize <= margin the
    // internal part read[e:-e] (:895) is not l bytes long; then the literal string form
    // of find_circ.py:907-908 is followed byte by byte: with -d 0, simple_match's `!=`
    // of unequal strings is True (:865-866, never a hit); otherwise numpy compares the
    // two byte arrays (:861-863) -- equal lengths elementwise, a 1-byte operand broadcast
    // against the other, anything else fails (-> ERR_WIN).
    const bool regular = (lenI == l && lenA == l + 2 && lenB == l + 2);
    int totB = 0;
    if (regular)
        for (int j = 0; j < l; ++j) totB += Bf[j + 2] != I[j];
    const int prim_minus = (flags & FC2_PAIR_PRIMARY_REV) ? 1 : 0;
    const int sp_plus = p.strandpref ? (prim_minus ? 0 : 100) : 0;
    const int sp_minus = p.strandpref ? (prim_minus ? 100 : 0) : 0;
    for (int pass = 0; pass < (want_ties ? 2 : 1); ++pass) {
        int d = totB;
        for (int x = 0; x <= l; ++x) {
            if (regular) {
                if (x > 0) d += (int)(Af[x - 1] != I[x - 1]) - (int)(Bf[x + 1] != I[x - 1]);
            } else {
                const int64_t n1 = x < lenA ? x : lenA;                                // A_flank[:x]
                const int64_t n2 = (int64_t)lenB - (x + 2) > 0 ? (int64_t)lenB - (x + 2) : 0;   // B_flank[x+2:]
                const int64_t sl = n1 + n2;
                int64_t dd = 0;
                if (sl == lenI) {   // B[x+2 : x+2+n2] lies in its slot: x + 2 + n2 <= l + 2 + lenI <= 2l + 2
                    for (int64_t j = 0; j < n1; ++j) dd += Af[j] != I[j];
                    for (int64_t j = 0; j < n2; ++j) dd += Bf[x + 2 + j] != I[n1 + j];
                    if (p.maxdist == 0) dd = dd != 0;                                  // the bool a != b
                } else if (p.maxdist == 0) {
                    continue;  // simple_match: unequal strings never qualify (find_circ.py:865-866)
                } else if (lenI == 1 && sl > 0) {                                      // I broadcast over spliced
                    const uint8_t c = I[0];
                    for (int64_t j = 0; j < n1; ++j) dd += Af[j] != c;
                    const int64_t b0 = x + 2, b1 = x + 2 + n2;                         // B bytes [b0, b1)
                    const int64_t st = b1 < sB ? b1 : sB;
                    for (int64_t j = b0; j < st; ++j) dd += Bf[j] != c;
                    if (b1 > sB) dd += tailB;                                          // B[slotB:], b0 < slotB
                } else if (sl == 1 && lenI > 0) {                                      // spliced[0] broadcast
                    const uint8_t c = n1 ? Af[0] : Bf[x + 2];                          // x + 2 < slotB
                    for (int j = 0; j < lenI; ++j) dd += I[j] != c;
                } else if (!((sl == 0 && lenI == 1) || (sl == 1 && lenI == 0))) {
                    err = FC2_RES_ERR_WIN;  // shapes numpy cannot broadcast
                    break;
                }                            // else (0,) against (1,): an empty comparison, dist 0
                d = dd > 0x7FFFFFFF ? 0x7FFFFFFF : (int)dd;
            }
            if (d > p.maxdist) continue;
            const bool have4 = (x + 1 < lenA) && (x + 1 < lenB);
            const uint8_t g0 = x < lenA ? Af[x] : 0, g1 = have4 ? Af[x + 1] : 0;
            const uint8_t g2 = x < lenB ? Bf[x] : 0, g3 = have4 ? Bf[x + 1] : 0;
            if (!(have4 && is_acgtn(g0) && is_acgtn(g1) && is_acgtn(g2) && is_acgtn(g3))) { err = FC2_RES_ERR_KEY; break; }
            const int cp = (g0 == 'G' && g1 == 'T' && g2 == 'A' && g3 == 'G');
            const int cm = (g0 == 'C' && g1 == 'T' && g2 == 'A' && g3 == 'C');
            const int ov = ov_of(x, l, p.margin);
            if (p.noncanonical) {
                const int s1 = 20 * cp - 10 * d - ov + sp_plus, s2 = 20 * cm - 10 * d - ov + sp_minus;
                if (pass == 0) { add_hit(Bst, x, 0, d, ov, s1); add_hit(Bst, x, 1, d, ov, s2); }
                else {
                    if (s1 == Bst.best_score) tie(0, x);
                    if (s2 == Bst.best_score) tie(1, x);
                }
            } else if (cp || cm) {
                const int s = 20 - 10 * d - ov + (cm ? sp_minus : sp_plus);
                if (pass == 0) add_hit(Bst, x, cm, d, ov, s);
                else if (s == Bst.best_score) tie(cm, x);
            }
        }
        if (err || !Bst.n_hits) break;
    }
    if (!err && Bst.n_hits) {
        const int x = Bst.best_x;
        gtag12 = code_of(Af[x]) | (code_of(Af[x + 1]) << 3) | (code_of(Bf[x]) << 6) | (code_of(Bf[x + 1]) << 9);
    }
}

__global__ __launch_bounds__(kBlock) void bp_bytes_kernel(fc2_params p, fc2_bytes_view v, uint64_t *__restrict__ out,
                                                          uint64_t *__restrict__ tiemask, uint32_t tw, uint64_t stride) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= v.m) return;
    const uint64_t i = v.index[k];
    const fc2_pair pr = v.pairs[k];
    const uint32_t half = tw / 2;
    if (p.allhits)
        for (uint32_t w = 0; w < tw; ++w) tiemask[(uint64_t)w * stride + i] = 0;
    Best Bst;
    unsigned err, gtag12;
    bytes_eval(p, (int)pr.read_len, pr.flags, v.arena + v.off[k], Bst, err, gtag12, [&](int minus, int x) {
        tiemask[(uint64_t)((minus ? half : 0) + (uint32_t)(x >> 6)) * stride + i] |= 1ull << (x & 63);
    });
    out[i] = err ? nohit_result(err) : pack_result(Bst, gtag12, 0);
}

// Long pairs (fc2_long_pair): the same evaluation with 32-bit results; pair j's ties at
// ties[tie_off[j] ...] ('+' half, then '-' half)
__global__ __launch_bounds__(kBlock) void bp_long_kernel(fc2_params p, uint64_t n, const fc2_long_pair *__restrict__ pairs,
                                                         const uint64_t *__restrict__ off, const uint8_t *__restrict__ arena,
                                                         const uint64_t *__restrict__ tie_off,
                                                         fc2_long_result *__restrict__ out, uint64_t *__restrict__ ties) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    const fc2_long_pair pr = pairs[j];
    uint64_t *tj = nullptr;
    uint64_t half = 0;
    if (p.allhits) {
        tj = ties + tie_off[j];
        half = (tie_off[j + 1] - tie_off[j]) / 2;
        for (uint64_t w = 0; w < 2 * half; ++w) tj[w] = 0;
    }
    Best Bst;
    unsigned err, gtag12;
    bytes_eval(p, (int)pr.read_len, pr.flags, arena + off[j], Bst, err, gtag12, [&](int minus, int x) {
        tj[(minus ? half : 0) + (uint64_t)(x >> 6)] |= 1ull << (x & 63);
    });
    fc2_long_result r;
    r._pad = 0;
    if (err || !Bst.n_hits) {
        r.best_x = -1;
        r.n_ties = 0;
        r.dist = 0;
        r.ov = 0;
        r.info = (uint16_t)(FC2_RES_DONE | err);
    } else {
        r.best_x = Bst.best_x;
        r.n_ties = Bst.n_hits >= 2 ? (uint32_t)Bst.n_ties : 1u;                   // find_circ.py:961-972
        r.dist = (uint8_t)(Bst.best_dist > 255 ? 255 : Bst.best_dist);
        r.ov = (uint8_t)Bst.best_ov;
        r.info = (uint16_t)(FC2_RES_DONE | (Bst.best_minus ? FC2_RES_MINUS : 0u) |
                            ((gtag12 << FC2_RES_GTAG_SHIFT) & FC2_RES_GTAG_MASK));
    }
    out[j] = r;
}

// ---------------------------------------------------------------------------
// synthetic workloads (bench / tests): counter-based RNG, fully reproducible
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t smix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void synth_genome_kernel(uint64_t seed, uint64_t *units, uint64_t *nplane, uint64_t n_units,
                                    const int64_t *n_lo, const int64_t *n_hi, uint32_t n_iv) {
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n_units) return;
    uint64_t lo = smix(seed * 0x2545F4914F6CDD1Dull ^ (2 * u));
    uint64_t hi = smix(seed * 0x2545F4914F6CDD1Dull ^ (2 * u + 1));
    const int64_t b0 = (int64_t)u * 64, b1 = b0 + 64;
    // first interval with n_hi > b0
    uint32_t a = 0, z = n_iv;
    while (a < z) {
        const uint32_t m = (a + z) >> 1;
        if (n_hi[m] <= b0) a = m + 1; else z = m;
    }
    uint64_t nm = 0;
    for (uint32_t k = a; k < n_iv && n_lo[k] < b1; ++k) {
        const int64_t s = n_lo[k] > b0 ? n_lo[k] - b0 : 0;
        const int64_t t = n_hi[k] < b1 ? n_hi[k] - b0 : 64;
        nm |= lowbits((int)t) & ~lowbits((int)s);
    }
    units[2 * u] = lo & ~nm;
    units[2 * u + 1] = hi & ~nm;
    nplane[u] = nm;
}

__global__ void coarse_kernel(const uint64_t *nplane, uint32_t *ncoarse, uint64_t n_units) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t n_blocks = (n_units + 15) >> 4;
    const uint64_t n_words = (n_blocks + 31) >> 5;
    if (w >= n_words) return;
    uint32_t bits = 0;
    for (int b = 0; b < 32; ++b) {
        const uint64_t blk = w * 32 + b;
        if (blk >= n_blocks) break;
        uint64_t acc = 0;
        for (int j = 0; j < 16; ++j) {
            const uint64_t u = blk * 16 + j;
            if (u < n_units) acc |= nplane[u];
        }
        if (acc) bits |= 1u << b;
    }
    ncoarse[w] = bits;
}

struct Rng {
    uint64_t s;
    __device__ uint64_t next() { s += 0x9E3779B97F4A7C15ull; return smix(s); }
    __device__ float uni() { return (float)(next() >> 40) * (1.0f / 16777216.0f); }
    __device__ int64_t below(int64_t n) { return n <= 0 ? 0 : (int64_t)(next() % (uint64_t)n); }
};

__device__ __forceinline__ unsigned gbase(const fc2_genome_view &g, uint64_t cstart, int64_t csize, int64_t p) {
    if (g.dummy || p < 0 || p >= csize) return 4u;
    const uint64_t q = cstart + (uint64_t)p;
    const uint64_t u = q >> 6;
    const unsigned b = (unsigned)(q & 63);
    if ((g.nplane[u] >> b) & 1ull) return 4u;
    return (unsigned)(((g.units[2 * u] >> b) & 1ull) | (((g.units[2 * u + 1] >> b) & 1ull) << 1));
}

__device__ __forceinline__ bool dinuc(const fc2_genome_view &g, uint64_t cs, int64_t sz, int64_t q, unsigned c0, unsigned c1) {
    return gbase(g, cs, sz, q) == c0 && gbase(g, cs, sz, q + 1) == c1;
}

constexpr unsigned cA = 0, cC = 1, cG = 2, cT = 3;

__global__ void synth_pairs_kernel(fc2_params p, fc2_synth_cfg cfg, fc2_genome_view g, const int64_t *chrom_cum,
                                   uint64_t n, fc2_pair *pairs, uint64_t *read_words, uint32_t rw,
                                   uint64_t *read_nwords, uint32_t nw, uint64_t stride, int32_t *truth) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Rng R{smix(cfg.seed ^ smix(cfg.first + i + 0x51ED2701ull))};
    const int e = p.asize - p.margin;
    const int amin = p.asize;
    const int64_t total = chrom_cum[g.n_chrom];
    // three-segment reads: stream pairs 2s and 2s+1 are the two anchor
    // pairs (s1,s2), (s2,s3) of ONE read from a short circle [start, end) of length c, read =
    // G[end-k1:end] + G[start:end] + G[start:start+k3]; both pairs draw the slot's geometry from the
    // slot's own stream, so a share boundary may split a slot (each pair depends on seed + index)
    const uint64_t gi = cfg.first + i;
    const uint64_t slot = gi >> 1;
    bool three = false;
    if (cfg.p_three_seg > 0.f && cfg.len_max >= 3 * amin) {   // (rows are sized for len_max)
        Rng RS{smix(cfg.seed ^ smix(slot * 0x2545F4914F6CDD1Dull + 0x3A5E9ull))};
        three = RS.uni() < cfg.p_three_seg;
    }
    int L, kA, kB;
    bool bs;
    uint32_t chrom = 0;
    uint64_t cs = 0;
    int64_t sz = 0, A0 = 0, B0 = 0, t0 = 0, t1 = 0;
    int64_t tg0 = 0;                // read position of read_part[0] (three-segment pair (s2,s3): k1)
    bool ok = false;
    bool prim_rev;
    int c0 = 0, c1 = 0;
    if (three) {
        Rng R3{smix(cfg.seed ^ smix(slot * 0x9E3779B97F4A7C15ull + 0x7C3E5ull))};
        int L3 = cfg.len_min + (int)R3.below(cfg.len_max - cfg.len_min + 1);
        if (L3 < 3 * amin) L3 = 3 * amin;
        // the read wraps the circle once: k1, k3 <= c (c >= L/3), every segment >= asize
        const int cmin = (L3 + 2) / 3 > amin ? (L3 + 2) / 3 : amin;
        const int c = cmin + (int)R3.below(L3 - 2 * amin - cmin + 1);
        const int klo = L3 - 2 * c > amin ? L3 - 2 * c : amin;
        const int khi = c < L3 - c - amin ? c : L3 - c - amin;
        const int k1 = klo + (int)R3.below(khi - klo + 1);
        const int k3 = L3 - c - k1;
        const bool planted = R3.uni() < cfg.p_planted;
        const bool msite = R3.uni() < cfg.p_minus_site;
        prim_rev = (R3.next() & 1ull) != 0;
        for (int attempt = 0; attempt < 16 && !ok; ++attempt) {
            int64_t gp = R3.below(total);
            uint32_t a = 0, z = g.n_chrom;
            while (z - a > 1) {
                const uint32_t m = (a + z) >> 1;
                if (chrom_cum[m] <= gp) a = m; else z = m;
            }
            chrom = a;
            cs = g.chrom_start[chrom];
            sz = g.chrom_size[chrom];
            int64_t end = gp - chrom_cum[chrom];
            if (planted) {      // donor at end, acceptor before end - c (both ends of the circle)
                for (int q = 0; q < 512; ++q)
                    if (dinuc(g, cs, sz, end + q, msite ? cC : cG, cT) &&
                        dinuc(g, cs, sz, end + q - c - 2, cA, msite ? cC : cG)) { end = end + q; break; }
            }
            const int64_t start = end - c;
            if (start >= 0 && end <= sz && gbase(g, cs, sz, end - 1) < 4u && gbase(g, cs, sz, start) < 4u) {
                t0 = start; t1 = end; ok = true;
            }
        }
        bs = true;
        if (!(gi & 1)) { kA = k1; kB = c; A0 = t1 - k1; tg0 = 0; }     // (s1, s2)
        else           { kA = c; kB = k3; A0 = t0; tg0 = k1; }        // (s2, s3)
        B0 = t0;
        if (!ok) A0 = B0 = 0;       // SKIP
        L = kA + kB;
    } else {
    L = cfg.len_min + (int)R.below(cfg.len_max - cfg.len_min + 1);
    if (L < 2 * amin) L = 2 * amin;
    kA = amin + (int)R.below(L - 2 * amin + 1);
    kB = L - kA;
    bs = R.uni() < cfg.p_backsplice;
    const bool planted = R.uni() < cfg.p_planted;
    const bool msite = R.uni() < cfg.p_minus_site;

    for (int attempt = 0; attempt < 16 && !ok; ++attempt) {
        int64_t gp;
        if (cfg.locus_ordered) {   // i-th of n strata (redraws stay in the stratum's neighbourhood)
            const double s = ((double)i + (double)R.uni()) / (double)n;
            gp = (int64_t)(s * (double)total) + (attempt ? R.below(4096) : 0);
            if (gp >= total) gp = total - 1;
        } else {
            gp = R.below(total);
        }
        uint32_t a = 0, z = g.n_chrom;  // chrom_cum[c] <= gp < chrom_cum[c+1]
        while (z - a > 1) {
            const uint32_t m = (a + z) >> 1;
            if (chrom_cum[m] <= gp) a = m; else z = m;
        }
        chrom = a;
        cs = g.chrom_start[chrom];
        sz = g.chrom_size[chrom];
        const int64_t off = gp - chrom_cum[chrom];
        const int64_t span = cfg.span_min + R.below(cfg.span_max - cfg.span_min + 1);
        if (bs) {
            // exon [start, end): read = G[end-kA:end] + G[start:start+kB]
            int64_t end = off;
            if (planted) {
                for (int q = 0; q < 512; ++q)
                    if (dinuc(g, cs, sz, off + q, msite ? cC : cG, cT)) { end = off + q; break; }
            }
            int64_t start = end - (span > (int64_t)(kA > kB ? kA : kB) ? span : (int64_t)(kA > kB ? kA : kB) + 1);
            if (planted) {
                for (int q = 0; q < 512; ++q)
                    if (dinuc(g, cs, sz, start - 2 - q, cA, msite ? cC : cG)) { start = start - q; break; }
            }
            // real alignments never sit on 'N': redraw loci whose junction bases are N
            if (start >= 0 && end <= sz && end - kA >= 0 && start + kB <= end && kA <= end - start &&
                gbase(g, cs, sz, end - 1) < 4u && gbase(g, cs, sz, start) < 4u) {
                A0 = end - kA; B0 = start; t0 = start; t1 = end; ok = true;
            }
        } else {
            // intron [d, a): read = G[d-kA:d] + G[a:a+kB]
            int64_t d = off;
            if (planted) {
                for (int q = 0; q < 512; ++q)
                    if (dinuc(g, cs, sz, off + q, msite ? cC : cG, cT)) { d = off + q; break; }
            }
            int64_t a = d + span;
            if (planted) {
                for (int q = 0; q < 512; ++q)
                    if (dinuc(g, cs, sz, a - 2 + q, cA, msite ? cC : cG)) { a = a + q; break; }
            }
            if (d - kA >= 0 && a + kB <= sz && a > d && gbase(g, cs, sz, d - 1) < 4u && gbase(g, cs, sz, a) < 4u) {
                A0 = d - kA; B0 = a; t0 = d; t1 = a; ok = true;
            }
        }
    }
    if (R.uni() < cfg.p_clip) { c0 = (int)R.below(4); c1 = (int)R.below(4); }
    prim_rev = (R.next() & 1ull) != 0;
    }
    const int Lp = L - c0 - c1;
    const int l = Lp - 2 * e;
    fc2_pair pr;
    pr.a_pos = (int32_t)(A0 + c0);
    pr.b_aend = (int32_t)(B0 + kB - c1);
    pr.chrom = chrom;
    pr.read_len = (uint16_t)Lp;
    pr.flags = (uint8_t)((bs ? FC2_PAIR_BACKSPLICE : 0u) | (prim_rev ? FC2_PAIR_PRIMARY_REV : 0u) |
                         (ok ? 0u : FC2_PAIR_SKIP));
    pr.npos = 0;
    if (truth) { truth[2 * i] = ok ? (int32_t)t0 : -1; truth[2 * i + 1] = ok ? (int32_t)t1 : -1; }

    // internal bases I[j] = read[c0 + e + j], j < l ; read[t] = t < kA ? G[A0+t] : G[B0+t-kA]
    uint64_t wlo = 0, whi_first = 0;
    (void)whi_first;
    bool anyN = false;
    int n_count = 0, n_first = 0;
    // pass 1: low plane bits [0,l) and N words; pass 2: high plane bits [l,2l)
    uint32_t wi = 0;   // next read word to store
    uint64_t acc = 0;
    int accn = 0;
    uint64_t nacc = 0;
    uint32_t ni = 0;
    const int lim = l > 0 ? l : 0;
    for (int pass = 0; pass < 2; ++pass) {
        Rng R2{smix(cfg.seed ^ smix((cfg.first + i) * 0x9E37ull + 0xABCDEFull))};   // same mutation stream both passes
        for (int j = 0; j < lim; ++j) {
            const int t = c0 + e + j;
            // a three-segment read's two pairs share its bases: mutations keyed by read position
            if (three) R2.s = smix(cfg.seed ^ smix(slot * 0x100000001B3ull + (uint64_t)(tg0 + t) * 0x9E37ull + 0x55ull));
            unsigned c = t < kA ? gbase(g, cs, sz, A0 + t) : gbase(g, cs, sz, B0 + t - kA);
            if (R2.uni() < cfg.mut_rate) c = (c >= 4u) ? (unsigned)R2.below(4) : ((c + 1u + (unsigned)R2.below(3)) & 3u);
            else (void)R2.next();
            if (R2.uni() < cfg.n_rate) c = 4u;
            const uint64_t bit = pass == 0 ? (c == 4u ? 0ull : (c & 1ull)) : (c == 4u ? 0ull : ((c >> 1) & 1ull));
            acc |= bit << accn;
            if (++accn == 64) {
                if (wi < rw) read_words[(uint64_t)wi * stride + i] = acc;
                ++wi; acc = 0; accn = 0;
            }
            if (pass == 0) {
                if (c == 4u) {
                    anyN = true;
                    nacc |= 1ull << (j & 63);
                    if (n_count++ == 0) n_first = j;
                }
                if ((j & 63) == 63 || j == lim - 1) {
                    if (ni < nw && read_nwords) read_nwords[(uint64_t)ni * stride + i] = nacc;
                    ++ni; nacc = 0;
                }
            }
        }
    }
    if (accn) { if (wi < rw) read_words[(uint64_t)wi * stride + i] = acc; ++wi; }
    for (; wi < rw; ++wi) read_words[(uint64_t)wi * stride + i] = 0;
    if (read_nwords)
        for (; ni < nw; ++ni) read_nwords[(uint64_t)ni * stride + i] = 0;
    (void)wlo;
    if (anyN) pr.flags |= FC2_PAIR_READ_N;
    if (n_count == 1 && n_first < 256) {
        pr.flags |= FC2_PAIR_READ_N1;
        pr.npos = (uint8_t)n_first;
    }
    pairs[i] = pr;
}

inline int hip_check(hipError_t e, const char *what) {
    if (e != hipSuccess) return fc2::fail(FC2_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return FC2_OK;
}

// units_twin[w] = units[w - 8] (4 units = 8 words later), zero outside the genome
__global__ void twin_kernel(const uint64_t *__restrict__ units, uint64_t n_units, uint64_t *__restrict__ twin) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= 2 * (n_units + 8)) return;
    twin[w] = (w >= 8 && w - 8 < 2 * n_units) ? units[w - 8] : 0ull;
}

// Word-pair layout (fc2_genome_view.wt): pair q = (low, high) 32-bit code words of bases
// [32q, 32q + 32), i.e. 32-bit halves of units[2u] / units[2u+1] with u = q >> 1.  The main copy holds
// pair q at slot q + 16 (16 zero pairs in front, 16 behind), then (at twin_off) the copy with pair q at
// slot q + 8.  Zero outside the genome.
__device__ __forceinline__ uint64_t wt_pair(const uint64_t *__restrict__ units, uint64_t n_q, int64_t q) {
    if (q < 0 || (uint64_t)q >= n_q) return 0ull;
    const uint64_t u = (uint64_t)q >> 1;
    const unsigned s = 32u * (unsigned)(q & 1);
    return ((units[2 * u] >> s) & 0xFFFFFFFFull) | (((units[2 * u + 1] >> s) & 0xFFFFFFFFull) << 32);
}

__global__ void wtab_kernel(const uint64_t *__restrict__ units, uint64_t n_units, uint64_t *__restrict__ wt,
                            uint64_t twin_pairs, uint64_t total_pairs) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= total_pairs) return;
    const uint64_t n_q = 2 * n_units;
    wt[j] = j < twin_pairs ? wt_pair(units, n_q, (int64_t)j - 16) : wt_pair(units, n_q, (int64_t)(j - twin_pairs) - 8);
}

// nsuper word w: bit b = OR of the coarse bits of blocks [(32w+b) << (shift-10), +1 << (shift-10))
__global__ void nsuper_kernel(const uint32_t *__restrict__ ncoarse, uint64_t n_units, uint32_t shift, uint32_t words,
                              uint32_t *__restrict__ nsuper) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    const uint64_t nb = (n_units + 15) >> 4;               // coarse blocks
    const uint64_t per = 1ull << (shift - 10);             // coarse blocks per super bit
    uint32_t out = 0;
    for (uint32_t b = 0; b < 32; ++b) {
        const uint64_t c0 = ((uint64_t)w * 32 + b) * per;
        bool any = false;
        for (uint64_t c = c0; c < c0 + per && c < nb && !any; ++c) any = (ncoarse[c >> 5] >> (c & 31)) & 1u;
        out |= (uint32_t)any << b;
    }
    nsuper[w] = out;
}

inline unsigned grid_for(uint64_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

// Tuning knobs (fc2_set_tuning) exist only in A/B builds (-DFC2_AB_FORMS=1, libfc2_ab.so), with the
// measured-and-rejected forms they select; the shipped library has the defaults as constants, so it
// keeps no mutable process-global state and instantiates only the forms the defaults pick.
#if FC2_AB_FORMS
int g_stream_nt = 1;
int g_kernel32 = 1;   // 1: bp_scan32_kernel (32-bit plane words), 0: bp_scan_kernel (64-bit)
int g_xcd_swizzle = 2; // XCD-contiguous block order in bp_scan32_kernel: 0 never, 1 always, 2 for locus-ordered batches
int g_extra_lds = 0;   // bytes of unused dynamic LDS per scan block (occupancy experiments)
int g_stage = 2;       // bp_scan32 LDS staging: 0 never, 1 always, 2 read-order batch over a large genome
int g_twin = 2;        // units_twin: 0 never, 1 always, 2 for batches not flagged locus-ordered
int g_words = 1;       // read-order STAGE scan uses the word-pair layout when the view carries one
int g_persist = 0;      // persistent STAGE kernel: 0 off, -1 occupancy-sized grid, k > 0 k blocks per CU
int g_stage_block = 512; // threads per block of the LDS-staging word-pair scan (FC2_TUNE_STAGE_BLOCK)
int g_tri = 3;           // long-window loads (FC2_TUNE_TRI): 0 two-lane always, 1 three-lane always, 2 three-lane when
                         // windows exceed 97 bases, 3 five-lane 8-B loads when windows exceed 97 bases
#else
constexpr int g_stream_nt = 1, g_kernel32 = 1, g_xcd_swizzle = 2, g_extra_lds = 0, g_stage = 2, g_twin = 2,
              g_words = 1, g_persist = 0, g_stage_block = 512, g_tri = 3;
#endif
inline bool stream_nt() { return g_stream_nt != 0; }
// The staged word-pair scan's window-load form: 0 two-lane, 1 three-lane 16-B, 2 five-lane 8-B (the
// default for 5-pair windows, longer than 97 bases); the per-call hints force any of them.
inline int long_window_form(uint32_t layout, int ml) {
    if (layout & FC2_BATCH_FORM_FIVE) return 2;
    if (layout & FC2_BATCH_FORM_TRI) return 1;
    if (layout & FC2_BATCH_FORM_TWOLANE) return 0;
    if (g_tri == 1) return 1;
    if ((g_tri == 2 || g_tri == 3) && ml + 2 > 97) return g_tri == 3 ? 2 : 1;
    return 0;
}

}  // namespace

// ===========================================================================
// C ABI: launches
// ===========================================================================
namespace {
// fc2_bp_scan_launch / fc2_bp_scan_compact_launch: argument checks and the choice of kernel form.
// sv carries the caller's view (and, for the compact launch, where the epilogue writes); out is the
// 8-byte result array (unused by a compact launch's scan kernels).
int scan_dispatch(const fc2_params *p, const fc2_genome_view *g, const fc2::ScanView &sv, uint64_t *out,
                  uint64_t *tiemask, uint32_t tw, void *stream) {
    const fc2_batch_view *b = &sv;
    if (!b->pairs || !b->read_words || b->stride < b->n || b->rw == 0)
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_launch: bad batch view");
    const bool carried = b->win_words != nullptr;   // window-carrying batch: no genome gather
    if (carried && (g->dummy || !g->chrom_size))
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_launch: window rows need the genome's chromosome sizes");
    if (!carried && !g->dummy && (!g->units || !g->nplane || !g->ncoarse || !g->chrom_start || !g->chrom_size))
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_launch: bad genome view");
    if (p->allhits && (!tiemask || tw < 2))
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_launch: --all-hits needs a tie mask");
    const int ml = b->max_l < 0 ? 0 : b->max_l;
    if (ml > fc2::kMaxFastL) return fc2::fail(FC2_E_RANGE, "fc2_bp_scan_launch: max_l exceeds the register kernel");
    const int nwords = (ml + 2 + 63) / 64;
    if (p->allhits && tw / 2 < (uint32_t)nwords)
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_launch: tie mask too narrow");
    if ((uint64_t)b->rw * 32 < (uint64_t)ml || (b->read_nwords && (uint64_t)b->nw * 64 < (uint64_t)ml))
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_launch: read rows too narrow for max_l");
    hipStream_t s = (hipStream_t)stream;
    const unsigned grid = grid_for(b->n, kBlock);
    const bool nt = stream_nt();
    if (carried) {
        const uint32_t pw = (uint32_t)((ml + 2 + 31) / 32);
        if (ml + 2 > 128) return fc2::fail(FC2_E_RANGE, "fc2_bp_scan_launch: window rows carry l + 2 <= 128 only");
        if (b->ww < 2 * pw || (b->win_nwords && b->wnw < pw) || !b->win_nwords)
            return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_launch: window rows too narrow for max_l");
        fc2::launch_scan32_win((int)pw, nt, s, *p, *g, sv, out, tiemask, tw);
        return hip_check(hipGetLastError(), "bp_scan32_win_kernel launch");
    }
    if ((b->layout & FC2_BATCH_FORM_WAVE) && fc2::wave_ok(ml, *g)) {
        fc2::launch_wave(s, *p, *g, sv, out, tiemask, tw);
        return hip_check(hipGetLastError(), "bp_wave_kernel launch");
    }
    if (g_kernel32) {
        const int sw = g_xcd_swizzle == 2 ? ((b->layout & FC2_BATCH_LOCUS_ORDERED) ? 1 : 0) : g_xcd_swizzle;
        fc2_genome_view gv = *g;
        // locus-ordered batches re-read their lines from L2: the twin only doubles the footprint there
        const bool ordered = (b->layout & FC2_BATCH_LOCUS_ORDERED) != 0;
        if (g_twin == 0 || (g_twin == 2 && ordered)) gv.units_twin = nullptr;
        const bool words = g_words && !(b->layout & FC2_BATCH_FORM_UNITS);
        if (!words || !gv.wt || gv.wt_bytes == 0 || ml + 2 > 128) gv.wt = nullptr;
        // LDS staging pays where every L2 request counts: read-order batch over a genome far larger
        // than the caches (profiles/r01/ab_stage.jsonl); the per-call hints force a form
        const bool big = !g->dummy && g->n_units * 16 >= (64ull << 20);
        const bool stage = (b->layout & FC2_BATCH_FORM_STAGED) ? true
                         : (b->layout & FC2_BATCH_FORM_PLAIN) ? false
                         : g_stage == 2 ? (big && !ordered) : g_stage != 0;
        const int tri = long_window_form(b->layout, ml);
        const int opts = sw ? fc2::kOptSwizzle : 0;
        const int nq = (ml + 2 + 31) / 32;
        if (stage && (g_stage_block != 256 || tri) && g_persist == 0 && fc2::stage_bt_ok(nq, gv)) {
            fc2::launch_scan32_stage_bt(g_stage_block, tri, nt, s, *p, gv, sv, out, tiemask, tw);
            return hip_check(hipGetLastError(), "bp_scan32_stage_bt_kernel launch");
        }
#if FC2_AB_FORMS
        if (stage && g_persist != 0 && fc2::persist_ok(nq, gv)) {
            fc2::launch_scan32_persist(nt, s, *p, gv, sv, out, tiemask, tw, g_persist < 0 ? 0 : g_persist);
            return hip_check(hipGetLastError(), "bp_scan32_persist_kernel launch");
        }
#endif
        fc2::launch_scan32((ml + 2 + 31) / 32, nt, opts, stage, grid, s, *p, gv, sv, out, tiemask, tw,
                           (unsigned)g_extra_lds);
        return hip_check(hipGetLastError(), "bp_scan32_kernel launch");
    }
#if FC2_AB_FORMS
    if (sv.c_words) return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_compact_launch: not with the 64-bit kernel (FC2_TUNE_KERNEL32 0)");
#define FC2_LAUNCH(NWV, NTV) \
    hipLaunchKernelGGL((bp_scan_kernel<NWV, NTV>), dim3(grid), dim3(kBlock), 0, s, *p, *g, *b, out, tiemask, tw)
    if (nwords <= 2) { if (nt) FC2_LAUNCH(2, true); else FC2_LAUNCH(2, false); }
    else if (nwords <= 4) { if (nt) FC2_LAUNCH(4, true); else FC2_LAUNCH(4, false); }
    else { if (nt) FC2_LAUNCH(8, true); else FC2_LAUNCH(8, false); }
#undef FC2_LAUNCH
    return hip_check(hipGetLastError(), "bp_scan_kernel launch");
#else
    (void)grid;
    (void)nwords;
    return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_launch: unreachable form");
#endif
}

__global__ void compact_count_move_kernel(uint32_t *count, uint32_t *out) {
    *out = *count;
    *count = 0u;
}

}  // namespace

extern "C" int fc2_bp_scan_launch(const fc2_params *p, const fc2_genome_view *g, const fc2_batch_view *b,
                                  fc2_result *results, uint64_t *tiemask, uint32_t tw, void *stream) {
    int rc = fc2::validate_params(p);
    if (rc) return rc;
    if (!g || !b || !results) return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_launch: null argument");
    if (b->n == 0) return FC2_OK;
    return scan_dispatch(p, g, fc2::ScanView(*b), reinterpret_cast<uint64_t *>(results), tiemask, tw, stream);
}

extern "C" int fc2_bp_scan_compact_launch(const fc2_params *p, const fc2_genome_view *g, const fc2_batch_view *b,
                                          const fc2_compact_out *co, void *stream) {
    int rc = fc2::validate_params(p);
    if (rc) return rc;
    if (!g || !b || !co) return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_compact_launch: null argument");
    if (p->noncanonical || p->allhits)
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_compact_launch: canonical mode without --all-hits only");
    if (co->width != 2 && co->width != 4) return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_compact_launch: width is 2 or 4");
    if (!co->esc_count || (b->n && !co->words) || (co->esc_cap && !co->esc))
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_compact_launch: bad output");
    if (b->n) {
        fc2::ScanView sv(*b);
        sv.c_words = co->words;
        sv.c_esc = co->esc;
        sv.c_count = co->esc_count;
        sv.c_cap = co->esc_cap;
        sv.c_width = co->width;
        rc = scan_dispatch(p, g, sv, nullptr, nullptr, 0, stream);
        if (rc) return rc;
    }
    if (co->count_out) {
        hipLaunchKernelGGL(compact_count_move_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, co->esc_count,
                           co->count_out);
        return hip_check(hipGetLastError(), "compact_count_move_kernel launch");
    }
    return FC2_OK;
}

extern "C" int fc2_gather_windows_launch(const fc2_params *p, const fc2_genome_view *g, const fc2_batch_view *b,
                                         fc2_pair *pairs, uint64_t *win_words, uint64_t *win_nwords, uint32_t pw,
                                         void *stream) {
    int rc = fc2::validate_params(p);
    if (rc) return rc;
    if (!g || !b || !pairs || !win_words || !win_nwords || g->dummy || !g->wt || !g->chrom_start || !g->chrom_size)
        return fc2::fail(FC2_E_PARAM, "fc2_gather_windows_launch: needs a genome with a word-pair table");
    if (pw < 1 || pw > 4) return fc2::fail(FC2_E_RANGE, "fc2_gather_windows_launch: pw is 1..4");
    if (b->n == 0) return FC2_OK;
    if (b->stride < b->n) return fc2::fail(FC2_E_PARAM, "fc2_gather_windows_launch: stride < n");
    fc2::launch_gather_windows((hipStream_t)stream, *p, *g, b->n, b->stride, pairs, win_words, win_nwords, pw);
    return hip_check(hipGetLastError(), "gather_windows_kernel launch");
}

extern "C" int fc2_probe_pattern_launch(const fc2_params *p, const fc2_genome_view *g, const fc2_batch_view *b,
                                        uint64_t *out, void *stream) {
    int rc = fc2::validate_params(p);
    if (rc) return rc;
    if (!g || !b || !out || g->dummy || !g->wt || !g->chrom_start || !b->pairs || !b->read_words)
        return fc2::fail(FC2_E_PARAM, "fc2_probe_pattern_launch: needs a genome with a word-pair table and a batch");
    if (b->n == 0) return FC2_OK;
    const int ml = b->max_l < 0 ? 0 : b->max_l;
    if (fc2::launch_probe_pattern((hipStream_t)stream, *p, *g, *b, out, long_window_form(b->layout, ml)))
        return fc2::fail(FC2_E_HIP, "probe_pattern_kernel launch failed");
    return FC2_OK;
}

extern "C" int fc2_bp_scan_bytes_launch(const fc2_params *p, const fc2_bytes_view *v, fc2_result *results,
                                        uint64_t *tiemask, uint32_t tw, uint64_t stride, void *stream) {
    int rc = fc2::validate_params(p);
    if (rc) return rc;
    if (!v || !results) return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_bytes_launch: null argument");
    if (v->m == 0) return FC2_OK;
    if (!v->index || !v->pairs || !v->arena || !v->off)
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_bytes_launch: bad view");
    if (p->allhits && (!tiemask || tw < 2))
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_bytes_launch: --all-hits needs a tie mask");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(bp_bytes_kernel, dim3(grid_for(v->m, kBlock)), dim3(kBlock), 0, s, *p, *v,
                       reinterpret_cast<uint64_t *>(results), tiemask, tw, stride);
    return hip_check(hipGetLastError(), "bp_bytes_kernel launch");
}

extern "C" int fc2_bp_scan_long_launch(const fc2_params *p, uint64_t n, const fc2_long_pair *pairs, const uint64_t *off,
                                       const uint8_t *arena, const uint64_t *tie_off, fc2_long_result *results,
                                       uint64_t *ties, void *stream) {
    int rc = fc2::validate_params(p);
    if (rc) return rc;
    if (n == 0) return FC2_OK;
    if (!pairs || !off || !arena || !results) return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_long_launch: null argument");
    if (p->allhits && (!ties || !tie_off))
        return fc2::fail(FC2_E_PARAM, "fc2_bp_scan_long_launch: --all-hits needs the tie words and their offsets");
    hipLaunchKernelGGL(bp_long_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, (hipStream_t)stream, *p, n, pairs,
                       off, arena, tie_off, results, ties);
    return hip_check(hipGetLastError(), "bp_long_kernel launch");
}

extern "C" int fc2_synth_genome_launch(uint64_t seed, uint64_t *units, uint64_t *nplane, uint32_t *ncoarse,
                                       uint64_t n_units, const int64_t *n_lo, const int64_t *n_hi,
                                       uint32_t n_intervals, void *stream) {
    if (!units || !nplane || !ncoarse || n_units == 0) return fc2::fail(FC2_E_PARAM, "fc2_synth_genome_launch: bad args");
    if (n_intervals && (!n_lo || !n_hi)) return fc2::fail(FC2_E_PARAM, "fc2_synth_genome_launch: intervals");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(synth_genome_kernel, dim3(grid_for(n_units, 256)), dim3(256), 0, s, seed, units, nplane,
                       n_units, n_lo, n_hi, n_intervals);
    int rc = hip_check(hipGetLastError(), "synth_genome_kernel launch");
    if (rc) return rc;
    return fc2_coarse_launch(nplane, ncoarse, n_units, stream);
}

extern "C" int fc2_twin_launch(const uint64_t *units, uint64_t n_units, uint64_t *units_twin, void *stream) {
    if (!units || !units_twin || n_units == 0) return fc2::fail(FC2_E_PARAM, "fc2_twin_launch: bad args");
    const uint64_t n_words = 2 * (n_units + 8);
    hipLaunchKernelGGL(twin_kernel, dim3(grid_for(n_words, 256)), dim3(256), 0, (hipStream_t)stream, units, n_units,
                       units_twin);
    return hip_check(hipGetLastError(), "twin_kernel launch");
}

extern "C" int fc2_wtab_geometry(uint64_t n_units, uint64_t *bytes, uint64_t *twin_off) {
    if (!bytes || !twin_off) return fc2::fail(FC2_E_PARAM, "fc2_wtab_geometry: null argument");
    const uint64_t n_q = 2 * n_units;
    const uint64_t main_bytes = ((n_q + 32) * 8 + 127) / 128 * 128;
    const uint64_t total = main_bytes + ((n_q + 24) * 8 + 127) / 128 * 128;
    if (total > 0xFFFFFF00ull) return fc2::fail(FC2_E_RANGE, "fc2_wtab_geometry: genome too large for 32-bit offsets");
    *bytes = total;
    *twin_off = main_bytes;
    return FC2_OK;
}

extern "C" int fc2_wtab_launch(const uint64_t *units, uint64_t n_units, uint32_t *wt, void *stream) {
    if (!units || !wt || n_units == 0) return fc2::fail(FC2_E_PARAM, "fc2_wtab_launch: bad args");
    uint64_t bytes = 0, twin_off = 0;
    const int rc = fc2_wtab_geometry(n_units, &bytes, &twin_off);
    if (rc) return rc;
    hipLaunchKernelGGL(wtab_kernel, dim3(grid_for(bytes / 8, 256)), dim3(256), 0, (hipStream_t)stream, units, n_units,
                       reinterpret_cast<uint64_t *>(wt), twin_off / 8, bytes / 8);
    return hip_check(hipGetLastError(), "wtab_kernel launch");
}

extern "C" int fc2_nsuper_geometry(uint64_t n_units, uint32_t *shift, uint32_t *words) {
    if (!shift || !words) return fc2::fail(FC2_E_PARAM, "fc2_nsuper_geometry: null argument");
    const uint64_t bases = (n_units ? n_units : 1) * 64;
    uint32_t s = 10;                               // >= one coarse block (1024 bases)
    while (((bases + (1ull << s) - 1) >> s) > 2048ull * 32) ++s;
    *shift = s;
    *words = (uint32_t)((((bases + (1ull << s) - 1) >> s) + 31) >> 5);
    return FC2_OK;
}

extern "C" int fc2_nsuper_launch(const uint32_t *ncoarse, uint64_t n_units, uint32_t *nsuper, void *stream) {
    if (!ncoarse || !nsuper || n_units == 0) return fc2::fail(FC2_E_PARAM, "fc2_nsuper_launch: bad args");
    uint32_t shift, words;
    fc2_nsuper_geometry(n_units, &shift, &words);
    hipLaunchKernelGGL(nsuper_kernel, dim3(grid_for(words, 256)), dim3(256), 0, (hipStream_t)stream, ncoarse, n_units,
                       shift, words, nsuper);
    return hip_check(hipGetLastError(), "nsuper_kernel launch");
}

extern "C" int fc2_coarse_launch(const uint64_t *nplane, uint32_t *ncoarse, uint64_t n_units, void *stream) {
    if (!nplane || !ncoarse) return fc2::fail(FC2_E_PARAM, "fc2_coarse_launch: bad args");
    const uint64_t n_words = (((n_units + 15) >> 4) + 31) >> 5;
    hipLaunchKernelGGL(coarse_kernel, dim3(grid_for(n_words, 256)), dim3(256), 0, (hipStream_t)stream, nplane, ncoarse,
                       n_units);
    return hip_check(hipGetLastError(), "coarse_kernel launch");
}

extern "C" int fc2_synth_pairs_launch(const fc2_params *p, const fc2_synth_cfg *cfg, const fc2_genome_view *g,
                                      const int64_t *chrom_cum, uint64_t n, fc2_pair *pairs, uint64_t *read_words,
                                      uint32_t rw, uint64_t *read_nwords, uint32_t nw, uint64_t stride, int32_t *truth,
                                      void *stream) {
    int rc = fc2::validate_params(p);
    if (rc) return rc;
    if (!cfg || !g || !chrom_cum || !pairs || !read_words || stride < n)
        return fc2::fail(FC2_E_PARAM, "fc2_synth_pairs_launch: bad args");
    if (cfg->len_min < 2 * p->asize || cfg->len_max < cfg->len_min || cfg->len_max > 65535)
        return fc2::fail(FC2_E_PARAM, "fc2_synth_pairs_launch: read length range");
    const int lmax = cfg->len_max - 2 * fc2::eff_anchor(p);
    if ((int64_t)rw * 32 < lmax || (read_nwords && (int64_t)nw * 64 < lmax))
        return fc2::fail(FC2_E_PARAM, "fc2_synth_pairs_launch: rows too narrow");
    if (n == 0) return FC2_OK;
    hipLaunchKernelGGL(synth_pairs_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, *p, *cfg, *g,
                       chrom_cum, n, pairs, read_words, rw, read_nwords, nw, stride, truth);
    return hip_check(hipGetLastError(), "synth_pairs_kernel launch");
}

// compact results (include/fc2_bp.h): 8 B in, 4 or 2 B out per pair, streamed; escapes are rare
template <int WIDTH>
__global__ void __launch_bounds__(256) result_compact_kernel(const uint64_t *__restrict__ res, uint64_t n,
                                                             void *__restrict__ words, fc2_result_escape *esc,
                                                             uint32_t cap, uint32_t *count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t w = __builtin_nontemporal_load(res + i);
    bool escape;
    const uint32_t c = fc2::compact_pack(w, WIDTH, escape);
    if (escape) {
        const uint32_t k = atomicAdd(count, 1u);
        if (k < cap) {
            esc[k].index = i;
            memcpy(&esc[k].result, &w, sizeof w);
        }
    }
    if constexpr (WIDTH == 2) __builtin_nontemporal_store((uint16_t)c, (uint16_t *)words + i);
    else __builtin_nontemporal_store(c, (uint32_t *)words + i);
}

extern "C" int fc2_result_compact_launch(const fc2_params *p, const fc2_result *results, uint64_t n, int width,
                                         void *words, fc2_result_escape *esc, uint32_t esc_cap, uint32_t *esc_count,
                                         void *stream) {
    int rc = fc2::validate_params(p);
    if (rc) return rc;
    if (p->noncanonical)
        return fc2::fail(FC2_E_PARAM, "fc2_result_compact_launch: the compact forms hold canonical-mode results only");
    if (width != 2 && width != 4) return fc2::fail(FC2_E_PARAM, "fc2_result_compact_launch: width is 2 or 4");
    if (!esc_count || (n && (!results || !words)) || (esc_cap && !esc))
        return fc2::fail(FC2_E_PARAM, "fc2_result_compact_launch: bad args");
    hipError_t e = hipMemsetAsync(esc_count, 0, sizeof(uint32_t), (hipStream_t)stream);
    if (e != hipSuccess) return hip_check(e, "result_compact count reset");
    if (n == 0) return FC2_OK;
    if (width == 2)
        hipLaunchKernelGGL(result_compact_kernel<2>, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                           (const uint64_t *)results, n, words, esc, esc_cap, esc_count);
    else
        hipLaunchKernelGGL(result_compact_kernel<4>, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                           (const uint64_t *)results, n, words, esc, esc_cap, esc_count);
    return hip_check(hipGetLastError(), "result_compact_kernel launch");
}

extern "C" int fc2_set_tuning(int key, int value) {
#if FC2_AB_FORMS
    switch (key) {
        case FC2_TUNE_STREAM_NT: g_stream_nt = value ? 1 : 0; return FC2_OK;
        case FC2_TUNE_KERNEL32: g_kernel32 = value ? 1 : 0; return FC2_OK;
        case FC2_TUNE_REORDER_ROUNDS:
            if (value < 1 || value > 32) return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: reorder rounds 1..32");
            fc2::g_reorder_rounds = value; return FC2_OK;
        case FC2_TUNE_REORDER_NT: fc2::g_reorder_nt = value ? 1 : 0; return FC2_OK;
        case FC2_TUNE_EXTRA_LDS:
            if (value < 0 || value > 65536) return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: extra LDS 0..65536");
            g_extra_lds = value; return FC2_OK;
        case FC2_TUNE_STAGE:
            if (value < 0 || value > 2) return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: stage is 0, 1 or 2");
            g_stage = value; return FC2_OK;
        case FC2_TUNE_TWIN:
            if (value < 0 || value > 2) return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: twin is 0, 1 or 2");
            g_twin = value; return FC2_OK;
        case FC2_TUNE_WORDS: g_words = value ? 1 : 0; return FC2_OK;
        case FC2_TUNE_TRI:
            if (value < 0 || value > 3) return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: tri is 0, 1, 2 or 3");
            g_tri = value; return FC2_OK;
        case FC2_TUNE_STAGE_BLOCK:
            if (value != 256 && value != 512 && value != 1024)
                return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: stage block is 256, 512 or 1024");
            g_stage_block = value; return FC2_OK;
        case FC2_TUNE_REORDER_SHIFT:
            if (value != 0 && (value < 16 || value > 40))
                return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: reorder shift is 0 or 16..40");
            fc2::g_reorder_shift = value; return FC2_OK;
        case FC2_TUNE_PERSIST:
            if (value < -1 || value > 32) return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: persist is -1..32");
            g_persist = value; return FC2_OK;
        case FC2_TUNE_XCD_SWIZZLE:
            if (value < 0 || value > 2) return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: swizzle is 0, 1 or 2");
            g_xcd_swizzle = value; return FC2_OK;
        default: return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: unknown key");
    }
#else
    (void)key;
    (void)value;
    return fc2::fail(FC2_E_PARAM, "fc2_set_tuning: tuning knobs exist only in A/B builds of the library "
                                  "(FC2_AB_FORMS=1, make -C find_circ2_amd/csrc ab); use the FC2_BATCH_FORM_* hints");
#endif
}

extern "C" int fc2_get_tuning(int key, int *value) {
    if (!value) return fc2::fail(FC2_E_PARAM, "fc2_get_tuning: null value");
    switch (key) {
        case FC2_TUNE_STREAM_NT: *value = g_stream_nt; return FC2_OK;
        case FC2_TUNE_KERNEL32: *value = g_kernel32; return FC2_OK;
        case FC2_TUNE_XCD_SWIZZLE: *value = g_xcd_swizzle; return FC2_OK;
        case FC2_TUNE_REORDER_ROUNDS: *value = fc2::g_reorder_rounds; return FC2_OK;
        case FC2_TUNE_REORDER_NT: *value = fc2::g_reorder_nt; return FC2_OK;
        case FC2_TUNE_TWIN: *value = g_twin; return FC2_OK;
        case FC2_TUNE_STAGE: *value = g_stage; return FC2_OK;
        case FC2_TUNE_EXTRA_LDS: *value = g_extra_lds; return FC2_OK;
        case FC2_TUNE_PERSIST: *value = g_persist; return FC2_OK;
        case FC2_TUNE_WORDS: *value = g_words; return FC2_OK;
        case FC2_TUNE_STAGE_BLOCK: *value = g_stage_block; return FC2_OK;
        case FC2_TUNE_TRI: *value = g_tri; return FC2_OK;
        case FC2_TUNE_REORDER_SHIFT: *value = fc2::g_reorder_shift; return FC2_OK;
        default: return fc2::fail(FC2_E_PARAM, "fc2_get_tuning: unknown key");
    }
}

extern "C" int fc2_device_count(int *count) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (count) *count = (e == hipSuccess) ? c : 0;
    return FC2_OK;
}

extern "C" int fc2_host_register(void *ptr, uint64_t bytes) {
    if (!ptr || !bytes) return fc2::fail(FC2_E_PARAM, "fc2_host_register: empty range");
    const hipError_t e = hipHostRegister(ptr, (size_t)bytes, hipHostRegisterPortable | hipHostRegisterMapped);
    if (e != hipSuccess) return fc2::fail(FC2_E_HIP, std::string("hipHostRegister: ") + hipGetErrorString(e));
    return FC2_OK;
}

extern "C" int fc2_host_device_pointer(void *host, void **dev) {
    if (!host || !dev) return fc2::fail(FC2_E_PARAM, "fc2_host_device_pointer: null argument");
    const hipError_t e = hipHostGetDevicePointer(dev, host, 0);
    if (e != hipSuccess) return fc2::fail(FC2_E_HIP, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
    return FC2_OK;
}

extern "C" int fc2_host_unregister(void *ptr) {
    if (!ptr) return fc2::fail(FC2_E_PARAM, "fc2_host_unregister: null pointer");
    const hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) return fc2::fail(FC2_E_HIP, std::string("hipHostUnregister: ") + hipGetErrorString(e));
    return FC2_OK;
}
