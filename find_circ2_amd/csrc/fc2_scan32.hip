// fc2_scan32.hip -- the breakpoint-search kernel on 32-bit bit-plane words.
//
// Same algorithm and results as bp_scan_kernel (fc2_kernels.hip; reference
// find_circ.py:854-974), re-cut for the gfx950 VALU: every plane is held as
// 32-bit words so that each funnel shift (window alignment, B[x+2], the
// dinucleotide shift) is ONE v_alignbit_b32 and each popcount ONE v_bcnt_u32,
// instead of the 64-bit shift/or/select sequences.  NQ = 32-bit words per
// plane: 4 / 8 / 16 <-> l + 2 <= 128 / 256 / 512.
//
// Kernel forms (fc2_bp_scan_launch picks one per batch; every form gives identical results,
// tests/test_gpu_kernel_forms.py):
//   bp_scan32_stage_bt_kernel<BT, NT, TRI>  read-order batch, genome >= 64 MiB, l + 2 <= 128: LDS
//        tables, cooperative word-pair window loads (two lanes per window, or three for windows
//        longer than 97 bases); the headline form
//   bp_scan32_kernel<NQ, NT, STAGE>          the same with 256-pair blocks (STAGE), the unit-plane
//        cooperative loads (no word-pair table), and the plain form for locus-ordered or
//        cache-resident batches (STAGE = false)
//   bp_scan32_win_kernel<PW, NT>             window-carrying batches: windows streamed with the record
//   bp_scan32_persist_kernel<NT>             persistent-grid experiment (FC2_TUNE_PERSIST, off)
//   probe_pattern_kernel                     measurement: the headline form's memory traffic only
//   gather_windows_kernel<PW>                builds window rows from the resident genome
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fc2_common.h"
#include "fc2_compact.h"
#include "fc2_scan32.h"

namespace {

// Measurement-only ablations (scripts/ablate_build.sh; WRONG results, never in the shipped library):
// bit 0 skips the owner's third-unit loads, bit 1 skips N-plane loads of flagged windows, bit 2
// skips the canonical candidate walk, bit 3 skips the fifth word pair of windows with W > 97, bit 4
// skips the read N-row loads.
#ifndef FC2_ABLATE
#define FC2_ABLATE 0
#endif

constexpr int kBlock = 256;
constexpr int kChromLds = 512;   // chromosome-table entries a block stages in LDS (8 KB)
constexpr int kSuperLds = 2048;  // nsuper words a block stages in LDS (8 KB)

__device__ __forceinline__ uint32_t lowbits32(int n) {  // bits [0, n), any n
    return n >= 32 ? ~0u : (n <= 0 ? 0u : ((1u << n) - 1u));
}
// bits [s, s+32) of the 64-bit value hi:lo, s in [0, 31]
__device__ __forceinline__ uint32_t alignr(uint32_t hi, uint32_t lo, unsigned s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}
__device__ __forceinline__ uint32_t rmask32(int a, int b, int k) {  // positions [a, b) in word k
    return lowbits32(b - 32 * k) & ~lowbits32(a - 32 * k);
}

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
// A pair's result: the 8-byte word to out[i], or (fc2_bp_scan_compact_launch) its compact word to
// bv.c_words[i] with an escape through the device counter when it does not fit (fc2_compact.h)
template <bool NT>
__device__ __forceinline__ void emit(const fc2::ScanView &bv, uint64_t *out, uint64_t i, uint64_t w) {
    if (bv.c_words) {
        bool esc;
        const uint32_t c = fc2::compact_pack(w, bv.c_width, esc);
        if (esc) {
            const uint32_t k = atomicAdd(bv.c_count, 1u);
            if (k < bv.c_cap) {
                bv.c_esc[k].index = i;
                __builtin_memcpy(&bv.c_esc[k].result, &w, sizeof w);
            }
        }
        if (bv.c_width == 2) __builtin_nontemporal_store((uint16_t)c, (uint16_t *)bv.c_words + i);
        else __builtin_nontemporal_store(c, (uint32_t *)bv.c_words + i);
    } else {
        st_stream<NT>(out + i, w);
    }
}

// A byte-path pair in a compact launch: the escape word without an escape record, so that
// fc2_result_expand fails (FC2_E_FORMAT: more escaped words than escapes) instead of decoding
// whatever the word held before -- the compact launch takes no byte-path pairs (fc2_bp.h).
__device__ __forceinline__ void mark_unscanned(const fc2::ScanView &bv, uint64_t i) {
    if (bv.c_width == 2) __builtin_nontemporal_store((uint16_t)FC2_R16_ESCAPE, (uint16_t *)bv.c_words + i);
    else __builtin_nontemporal_store((uint32_t)FC2_R32_ESCAPE, (uint32_t *)bv.c_words + i);
}

template <bool NT>
__device__ __forceinline__ u64x2 ld_pair_raw(const fc2_pair *p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
    else return *reinterpret_cast<const u64x2 *>(p);
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

template <int NQ>
struct P32 {
    uint32_t lo[NQ + 1], hi[NQ + 1], n[NQ + 1];
};

// shift the word array left by `sel` words (sel in [0, 2^levels)), selects only
template <int M>
__device__ __forceinline__ void word_shift(uint32_t (&a)[M], int sel, int levels) {
#pragma unroll
    for (int lv = 0; lv < 5; ++lv) {
        if (lv >= levels) break;
        const int d = 1 << lv;
        const bool on = (sel >> lv) & 1;
#pragma unroll
        for (int k = 0; k < M; ++k) a[k] = on ? (k + d < M ? a[k + d] : 0u) : a[k];
    }
}

// Genome window [ws, ws+W) of a chromosome starting at global base cstart, in two
// phases so that a lane's loads for BOTH windows (units + coarse N words) are in
// flight together: window_issue only issues loads (straight-line, clamped
// addresses, no branches), window_finish consumes them.  Only the N plane of a
// window whose 1024-base blocks contain an N costs a further round trip.
template <int NQ>
struct WinRaw {
    static constexpr int NU = NQ / 2 + 1;    // 64-bit units covering NQ+1 32-bit words at any parity
    ulonglong2 v[NU];                        // code planes (lo, hi) of units u0 .. u0+jl
    uint64_t nv[NU];                         // N plane of the same units (super-map path, flagged windows)
    uint64_t cw;                             // coarse path: N bits of 1024-base blocks [32*w, 32*w + 64),
                                             // w = coarse_word(u0) (recomputed, not carried)
    int64_t u0;
    unsigned sh;
    int odd, jl;                             // word parity; last needed unit (relative to u0)
};

// Does any base of [g0, g0 + W) (clipped to the genome) lie in a super block holding an N?
__device__ __forceinline__ bool super_flag(const uint32_t *s_nsuper, uint32_t shift, int64_t g0, int W,
                                           uint64_t n_units) {
    int64_t lo = g0, hi = g0 + W - 1;
    const int64_t top = (int64_t)(n_units * 64) - 1;
    lo = lo < 0 ? 0 : lo;
    hi = hi > top ? top : hi;
    if (lo > hi) return false;
    const uint64_t k0 = (uint64_t)lo >> shift, k1 = (uint64_t)hi >> shift;   // k1 <= k0 + 1 (W <= 2^shift)
    return ((s_nsuper[k0 >> 5] >> (k0 & 31)) & 1u) || ((s_nsuper[k1 >> 5] >> (k1 & 31)) & 1u);
}

// First of the two coarse-map words loaded for a window whose first unit is u0.
__device__ __forceinline__ int64_t coarse_word(const fc2_genome_view &g, int64_t u0) {
    const int64_t nb = (int64_t)((g.n_units + 15) >> 4);
    const int64_t nw = (nb + 31) >> 5;
    int64_t b0 = u0 >> 4;
    b0 = b0 < 0 ? 0 : (b0 >= nb ? nb - 1 : b0);
    const int64_t w = b0 >> 5;
    return nw >= 2 ? (w > nw - 2 ? nw - 2 : w) : 0;
}

// s_nsuper: the LDS copy of g.nsuper, or nullptr (then the coarse map decides in window_finish,
// one round trip later).
template <int NQ>
__device__ __forceinline__ void window_issue(const fc2_genome_view &g, const uint32_t *s_nsuper, uint64_t cstart,
                                             int64_t ws, int W, WinRaw<NQ> &R) {
    constexpr int NU = WinRaw<NQ>::NU;
    const int64_t g0 = (int64_t)cstart + ws;
    const int64_t q0 = g0 >> 5;              // first 32-bit word (floor)
    R.sh = (unsigned)(g0 & 31);
    R.u0 = q0 >> 1;
    R.odd = (int)(q0 & 1);
    const int qlast = R.odd + (((int)R.sh + W - 1) >> 5);   // last word needed, relative to 2*u0
    R.jl = qlast >> 1;
    // A window straddling a 128-B line (8 units) of `units` sits inside one line of the twin
    // copy (shifted by 4 units): one line fill per window instead of two.
    const bool straddle = (int)(R.u0 & 7) + R.jl >= 8;
    const ulonglong2 *U = (straddle && g.units_twin) ? reinterpret_cast<const ulonglong2 *>(g.units_twin) + 4
                                                     : reinterpret_cast<const ulonglong2 *>(g.units);
    const int64_t last = (int64_t)g.n_units - 1;
    const bool nflag = s_nsuper && super_flag(s_nsuper, g.nsuper_shift, g0, W, g.n_units);
#pragma unroll
    for (int j = 0; j < NU; ++j) {
        const int64_t u = R.u0 + j;
        const int64_t uc = u < 0 ? 0 : (u > last ? last : u);
        // every request is an L2 transaction even when it hits (profiles/r01: ~0.29 ms per extra
        // request per pair at 50M pairs), so units past the window are not loaded at all
        R.v[j] = ulonglong2{0ull, 0ull};
        R.nv[j] = 0;
        if (j < 2 || j <= R.jl) R.v[j] = U[uc];
        if (nflag && j <= R.jl) R.nv[j] = g.nplane[uc];
    }
    R.cw = 0;
    if (!s_nsuper) {
        // coarse N bits of the window's first and last 1024-base block (b1 <= b0 + 1) with ONE
        // dword-aligned 8-byte load covering words w, w+1; consumed only in window_finish
        const int64_t w = coarse_word(g, R.u0);
        if ((((g.n_units + 15) >> 4) + 31) >> 5 >= 2)
            R.cw = *reinterpret_cast<const uint64_t *>(g.ncoarse + w);   // 4-B aligned: a dwordx2 needs no more
        else
            R.cw = g.ncoarse[0];
    }
}

// ---------------------------------------------------------------------------------------------
// Cooperative unit loads (read-order batches, NQ == 4).  Every 16-B load instruction is one L2
// request per distinct line it touches, and a lane's two unit loads of one window sit in two
// instructions: two requests for one line.  Here lanes 2m and 2m+1 load units 0 and 1 of the
// window of pair 32c + m in instruction c, so one request serves both (profiles/r01:
// pattern_probe paired vs unpaired); the units travel back to their owner lane through LDS.
// The owner still loads a window's rare third unit and its N-plane units itself.
// Packed window for the loading lanes: (u0 + 8) in bits 0..30, bit 31 = read the twin.
template <int NQ>
__device__ __forceinline__ uint32_t window_geom(const fc2_genome_view &g, uint64_t cstart, int64_t ws, int W,
                                                WinRaw<NQ> &R) {
    const int64_t g0 = (int64_t)cstart + ws;
    const int64_t q0 = g0 >> 5;
    R.sh = (unsigned)(g0 & 31);
    R.u0 = q0 >> 1;
    R.odd = (int)(q0 & 1);
    R.jl = (R.odd + (((int)R.sh + W - 1) >> 5)) >> 1;
    const bool twin = g.units_twin && (int)(R.u0 & 7) + R.jl >= 8;
    return (uint32_t)(R.u0 + 8) | ((uint32_t)twin << 31);
}

__device__ __forceinline__ const ulonglong2 *unit_base(const fc2_genome_view &g, uint32_t packed) {
    return (packed >> 31) ? reinterpret_cast<const ulonglong2 *>(g.units_twin) + 4
                          : reinterpret_cast<const ulonglong2 *>(g.units);
}

__device__ __forceinline__ ulonglong2 unit_load(const fc2_genome_view &g, uint32_t packed, int j) {
    const int64_t last = (int64_t)g.n_units - 1;
    int64_t u = (int64_t)(packed & 0x7FFFFFFFu) - 8 + j;
    u = u < 0 ? 0 : (u > last ? last : u);   // out-of-genome positions are masked to 'N' in window_finish
    return unit_base(g, packed)[u];
}

// Issue phase for BOTH windows of the lane's pair; all 64 lanes must execute it (inactive lanes
// pass a harmless geometry).  cl[X][c]: the unit this lane loaded for window X in instruction c.
template <int NQ>
__device__ __forceinline__ void windows_issue_coop(const fc2_genome_view &g, const uint32_t *s_nsuper,
                                                   uint64_t cstart, int64_t wsA, int64_t wsB, int W, bool active,
                                                   WinRaw<NQ> &rA, WinRaw<NQ> &rB, ulonglong2 (&cl)[2][2]) {
    constexpr int NU = WinRaw<NQ>::NU;
    static_assert(NU == 3, "cooperative loads cover units 0 and 1; the owner loads unit 2");
    const uint32_t pk[2] = {window_geom<NQ>(g, cstart, wsA, W, rA), window_geom<NQ>(g, cstart, wsB, W, rB)};
    const int lane = (int)(threadIdx.x & 63);
    const int64_t wsx[2] = {wsA, wsB};
    // All LDS traffic of the issue phase in ONE batch ahead of the first global load: the four
    // geometry permutes and both windows' two super-map words (read unconditionally, so no
    // short-circuit branch waits on a first LDS read before issuing the second).
    uint32_t src[2][2], sw[2][2] = {{0u, 0u}, {0u, 0u}};
    uint32_t sb[2][2] = {{0u, 0u}, {0u, 0u}};
    bool sv[2] = {false, false};
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int c = 0; c < 2; ++c)
            src[x][c] = (uint32_t)__builtin_amdgcn_ds_bpermute((32 * c + (lane >> 1)) << 2, (int)pk[x]);
    if (!(FC2_ABLATE & 2) && s_nsuper) {
        const int64_t top = (int64_t)(g.n_units * 64) - 1;
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            int64_t lo = (int64_t)cstart + wsx[x], hi = lo + W - 1;
            lo = lo < 0 ? 0 : lo;
            hi = hi > top ? top : hi;
            sv[x] = active && lo <= hi;
            const uint64_t k0 = sv[x] ? (uint64_t)lo >> g.nsuper_shift : 0,
                           k1 = sv[x] ? (uint64_t)hi >> g.nsuper_shift : 0;   // k1 <= k0 + 1
            sw[x][0] = s_nsuper[k0 >> 5];
            sw[x][1] = s_nsuper[k1 >> 5];
            sb[x][0] = (uint32_t)(k0 & 31);
            sb[x][1] = (uint32_t)(k1 & 31);
        }
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int c = 0; c < 2; ++c) cl[x][c] = unit_load(g, src[x][c], lane & 1);
    WinRaw<NQ> *R[2] = {&rA, &rB};
#pragma unroll
    for (int x = 0; x < 2; ++x) {
        WinRaw<NQ> &Q = *R[x];
        Q.v[0] = Q.v[1] = Q.v[2] = ulonglong2{0ull, 0ull};
        if (!(FC2_ABLATE & 1) && active && Q.jl >= 2) Q.v[2] = unit_load(g, pk[x], 2);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x) {
        WinRaw<NQ> &Q = *R[x];
        const bool nflag = sv[x] && (((sw[x][0] >> sb[x][0]) | (sw[x][1] >> sb[x][1])) & 1u);
        const int64_t last = (int64_t)g.n_units - 1;
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            const int64_t u = Q.u0 + j;
            Q.nv[j] = 0;
            if (nflag && j <= Q.jl) Q.nv[j] = g.nplane[u < 0 ? 0 : (u > last ? last : u)];
        }
        Q.cw = 0;
        if (!s_nsuper && active) {
            const int64_t w = coarse_word(g, Q.u0);
            if ((((g.n_units + 15) >> 4) + 31) >> 5 >= 2)
                Q.cw = *reinterpret_cast<const uint64_t *>(g.ncoarse + w);
            else
                Q.cw = g.ncoarse[0];
        }
    }
}

// Exchange: every lane parks what it loaded in its wave's LDS slots, then takes its own units.
template <int NQ>
__device__ __forceinline__ void windows_exchange_coop(ulonglong2 *xchg, const ulonglong2 (&cl)[2][2],
                                                      WinRaw<NQ> &rA, WinRaw<NQ> &rB) {
    const int lane = (int)(threadIdx.x & 63);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int c = 0; c < 2; ++c) xchg[(2 * x + c) * 64 + lane] = cl[x][c];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int c = lane >> 5, m = lane & 31;
    rA.v[0] = xchg[(0 + c) * 64 + 2 * m];
    rA.v[1] = xchg[(0 + c) * 64 + 2 * m + 1];
    rB.v[0] = xchg[(2 + c) * 64 + 2 * m];
    rB.v[1] = xchg[(2 + c) * 64 + 2 * m + 1];
}

template <int NQ>
__device__ __forceinline__ void window_finish(const fc2_genome_view &g, const uint32_t *s_nsuper, const WinRaw<NQ> &R,
                                              int64_t csize, int64_t ws, int W, P32<NQ> &P) {
    constexpr int NU = WinRaw<NQ>::NU;
    uint32_t xl[2 * NU], xh[2 * NU], xn[2 * NU];
#pragma unroll
    for (int j = 0; j < NU; ++j) {
        // units outside the genome were loaded from a clamped index: their positions lie outside
        // the chromosome, which the [vlo, vhi) mask below turns into 'N' whatever was loaded
        const ulonglong2 v = R.v[j];
        const uint64_t n = R.nv[j];
        xl[2 * j] = (uint32_t)v.x; xl[2 * j + 1] = (uint32_t)(v.x >> 32);
        xh[2 * j] = (uint32_t)v.y; xh[2 * j + 1] = (uint32_t)(v.y >> 32);
        xn[2 * j] = (uint32_t)n; xn[2 * j + 1] = (uint32_t)(n >> 32);
    }
    const int odd = R.odd;
    const unsigned sh = R.sh;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        const uint32_t l0 = odd ? xl[k + 1] : xl[k], l1 = odd ? xl[k + 2] : xl[k + 1];
        const uint32_t h0 = odd ? xh[k + 1] : xh[k], h1 = odd ? xh[k + 2] : xh[k + 1];
        P.lo[k] = alignr(l1, l0, sh);
        P.hi[k] = alignr(h1, h0, sh);
    }
    P.lo[NQ] = 0; P.hi[NQ] = 0;

    if (s_nsuper) {                          // N plane already loaded for flagged windows (else zero)
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const uint32_t n0 = odd ? xn[k + 1] : xn[k], n1 = odd ? xn[k + 2] : xn[k + 1];
            P.n[k] = alignr(n1, n0, sh);
        }
    } else {
        // blocks outside the genome hold no N; the clamped coarse words then belong to another block
        const int64_t nb = (int64_t)((g.n_units + 15) >> 4);
        const int64_t b0 = R.u0 >> 4, b1 = (R.u0 + NU - 1) >> 4;
        const int64_t cwi = coarse_word(g, R.u0);
        auto nbit = [&](int64_t b) -> bool {
            const int64_t k = b - 32 * cwi;
            return b >= 0 && b < nb && k >= 0 && k < 64 && ((R.cw >> k) & 1ull);
        };
        const bool anyN = nbit(b0) || (b1 != b0 && nbit(b1));
        if (anyN) {
#pragma unroll
            for (int j = 0; j < NU; ++j) {
                const int64_t u = R.u0 + j;
                const uint64_t v = (u >= 0 && (uint64_t)u < g.n_units) ? g.nplane[u] : 0ull;
                xn[2 * j] = (uint32_t)v; xn[2 * j + 1] = (uint32_t)(v >> 32);
            }
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                const uint32_t n0 = odd ? xn[k + 1] : xn[k], n1 = odd ? xn[k + 2] : xn[k + 1];
                P.n[k] = alignr(n1, n0, sh);
            }
        } else {
#pragma unroll
            for (int k = 0; k < NQ; ++k) P.n[k] = 0;
        }
    }
    P.n[NQ] = 0;

    // positions outside [0, csize) of the chromosome read as 'N'
    int64_t vlo = -ws, vhi = csize - ws;
    vlo = vlo < 0 ? 0 : (vlo > W ? W : vlo);
    vhi = vhi < 0 ? 0 : (vhi > W ? W : vhi);
    if (vlo != 0 || vhi != W) {
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const uint32_t v = rmask32((int)vlo, (int)vhi, k);
            P.lo[k] &= v; P.hi[k] &= v; P.n[k] = (P.n[k] & v) | ~v;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Word-pair layout (g.wt, fc2_wtab_launch): the genome as 8-byte pairs (lo, hi) of 32-base code
// words, followed in the same allocation by a copy shifted by half a 128-B line (64 B).  A window
// of W <= 128 bases starting at base g0 needs the nwd = ceil(((g0 & 31) + W) / 32) <= 5 pairs from
// q0 = g0 >> 5: ONE contiguous 32 B (nwd <= 4: every 100-bp pair) or 40 B run that lies inside one
// line of either copy.  Both copies carry zero pairs in front (q0 >= -4 for any window the scan
// evaluates), so no offset is negative.  Lanes 2m, 2m+1 load its two 16-B halves in one
// instruction (one L2 request, like the cooperative unit loads); the owner adds the fifth pair only
// when nwd = 5 (or three lanes load 48 B, windows_issue_w3).  Loads are
// buffer loads with 32-bit offsets: the hardware range check returns 0 past the table, and windows
// outside the chromosome are masked to 'N' in window_finish_w whatever was read, so no index is
// clamped.  Compared with the 64-base unit layout there is no word-parity select, no third unit
// request (17 % of 76-base windows) and no 64-bit address arithmetic.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

struct WinW {
    uint32_t off;       // byte offset of the window's first pair in g.wt (either copy)
    uint32_t q0;        // first 32-base word (two's complement when the window starts before base 0)
    unsigned sh;        // g0 & 31
    int nwd;            // word pairs needed, 1..5
    u32x4 v0, v1;       // pairs 0-1, 2-3 (lo, hi, lo, hi)
    u32x2 v4;           // pair 4 (nwd == 5 only)
    u32x4 n03;          // N-plane words q0 .. q0+3 (flagged windows only)
    uint32_t n4;        // N-plane word q0+4
};

// tri: the window is read as a 48-B region from its run start, so the run must start within the
// first 80 B of its line: the copy is chosen by start offset (main copy if <= 80 B into the line,
// else the shifted copy, where it starts 16..64 B in) instead of by run end.
__device__ __forceinline__ void window_geom_w(const fc2_genome_view &g, uint64_t cstart, int64_t ws, int W, WinW &R,
                                              bool tri = false) {
    const int64_t g0 = (int64_t)cstart + ws;
    const int32_t q0 = (int32_t)(g0 >> 5);
    R.q0 = (uint32_t)q0;
    R.sh = (unsigned)(g0 & 31);
    R.nwd = ((int)R.sh + W + 31) >> 5;
    const bool twin = tri ? (q0 & 15) > 10                   // would start more than 80 B into a main line
                          : (int)(q0 & 15) + R.nwd > 16;     // would cross a 128-B line of the main copy
    R.off = twin ? (uint32_t)g.wt_twin_off + (uint32_t)(q0 + 8) * 8u : 128u + (uint32_t)q0 * 8u;   // main copy: 16 zero pairs in front
}

// Issue phase (all 64 lanes; inactive lanes pass a harmless geometry).  rs/rn: buffer resources of
// g.wt and of the N plane viewed as 32-bit words.
__device__ __forceinline__ void windows_issue_w(const fc2_genome_view &g, __amdgpu_buffer_rsrc_t rs,
                                                __amdgpu_buffer_rsrc_t rn, const uint32_t *s_nsuper, uint64_t cstart,
                                                int64_t wsA, int64_t wsB, int W, bool active, WinW &rA, WinW &rB,
                                                u32x4 (&cl)[2][2]) {
    window_geom_w(g, cstart, wsA, W, rA);
    window_geom_w(g, cstart, wsB, W, rB);
    const int lane = (int)(threadIdx.x & 63);
    const int64_t wsx[2] = {wsA, wsB};
    WinW *R[2] = {&rA, &rB};
    // all LDS traffic of the issue phase in one batch: four offset permutes + super-map words
    uint32_t src[2][2], sw[2][2] = {{0u, 0u}, {0u, 0u}}, sb[2][2] = {{0u, 0u}, {0u, 0u}};
    bool sv[2] = {false, false};
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int c = 0; c < 2; ++c)
            src[x][c] = (uint32_t)__builtin_amdgcn_ds_bpermute((32 * c + (lane >> 1)) << 2, (int)R[x]->off);
    if (!(FC2_ABLATE & 2) && s_nsuper) {
        const int64_t top = (int64_t)(g.n_units * 64) - 1;
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            int64_t lo = (int64_t)cstart + wsx[x], hi = lo + W - 1;
            lo = lo < 0 ? 0 : lo;
            hi = hi > top ? top : hi;
            sv[x] = active && lo <= hi;
            const uint32_t k0 = sv[x] ? (uint32_t)((uint64_t)lo >> g.nsuper_shift) : 0u,
                           k1 = sv[x] ? (uint32_t)((uint64_t)hi >> g.nsuper_shift) : 0u;   // k1 <= k0 + 1
            sw[x][0] = s_nsuper[k0 >> 5];
            sw[x][1] = s_nsuper[k1 >> 5];
            sb[x][0] = k0 & 31u;
            sb[x][1] = k1 & 31u;
        }
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int c = 0; c < 2; ++c)
            cl[x][c] = __builtin_amdgcn_raw_buffer_load_b128(rs, src[x][c] + 16u * (uint32_t)(lane & 1), 0, 0);
#pragma unroll
    for (int x = 0; x < 2; ++x) {
        WinW &Q = *R[x];
        Q.v4 = u32x2{0u, 0u};
        if (!(FC2_ABLATE & 8) && active && Q.nwd > 4) Q.v4 = __builtin_amdgcn_raw_buffer_load_b64(rs, Q.off + 32u, 0, 0);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x) {
        WinW &Q = *R[x];
        const bool nflag = sv[x] && (((sw[x][0] >> sb[x][0]) | (sw[x][1] >> sb[x][1])) & 1u);
        Q.n03 = u32x4{0u, 0u, 0u, 0u};
        Q.n4 = 0u;
        if (nflag) {
            // one dword per load, each range-checked on its own (a 16-B load past the plane's end would
            // drop all four); words before base 0 (chromosome 0, window starting at g0 < 0) are not
            // loaded at all, so no offset ever wraps
            uint32_t nw[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const int32_t w = (int32_t)Q.q0 + j;
                nw[j] = 0u;
                if (w >= 0 && j < Q.nwd) nw[j] = __builtin_amdgcn_raw_buffer_load_b32(rn, (uint32_t)w * 4u, 0, 0);
            }
            Q.n03 = u32x4{nw[0], nw[1], nw[2], nw[3]};
            Q.n4 = nw[4];
        }
    }
}

__device__ __forceinline__ void windows_exchange_w(u32x4 *xchg, const u32x4 (&cl)[2][2], WinW &rA, WinW &rB) {
    const int lane = (int)(threadIdx.x & 63);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int c = 0; c < 2; ++c) xchg[(2 * x + c) * 64 + lane] = cl[x][c];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int c = lane >> 5, m = lane & 31;
    rA.v0 = xchg[(0 + c) * 64 + 2 * m];
    rA.v1 = xchg[(0 + c) * 64 + 2 * m + 1];
    rB.v0 = xchg[(2 + c) * 64 + 2 * m];
    rB.v1 = xchg[(2 + c) * 64 + 2 * m + 1];
}

// Plain (one lane, one window) form of the word-pair loads, for locus-ordered or cache-resident
// batches: two 16-B loads (+ the fifth pair), no LDS.  twin_ok = 0 keeps every window in the main
// copy (an ordered batch re-reads its lines from L2; the shifted copy would only double that
// footprint).  The N test is the coarse map (one 8-byte word from L2, consumed in
// window_nwords_plain); flagged windows read their N words one round trip later.
__device__ __forceinline__ void window_issue_w_plain(const fc2_genome_view &g, __amdgpu_buffer_rsrc_t rs,
                                                     uint64_t cstart, int64_t ws, int W, bool twin_ok, WinW &R,
                                                     uint64_t &cw) {
    const int64_t g0 = (int64_t)cstart + ws;
    const int32_t q0 = (int32_t)(g0 >> 5);
    R.q0 = (uint32_t)q0;
    R.sh = (unsigned)(g0 & 31);
    R.nwd = ((int)R.sh + W + 31) >> 5;
    const bool twin = twin_ok && (int)(q0 & 15) + R.nwd > 16;
    R.off = twin ? (uint32_t)g.wt_twin_off + (uint32_t)(q0 + 8) * 8u : 128u + (uint32_t)q0 * 8u;   // main copy: 16 zero pairs in front
    R.v0 = __builtin_amdgcn_raw_buffer_load_b128(rs, R.off, 0, 0);
    R.v1 = __builtin_amdgcn_raw_buffer_load_b128(rs, R.off + 16u, 0, 0);
    R.v4 = u32x2{0u, 0u};
    if (R.nwd > 4) R.v4 = __builtin_amdgcn_raw_buffer_load_b64(rs, R.off + 32u, 0, 0);
    const int64_t w = coarse_word(g, (int64_t)(q0 >> 1));
    cw = ((((g.n_units + 15) >> 4) + 31) >> 5 >= 2) ? *reinterpret_cast<const uint64_t *>(g.ncoarse + w)
                                                     : (uint64_t)g.ncoarse[0];
}

__device__ __forceinline__ void window_nwords_plain(const fc2_genome_view &g, __amdgpu_buffer_rsrc_t rn, uint64_t cw,
                                                    WinW &R) {
    const int64_t nb = (int64_t)((g.n_units + 15) >> 4);
    const int32_t q0 = (int32_t)R.q0;
    const int64_t g0 = (int64_t)q0 * 32 + R.sh;
    const int64_t b0 = g0 >> 10, b1 = (g0 + 32 * R.nwd - 1) >> 10;
    const int64_t cwi = coarse_word(g, (int64_t)(q0 >> 1));
    auto nbit = [&](int64_t b) -> bool {
        const int64_t k = b - 32 * cwi;
        return b >= 0 && b < nb && k >= 0 && k < 64 && ((cw >> k) & 1ull);
    };
    R.n03 = u32x4{0u, 0u, 0u, 0u};
    R.n4 = 0u;
    if (nbit(b0) || (b1 != b0 && nbit(b1))) {
        uint32_t nw[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int32_t wj = q0 + j;
            nw[j] = 0u;
            if (wj >= 0 && j < R.nwd) nw[j] = __builtin_amdgcn_raw_buffer_load_b32(rn, (uint32_t)wj * 4u, 0, 0);
        }
        R.n03 = u32x4{nw[0], nw[1], nw[2], nw[3]};
        R.n4 = nw[4];
    }
}

// Long-window forms (three- and five-lane): the N test of both windows from the LDS super map,
// looked up before any load is issued (all LDS traffic of the issue phase first) ...
struct SuperN {
    uint32_t sw[2][2], sb[2][2];
    bool sv[2];
};
__device__ __forceinline__ void super_lookup_long(const fc2_genome_view &g, const uint32_t *s_nsuper, uint64_t cstart,
                                                  const int64_t (&wsx)[2], int W, bool active, SuperN &S) {
#pragma unroll
    for (int x = 0; x < 2; ++x) {
        S.sv[x] = false;
        S.sw[x][0] = S.sw[x][1] = S.sb[x][0] = S.sb[x][1] = 0u;
    }
    if ((FC2_ABLATE & 2) || !s_nsuper) return;
    const int64_t top = (int64_t)(g.n_units * 64) - 1;
#pragma unroll
    for (int x = 0; x < 2; ++x) {
        int64_t lo = (int64_t)cstart + wsx[x], hi = lo + W - 1;
        lo = lo < 0 ? 0 : lo;
        hi = hi > top ? top : hi;
        S.sv[x] = active && lo <= hi;
        const uint32_t k0 = S.sv[x] ? (uint32_t)((uint64_t)lo >> g.nsuper_shift) : 0u,
                       k1 = S.sv[x] ? (uint32_t)((uint64_t)hi >> g.nsuper_shift) : 0u;
        S.sw[x][0] = s_nsuper[k0 >> 5];
        S.sw[x][1] = s_nsuper[k1 >> 5];
        S.sb[x][0] = k0 & 31u;
        S.sb[x][1] = k1 & 31u;
    }
}
// ... and, after the window loads are in flight, the N-plane words of the flagged windows (one
// range-checked dword load each; words before base 0 are not loaded at all)
__device__ __forceinline__ void window_nwords_long(__amdgpu_buffer_rsrc_t rn, const SuperN &S, int x, WinW &Q) {
    Q.v4 = u32x2{0u, 0u};
    const bool nflag = S.sv[x] && (((S.sw[x][0] >> S.sb[x][0]) | (S.sw[x][1] >> S.sb[x][1])) & 1u);
    Q.n03 = u32x4{0u, 0u, 0u, 0u};
    Q.n4 = 0u;
    if (nflag) {
        uint32_t nw[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int32_t wj = (int32_t)Q.q0 + j;
            nw[j] = 0u;
            if (wj >= 0 && j < Q.nwd) nw[j] = __builtin_amdgcn_raw_buffer_load_b32(rn, (uint32_t)wj * 4u, 0, 0);
        }
        Q.n03 = u32x4{nw[0], nw[1], nw[2], nw[3]};
        Q.n4 = nw[4];
    }
}

// Three-lane form of the cooperative word-pair loads, for batches with windows longer than 97
// bases (150-bp reads: a window needs 5 pairs = 40 B, more than two 16-B lane loads).  Each window is
// read as the 48 B from its run start r -- inside one 128-B line because the copy is picked so
// that r lies at most 80 B into its line (window_geom_w, tri) -- by three consecutive lanes of ONE
// instruction: 21 windows per instruction, 7 instructions for the wave's 128 windows, one L2
// request per window (the two-lane form spends a second request on the owner's fifth-pair load:
// +13 % at 150 bp, profiles/r01/ab_fifth_pair.jsonl).
__device__ __forceinline__ void windows_issue_w3(const fc2_genome_view &g, __amdgpu_buffer_rsrc_t rs,
                                                 __amdgpu_buffer_rsrc_t rn, const uint32_t *s_nsuper,
                                                 uint64_t cstart, int64_t wsA, int64_t wsB, int W, bool active,
                                                 WinW &rA, WinW &rB, u32x4 (&cl)[7]) {
    window_geom_w(g, cstart, wsA, W, rA, true);
    window_geom_w(g, cstart, wsB, W, rB, true);
    const int lane = (int)(threadIdx.x & 63);
    const int64_t wsx[2] = {wsA, wsB};
    WinW *R[2] = {&rA, &rB};
    const uint32_t sA = rA.off, sB = rB.off;                // region = [off, off + 48), inside one line
    uint32_t src[7];
    int part[7];
    bool ok[7];
#pragma unroll
    for (int c = 0; c < 7; ++c) {
        const int w = 21 * c + lane / 3;                  // window served by this lane in instruction c
        ok[c] = lane < 63 && w < 128;
        part[c] = lane % 3;
        const int owner = w & 63;
        // instructions 0-2 serve only A windows (w <= 62), 4-6 only B windows (w >= 84): one permute
        if (21 * c + 20 < 64) {
            src[c] = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)sA);
        } else if (21 * c >= 64) {
            src[c] = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)sB);
        } else {
            const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)sA);
            const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)sB);
            src[c] = (w >> 6) ? b : a;
        }
    }
    SuperN S;
    super_lookup_long(g, s_nsuper, cstart, wsx, W, active, S);
#pragma unroll
    for (int c = 0; c < 7; ++c) {
        cl[c] = u32x4{0u, 0u, 0u, 0u};
        if (ok[c]) cl[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, src[c] + 16u * (uint32_t)part[c], 0, 0);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x) window_nwords_long(rn, S, x, *R[x]);
}

// Owner side: the first 40 B of each window's three 16-B pieces, in two phases through 4 LDS slots
// (4 KB per wave instead of 7; 1.5 % faster at 150 bp, profiles/r01/ab_tri_4slot.jsonl): instructions
// 0-3 hold every A window and B windows 64..83, then instructions 4-6 overwrite slots 0-2 with B
// windows 84..127.
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void take_w3(const u32x4 *xchg, int slot, int w, WinW &Q) {
    const int base = slot * 64 + 3 * (w % 21);
    const u32x4 p0 = xchg[base], p1 = xchg[base + 1];
    const u32x2 p2 = *reinterpret_cast<const u32x2 *>(xchg + base + 2);
    Q.v0 = p0;
    Q.v1 = p1;
    Q.v4 = p2;
}
__device__ __forceinline__ void windows_exchange_w3(u32x4 *xchg, const u32x4 (&cl)[7], WinW &rA, WinW &rB) {
    const int lane = (int)(threadIdx.x & 63);
    const int wB = 64 + lane;
#pragma unroll
    for (int c = 0; c < 4; ++c) xchg[c * 64 + lane] = cl[c];
    wave_sync_lds();
    take_w3(xchg, lane / 21, lane, rA);
    if (wB < 84) take_w3(xchg, 3, wB, rB);
    wave_sync_lds();                           // every phase-1 read done before slots 0-2 are reused
#pragma unroll
    for (int c = 4; c < 7; ++c) xchg[(c - 4) * 64 + lane] = cl[c];
    wave_sync_lds();
    if (wB >= 84) take_w3(xchg, wB / 21 - 4, wB, rB);
}

// Five-lane form of the long-window loads (the default for windows longer than 97 bases since round
// 3; FC2_TUNE_TRI = 3): each window's 40 B (its five word pairs from the run start, the copy chosen as
// for the three-lane form) by five consecutive lanes of ONE 8-B load instruction: 12 windows per
// instruction (lanes 60-63 idle), 11 instructions for the wave's 128 windows, still one L2 request
// per window, but 22 VGPRs of loads in flight where the three-lane form holds 28: 74 instead of 84
// VGPRs, 6 instead of 4 waves per SIMD, 3 % faster at 150 bp (profiles/r03/ab_tri5.jsonl).
__device__ __forceinline__ void windows_issue_w5(const fc2_genome_view &g, __amdgpu_buffer_rsrc_t rs,
                                                 __amdgpu_buffer_rsrc_t rn, const uint32_t *s_nsuper,
                                                 uint64_t cstart, int64_t wsA, int64_t wsB, int W, bool active,
                                                 WinW &rA, WinW &rB, u32x2 (&cl)[11]) {
    window_geom_w(g, cstart, wsA, W, rA, true);
    window_geom_w(g, cstart, wsB, W, rB, true);
    const int lane = (int)(threadIdx.x & 63);
    const int64_t wsx[2] = {wsA, wsB};
    WinW *R[2] = {&rA, &rB};
    const uint32_t sA = rA.off, sB = rB.off;                // region = [off, off + 40), inside one line
    uint32_t src[11];
    bool ok[11];
    const uint32_t part = 8u * (uint32_t)(lane % 5);
#pragma unroll
    for (int c = 0; c < 11; ++c) {
        const int w = 12 * c + lane / 5;                  // window served by this lane in instruction c
        ok[c] = lane < 60 && w < 128;
        const int owner = w & 63;
        // instructions 0-4 serve only A windows (w <= 59), 6-10 only B windows (w >= 72)
        if (12 * c + 11 < 64) {
            src[c] = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)sA);
        } else if (12 * c >= 64) {
            src[c] = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)sB);
        } else {
            const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)sA);
            const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)sB);
            src[c] = (w >> 6) ? b : a;
        }
    }
    SuperN S;
    super_lookup_long(g, s_nsuper, cstart, wsx, W, active, S);
#pragma unroll
    for (int c = 0; c < 11; ++c) {
        cl[c] = u32x2{0u, 0u};
        if (ok[c]) cl[c] = __builtin_amdgcn_raw_buffer_load_b64(rs, src[c] + part, 0, 0);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x) window_nwords_long(rn, S, x, *R[x]);
}

// Owner side of the five-lane form: the wave's 4 KB of LDS slots hold eight instructions' 8-B pieces
// (64 each); instructions 0-7 carry every A window and B windows 64..95, then 8-10 overwrite slots
// 0-2 with B windows 96..127.
__device__ __forceinline__ void take_w5(const u32x2 *xchg, int slot, int w, WinW &Q) {
    const int base = slot * 64 + 5 * (w % 12);
    const u32x2 p0 = xchg[base], p1 = xchg[base + 1], p2 = xchg[base + 2], p3 = xchg[base + 3], p4 = xchg[base + 4];
    Q.v0 = u32x4{p0.x, p0.y, p1.x, p1.y};
    Q.v1 = u32x4{p2.x, p2.y, p3.x, p3.y};
    Q.v4 = p4;
}
__device__ __forceinline__ void windows_exchange_w5(u32x2 *xchg, const u32x2 (&cl)[11], WinW &rA, WinW &rB) {
    const int lane = (int)(threadIdx.x & 63);
    const int wB = 64 + lane;
#pragma unroll
    for (int c = 0; c < 8; ++c) xchg[c * 64 + lane] = cl[c];
    wave_sync_lds();
    take_w5(xchg, lane / 12, lane, rA);
    if (wB < 96) take_w5(xchg, wB / 12, wB, rB);
    wave_sync_lds();                           // every phase-1 read done before slots 0-2 are reused
#pragma unroll
    for (int c = 8; c < 11; ++c) xchg[(c - 8) * 64 + lane] = cl[c];
    wave_sync_lds();
    if (wB >= 96) take_w5(xchg, wB / 12 - 8, wB, rB);
}

template <int NQ>
__device__ __forceinline__ void window_finish_w(const WinW &R, int64_t csize, int64_t ws, int W, P32<NQ> &P) {
    static_assert(NQ == 4, "word-pair windows cover W <= 128");
    const uint32_t lo[6] = {R.v0.x, R.v0.z, R.v1.x, R.v1.z, R.v4.x, 0u};
    const uint32_t hi[6] = {R.v0.y, R.v0.w, R.v1.y, R.v1.w, R.v4.y, 0u};
    const uint32_t nn[6] = {R.n03.x, R.n03.y, R.n03.z, R.n03.w, R.n4, 0u};
    const unsigned sh = R.sh;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        P.lo[k] = alignr(lo[k + 1], lo[k], sh);
        P.hi[k] = alignr(hi[k + 1], hi[k], sh);
        P.n[k] = alignr(nn[k + 1], nn[k], sh);
    }
    P.lo[NQ] = 0; P.hi[NQ] = 0; P.n[NQ] = 0;
    // positions outside [0, csize) of the chromosome read as 'N'
    int64_t vlo = -ws, vhi = csize - ws;
    vlo = vlo < 0 ? 0 : (vlo > W ? W : vlo);
    vhi = vhi < 0 ? 0 : (vhi > W ? W : vhi);
    if (vlo != 0 || vhi != W) {
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const uint32_t v = rmask32((int)vlo, (int)vhi, k);
            P.lo[k] &= v; P.hi[k] &= v; P.n[k] = (P.n[k] & v) | ~v;
        }
    }
}

template <int NQ>
__device__ __forceinline__ void window_dummy(P32<NQ> &P) {
#pragma unroll
    for (int k = 0; k <= NQ; ++k) { P.lo[k] = 0; P.hi[k] = 0; P.n[k] = ~0u; }
}

template <int NQ>
__device__ __forceinline__ unsigned code_at32(const P32<NQ> &P, int pos) {
    const int k = pos >> 5, b = pos & 31;
    uint32_t lo = 0, hi = 0, nn = 0;
#pragma unroll
    for (int kk = 0; kk < NQ; ++kk)
        if (kk == k) { lo = P.lo[kk]; hi = P.hi[kk]; nn = P.n[kk]; }
    return ((nn >> b) & 1u) ? 4u : (((lo >> b) & 1u) | (((hi >> b) & 1u) << 1));
}

struct Best32 {
    int n_hits = 0, best_score = 0, best_x = -1, best_minus = 0, best_dist = 0, best_ov = 0, n_ties = 0;
};

__device__ __forceinline__ int ov_of(int x, int l, int margin) {  // find_circ.py:917-922
    int ov = 0;
    if (margin) {
        if (x < margin) ov = margin - x;
        if (l - x < margin) ov = margin - (l - x);
    }
    return ov;
}

__device__ __forceinline__ void add_hit(Best32 &B, int x, int minus, int dist, int ov, int score) {
    if (B.n_hits == 0 || score > B.best_score) {
        B.best_score = score; B.best_x = x; B.best_minus = minus; B.best_dist = dist; B.best_ov = ov; B.n_ties = 1;
    } else if (score == B.best_score) {
        B.n_ties += 1;
    }
    B.n_hits += 1;
}

__device__ __forceinline__ uint64_t pack_result(const Best32 &B, unsigned gtag12, unsigned err) {
    if (B.n_hits == 0) return (uint64_t)(uint16_t)(int16_t)-1 | ((uint64_t)(FC2_RES_DONE | err) << 48);
    const unsigned nt = B.n_hits >= 2 ? (unsigned)B.n_ties : 1u;   // find_circ.py:961-972
    const unsigned dist = B.best_dist > 255 ? 255u : (unsigned)B.best_dist;
    const unsigned info = FC2_RES_DONE | err | (B.best_minus ? FC2_RES_MINUS : 0u) |
                          ((gtag12 << FC2_RES_GTAG_SHIFT) & FC2_RES_GTAG_MASK);
    return (uint64_t)(uint16_t)(int16_t)B.best_x | ((uint64_t)(dist & 0xFF) << 16) |
           ((uint64_t)(B.best_ov & 0xFF) << 24) | ((uint64_t)(nt > 0xFFFF ? 0xFFFFu : nt) << 32) |
           ((uint64_t)info << 48);
}

// XCD-aware block order (guide §5.5 T1): the dispatcher deals blocks round-robin
// over the 8 XCDs, so block b runs on XCD b % 8; remap so that XCD x processes a
// contiguous range of the batch (bijective for any grid size).  Only a
// performance hint: correctness never depends on placement.
__device__ __forceinline__ uint64_t xcd_block(uint32_t b, uint32_t nwg) {
    const uint32_t x = b & 7u, j = b >> 3, q = nwg >> 3, r = nwg & 7u;
    return (uint64_t)x * q + (x < r ? x : r) + j;
}

// One pair per lane of tile t: the hot path.  s_cstart/s_csize: LDS chromosome table (if lds_tab);
// s_nsuper: LDS super-coarse N map or nullptr.
// COOP: cooperative window loads (windows_issue_coop); then no lane may leave before the
// exchange, so exits are deferred through `active`.  xchg: this wave's 4 x 64 LDS slots.
// PW > 0: window-carrying batch (fc2_batch_view.win_words, pw = PW): the windows arrive with the
// record in round trip 1 and nothing is gathered from the genome (NQ == 4, !COOP, !WL).
template <int NQ, bool NT, bool COOP, bool WL = false, int PW = 0, int TRI = 0>
__device__ __forceinline__ void scan_pair(const fc2_params &p, const fc2_genome_view &g, const fc2::ScanView &bv,
                                          uint64_t *__restrict__ out, uint64_t *__restrict__ tiemask, uint32_t tw,
                                          uint64_t i, const uint64_t *s_cstart, const int64_t *s_csize, bool lds_tab,
                                          const uint32_t *s_nsuper, ulonglong2 *xchg) {
    const bool live = i < bv.n;
    if (!COOP && !live) return;
    // round trip 1: the pair record and its read rows (both indexed by i only)
    constexpr int R = NQ + 1;                  // 64-bit row words the largest row can use (2l <= 64R)
    u64x2 prv = {0ull, 0ull};
    uint64_t rv[R];
#pragma unroll
    for (int j = 0; j < R; ++j) rv[j] = 0;
    static_assert(PW == 0 || (NQ == 4 && !COOP && !WL && PW <= 4), "window rows: plain form, l + 2 <= 128");
    uint64_t wv[PW > 0 ? 2 * PW : 1];
#pragma unroll
    for (int j = 0; j < (PW > 0 ? 2 * PW : 1); ++j) wv[j] = 0;
    if (live) {
        prv = ld_pair_raw<NT>(bv.pairs + i);
#pragma unroll
        for (int j = 0; j < R; ++j)
            rv[j] = ((uint32_t)j < bv.rw) ? ld_stream<NT>(bv.read_words + (uint64_t)j * bv.stride + i) : 0ull;
        if constexpr (PW > 0) {
#pragma unroll
            for (int j = 0; j < 2 * PW; ++j) wv[j] = ld_stream<NT>(bv.win_words + (uint64_t)j * bv.stride + i);
        }
    }
    fc2_pair pr;
    __builtin_memcpy(&pr, &prv, sizeof pr);
    bool active = live && !(pr.flags & FC2_PAIR_BYTEPATH);   // BYTEPATH: left for the byte-exact kernel
    if (live && !active && bv.c_words) mark_unscanned(bv, i);
    if (!COOP && !active) return;

    const int e = p.asize - p.margin;
    const int l = (int)pr.read_len - 2 * e;
    const bool want_ties = p.allhits != 0;
    int W = l + 2;                             // flank, find_circ.py:900
    // chromosome of the pair: LDS, or (very many contigs) one more round trip to L2
    uint64_t cstart = 0;
    int64_t csize = (int64_t)1 << 62;          // dummy genome: every window is all 'N'
    if (!g.dummy) {
        const bool known = pr.chrom < g.n_chrom;
        const uint32_t c = known ? pr.chrom : 0u;
        if constexpr (PW > 0) {
            csize = g.chrom_size[c];           // only the window-range check needs the chromosome
        } else if (lds_tab) {
            cstart = s_cstart[c];
            csize = s_csize[c];
        } else {
            cstart = g.chrom_start[c];
            csize = g.chrom_size[c];
            __builtin_amdgcn_sched_barrier(0); // both loads issued before either is waited on
        }
        if (!known) { cstart = 0; csize = 0; }
    }
    const int64_t wsA = (int64_t)pr.a_pos + e;
    const int64_t wsB = (int64_t)pr.b_aend - e - W;
    // (the dummy genome's "N"*(end-start), find_circ.py:370-371, has the requested length anywhere)
    if (active && ((pr.flags & FC2_PAIR_SKIP) || l < 0 || l > 32 * NQ - 2 || pr.chrom >= g.n_chrom ||
                   (!g.dummy && (wsA > csize || wsA + W < 0 || wsB > csize || wsB + W < 0)))) {
        // skipped / empty x-range: no hit; anything else is routed to the byte path by the host
        const bool err = !(pr.flags & FC2_PAIR_SKIP) && l >= 0;
        Best32 none;
        emit<NT>(bv, out, i, pack_result(none, 0, err ? FC2_RES_ERR_WIN : 0u));
        if (want_ties)
            for (uint32_t k = 0; k < tw; ++k) tiemask[(uint64_t)k * bv.stride + i] = 0;
        if (!COOP) return;
        active = false;
    }

    // round trip 3: both genome windows (find_circ.py:900-902) and their coarse N words
    WinRaw<NQ> rA, rB;
    ulonglong2 cl[2][2];
    WinW wA, wB;
    u32x4 wcl[2][2];
    u32x4 wcl3[TRI == 1 ? 7 : 1];
    u32x2 wcl5[TRI == 2 ? 11 : 1];
    uint64_t cwA = 0, cwB = 0;
    __amdgpu_buffer_rsrc_t rs, rn;
    if constexpr (WL) {
        rs = __builtin_amdgcn_make_buffer_rsrc((void *)g.wt, 0, (int)(uint32_t)g.wt_bytes, 0x00020000);
        const uint64_t nb = g.n_units * 8;
        rn = __builtin_amdgcn_make_buffer_rsrc((void *)g.nplane, 0,
                                               (int)(uint32_t)(nb > 0xFFFFFFFFull ? 0xFFFFFFFFull : nb), 0x00020000);
    }
    if constexpr (COOP && WL && TRI == 1) {
        static_assert(NQ == 4, "word-pair windows: l + 2 <= 128");
        if (!active) W = 2;
        windows_issue_w3(g, rs, rn, s_nsuper, active ? cstart : 0, active ? wsA : 0, active ? wsB : 0, W, active, wA,
                         wB, wcl3);
    } else if constexpr (COOP && WL && TRI == 2) {
        static_assert(NQ == 4, "word-pair windows: l + 2 <= 128");
        if (!active) W = 2;
        windows_issue_w5(g, rs, rn, s_nsuper, active ? cstart : 0, active ? wsA : 0, active ? wsB : 0, W, active, wA,
                         wB, wcl5);
    } else if constexpr (COOP && WL) {
        static_assert(NQ == 4, "word-pair windows: l + 2 <= 128");
        if (!active) W = 2;
        windows_issue_w(g, rs, rn, s_nsuper, active ? cstart : 0, active ? wsA : 0, active ? wsB : 0, W, active, wA,
                        wB, wcl);
    } else if constexpr (WL) {
        static_assert(NQ == 4, "word-pair windows: l + 2 <= 128");
        window_issue_w_plain(g, rs, cstart, wsA, W, g.units_twin != nullptr, wA, cwA);
        window_issue_w_plain(g, rs, cstart, wsB, W, g.units_twin != nullptr, wB, cwB);
    } else if constexpr (COOP) {
        if (!active) W = 2;                    // a harmless window for a lane that only loads for others
        windows_issue_coop<NQ>(g, s_nsuper, active ? cstart : 0, active ? wsA : 0, active ? wsB : 0, W, active,
                               rA, rB, cl);
    } else if constexpr (PW > 0) {
        // windows came with the record
    } else if (!g.dummy) {
        window_issue<NQ>(g, s_nsuper, cstart, wsA, W, rA);
        window_issue<NQ>(g, s_nsuper, cstart, wsB, W, rB);
    }
    __builtin_amdgcn_sched_barrier(0);         // every window load in flight before the first wait

    // --- internal read part: 32-bit plane words (while the windows are in flight) ---
    uint32_t Ilo[NQ], Ihi[NQ], In[NQ];
    {
        uint32_t r[2 * R + 1];
#pragma unroll
        for (int j = 0; j < R; ++j) { r[2 * j] = (uint32_t)rv[j]; r[2 * j + 1] = (uint32_t)(rv[j] >> 32); }
        r[2 * R] = 0;
#pragma unroll
        for (int k = 0; k < NQ; ++k) Ilo[k] = r[k] & rmask32(0, l, k);
        // high plane starts at bit l: shift by l>>5 words (selects), then by l&31 bits (alignbit)
        uint32_t h[2 * R + 1];
#pragma unroll
        for (int k = 0; k < 2 * R + 1; ++k) h[k] = r[k];
        constexpr int LV = NQ <= 4 ? 2 : (NQ <= 8 ? 3 : 4);
        word_shift(h, l >> 5, LV);
        const unsigned s = (unsigned)(l & 31);
#pragma unroll
        for (int k = 0; k < NQ; ++k) Ihi[k] = alignr(h[k + 1], h[k], s) & rmask32(0, l, k);
        if (active && (pr.flags & (FC2_PAIR_READ_N | FC2_PAIR_READ_N1)) == (FC2_PAIR_READ_N | FC2_PAIR_READ_N1)) {
            // a single 'N': its position came with the record, no N-row request
#pragma unroll
            for (int k = 0; k < NQ; ++k) In[k] = ((int)pr.npos >> 5) == k ? 1u << (pr.npos & 31) : 0u;
        } else if (!(FC2_ABLATE & 16) && active && (pr.flags & FC2_PAIR_READ_N)) {
#pragma unroll
            for (int j = 0; j < (NQ + 1) / 2; ++j) {
                const uint64_t v =
                    ((uint32_t)j < bv.nw) ? ld_stream<NT>(bv.read_nwords + (uint64_t)j * bv.stride + i) : 0ull;
                In[2 * j] = (uint32_t)v & rmask32(0, l, 2 * j);
                if (2 * j + 1 < NQ) In[2 * j + 1] = (uint32_t)(v >> 32) & rmask32(0, l, 2 * j + 1);
            }
        } else {
#pragma unroll
            for (int k = 0; k < NQ; ++k) In[k] = 0;
        }
    }

    P32<NQ> A, B;
    if constexpr (PW > 0) {
        // plane p word k = 32-bit word p*PW + k of the row; N rows only for flagged pairs
        uint32_t w32[8 * PW], n32[2 * PW];
#pragma unroll
        for (int j = 0; j < 2 * PW; ++j) { w32[2 * j] = (uint32_t)wv[j]; w32[2 * j + 1] = (uint32_t)(wv[j] >> 32); }
#pragma unroll
        for (int j = 0; j < 2 * PW; ++j) n32[j] = 0u;
        if (active && (pr.flags & FC2_PAIR_WIN_N)) {
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const uint64_t v = ld_stream<NT>(bv.win_nwords + (uint64_t)j * bv.stride + i);
                n32[2 * j] = (uint32_t)v;
                n32[2 * j + 1] = (uint32_t)(v >> 32);
            }
        }
#pragma unroll
        for (int k = 0; k <= NQ; ++k) {
            A.lo[k] = k < PW ? w32[0 * PW + (k < PW ? k : 0)] : 0u;
            A.hi[k] = k < PW ? w32[1 * PW + (k < PW ? k : 0)] : 0u;
            B.lo[k] = k < PW ? w32[2 * PW + (k < PW ? k : 0)] : 0u;
            B.hi[k] = k < PW ? w32[3 * PW + (k < PW ? k : 0)] : 0u;
            A.n[k] = k < PW ? n32[(k < PW ? k : 0)] : 0u;
            B.n[k] = k < PW ? n32[PW + (k < PW ? k : 0)] : 0u;
        }
        if (!active) return;
    } else if constexpr (COOP && WL && TRI == 1) {
        windows_exchange_w3(reinterpret_cast<u32x4 *>(xchg), wcl3, wA, wB);
        if (!active) return;
        window_finish_w<NQ>(wA, csize, wsA, W, A);
        window_finish_w<NQ>(wB, csize, wsB, W, B);
    } else if constexpr (COOP && WL && TRI == 2) {
        windows_exchange_w5(reinterpret_cast<u32x2 *>(xchg), wcl5, wA, wB);
        if (!active) return;
        window_finish_w<NQ>(wA, csize, wsA, W, A);
        window_finish_w<NQ>(wB, csize, wsB, W, B);
    } else if constexpr (COOP && WL) {
        windows_exchange_w(reinterpret_cast<u32x4 *>(xchg), wcl, wA, wB);
        if (!active) return;
        window_finish_w<NQ>(wA, csize, wsA, W, A);
        window_finish_w<NQ>(wB, csize, wsB, W, B);
    } else if constexpr (WL) {
        window_nwords_plain(g, rn, cwA, wA);
        window_nwords_plain(g, rn, cwB, wB);
        window_finish_w<NQ>(wA, csize, wsA, W, A);
        window_finish_w<NQ>(wB, csize, wsB, W, B);
    } else if constexpr (COOP) {
        windows_exchange_coop<NQ>(xchg, cl, rA, rB);
        if (!active) return;
    }
    if constexpr (!WL && PW == 0) {
        if (!g.dummy) {
            window_finish<NQ>(g, s_nsuper, rA, csize, wsA, W, A);
            window_finish<NQ>(g, s_nsuper, rB, csize, wsB, W, B);
        } else {
            window_dummy<NQ>(A);
            window_dummy<NQ>(B);
        }
    }

    // --- mismatch planes and prefix counts ---------------------------------------
    uint32_t mA[NQ], mB[NQ];
    int cA[NQ], cB[NQ];
    int totB = 0, accA = 0;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        const uint32_t m = rmask32(0, l, k);
        mA[k] = ((A.lo[k] ^ Ilo[k]) | (A.hi[k] ^ Ihi[k]) | (A.n[k] ^ In[k])) & m;
        const uint32_t blo = alignr(B.lo[k + 1], B.lo[k], 2), bhi = alignr(B.hi[k + 1], B.hi[k], 2),
                       bn = alignr(B.n[k + 1], B.n[k], 2);
        mB[k] = ((blo ^ Ilo[k]) | (bhi ^ Ihi[k]) | (bn ^ In[k])) & m;
        cA[k] = accA; cB[k] = totB;
        accA += __popc(mA[k]);
        totB += __popc(mB[k]);
    }

    // --- GTAG ('+') / CTAC ('-') masks for every x at once (find_circ.py:924-954) --
    uint32_t plus[NQ], minus[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        const uint32_t xm = rmask32(0, l + 1, k);
        const uint32_t aLo1 = alignr(A.lo[k + 1], A.lo[k], 1), aHi1 = alignr(A.hi[k + 1], A.hi[k], 1);
        const uint32_t bLo1 = alignr(B.lo[k + 1], B.lo[k], 1), bHi1 = alignr(B.hi[k + 1], B.hi[k], 1);
        const uint32_t A_T1 = aHi1 & aLo1;
        const uint32_t B_A0 = ~(B.lo[k] | B.hi[k] | B.n[k]);
        const uint32_t common = A_T1 & B_A0 & xm;
        plus[k] = (A.hi[k] & ~A.lo[k]) & (bHi1 & ~bLo1) & common;
        minus[k] = (A.lo[k] & ~A.hi[k]) & (bLo1 & ~bHi1) & common;
    }

    const int prim_minus = (pr.flags & FC2_PAIR_PRIMARY_REV) ? 1 : 0;
    const int sp_plus = p.strandpref ? (prim_minus ? 0 : 100) : 0;     // find_circ.py:796-797
    const int sp_minus = p.strandpref ? (prim_minus ? 100 : 0) : 0;
    Best32 Bst;
    if (!p.noncanonical) {
        // Every x of word k has dist >= (A mismatches before the word) + (B mismatches after it).
        // Words whose floor exceeds maxdist hold no hit (random pairs: none survive; planted: one,
        // rarely two).  The surviving words of a lane are walked in ascending order, one selected
        // word at a time, so a wave iterates over max(candidates per lane), not over the sum of
        // per-word maxima; x still ascends, as the stable sort at find_circ.py:966 requires.
        uint32_t cw[NQ];
        uint32_t live = 0;
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const int floor_k = cA[k] + (totB - cB[k] - __popc(mB[k]));
            cw[k] = floor_k <= p.maxdist ? (plus[k] | minus[k]) : 0u;
            live |= (cw[k] ? 1u : 0u) << k;
        }
        if (FC2_ABLATE & 4) live = 0;     // timing-only: no candidate walk
        while (live) {
            const int k = __ffs(live) - 1;
            live &= live - 1;
            uint32_t w = 0, a = 0, bm = 0, mi = 0;
            int base = 0;
#pragma unroll
            for (int kk = 0; kk < NQ; ++kk)
                if (kk == k) { w = cw[kk]; a = mA[kk]; bm = mB[kk]; mi = minus[kk]; base = cA[kk] + totB - cB[kk]; }
            while (w) {
                const int b = __ffs(w) - 1;
                w &= w - 1;
                const uint32_t below = (1u << b) - 1u;
                const int dist = base + __popc(a & below) - __popc(bm & below);
                if (dist <= p.maxdist) {
                    const int x = 32 * k + b;
                    const int isminus = (int)((mi >> b) & 1u);
                    const int ov = ov_of(x, l, p.margin);
                    add_hit(Bst, x, isminus, dist, ov, 20 - 10 * dist - ov + (isminus ? sp_minus : sp_plus));
                }
            }
        }
    } else {
        int d = totB;
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            for (int b = 0; b < 32; ++b) {
                const int x = 32 * k + b;
                if (x > l) break;
                if (d <= p.maxdist) {
                    const int ov = ov_of(x, l, p.margin);
                    const int cp = (int)((plus[k] >> b) & 1u), cm = (int)((minus[k] >> b) & 1u);
                    add_hit(Bst, x, 0, d, ov, 20 * cp - 10 * d - ov + sp_plus);
                    add_hit(Bst, x, 1, d, ov, 20 * cm - 10 * d - ov + sp_minus);
                }
                d += (int)((mA[k] >> b) & 1u) - (int)((mB[k] >> b) & 1u);
            }
        }
    }

    unsigned gtag12 = 0;
    if (Bst.n_hits) {
        if (!p.noncanonical) {
            // a canonical hit sits where the GTAG / CTAC mask is set: A[x]A[x+1]B[x]B[x+1] is
            // "GTAG" or "CTAC" by construction (codes A0 C1 G2 T3), no base lookup needed
            constexpr unsigned kGTAG = 2u | (3u << 3) | (0u << 6) | (2u << 9);
            constexpr unsigned kCTAC = 1u | (3u << 3) | (0u << 6) | (1u << 9);
            gtag12 = Bst.best_minus ? kCTAC : kGTAG;
        } else {
            const int x = Bst.best_x;
            gtag12 = code_at32<NQ>(A, x) | (code_at32<NQ>(A, x + 1) << 3) | (code_at32<NQ>(B, x) << 6) |
                     (code_at32<NQ>(B, x + 1) << 9);
        }
    }
    emit<NT>(bv, out, i, pack_result(Bst, gtag12, 0));

    if (want_ties) {
        // --all-hits: every tie (find_circ.py:966-974); tie words are 64-bit, x-major
        uint32_t tp[NQ], tm[NQ];
#pragma unroll
        for (int k = 0; k < NQ; ++k) { tp[k] = 0; tm[k] = 0; }
        if (Bst.n_hits) {
            const int best = Bst.best_score;
            int d = totB;
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                for (int b = 0; b < 32; ++b) {
                    const int x = 32 * k + b;
                    if (x > l) break;
                    if (d <= p.maxdist) {
                        const int ov = ov_of(x, l, p.margin);
                        const int cp = (int)((plus[k] >> b) & 1u), cm = (int)((minus[k] >> b) & 1u);
                        if (p.noncanonical) {
                            if (20 * cp - 10 * d - ov + sp_plus == best) tp[k] |= 1u << b;
                            if (20 * cm - 10 * d - ov + sp_minus == best) tm[k] |= 1u << b;
                        } else if (cp || cm) {
                            if (20 - 10 * d - ov + (cm ? sp_minus : sp_plus) == best) {
                                if (cm) tm[k] |= 1u << b; else tp[k] |= 1u << b;
                            }
                        }
                    }
                    d += (int)((mA[k] >> b) & 1u) - (int)((mB[k] >> b) & 1u);
                }
            }
        }
        const uint32_t half = tw / 2;
        for (uint32_t k = 0; k < half; ++k) {
            uint64_t vp = 0, vm = 0;
#pragma unroll
            for (int kk = 0; kk < NQ / 2; ++kk)
                if ((uint32_t)kk == k) {
                    vp = (uint64_t)tp[2 * kk] | ((uint64_t)tp[2 * kk + 1] << 32);
                    vm = (uint64_t)tm[2 * kk] | ((uint64_t)tm[2 * kk + 1] << 32);
                }
            tiemask[(uint64_t)k * bv.stride + i] = vp;
            tiemask[(uint64_t)(half + k) * bv.stride + i] = vm;
        }
    }
}


// STAGE: the block stages the chromosome table and the super-coarse N map in LDS (8 + 8 KB)
// behind one barrier, so a window's N test and its chromosome cost no memory request (read-order
// batches over a large genome: every L2 request counts there).  Without STAGE both come from L2,
// which is cheaper when the batch is locus-ordered or the genome is cache-resident (the kernel is
// then VALU-bound and the staging's registers and barrier cost more than they save).
template <int NQ, bool NT, bool STAGE>
__global__ __launch_bounds__(kBlock) void bp_scan32_kernel(fc2_params p, fc2_genome_view g, fc2::ScanView bv,
                                                           uint64_t *__restrict__ out, uint64_t *__restrict__ tiemask,
                                                           uint32_t tw, int opts) {
    const bool swizzle = opts & fc2::kOptSwizzle;
    const uint64_t blk = swizzle ? xcd_block(blockIdx.x, gridDim.x) : (uint64_t)blockIdx.x;
    const uint64_t i = blk * kBlock + threadIdx.x;
    if constexpr (STAGE) {
        __shared__ uint64_t s_cstart[kChromLds];
        __shared__ int64_t s_csize[kChromLds];
        __shared__ __attribute__((aligned(16))) uint32_t s_nsuper_buf[kSuperLds];
        const bool lds_tab = !g.dummy && g.n_chrom <= (uint32_t)kChromLds;
        const bool lds_super = !g.dummy && g.nsuper && g.nsuper_words <= (uint32_t)kSuperLds;
        if (lds_super) {                       // 4 words per thread per pass, two passes (8 KB)
            uint4 q[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const uint32_t w = c * (kSuperLds / 2) + 4 * threadIdx.x;
                q[c] = uint4{0u, 0u, 0u, 0u}; // allocation is a multiple of 4 words (fc2_bp.h)
                if (w < g.nsuper_words) q[c] = *reinterpret_cast<const uint4 *>(g.nsuper + w);
            }
#pragma unroll
            for (int c = 0; c < 2; ++c)
                *reinterpret_cast<uint4 *>(s_nsuper_buf + c * (kSuperLds / 2) + 4 * threadIdx.x) = q[c];
        }
        if (lds_tab) {
            static_assert(kChromLds == 2 * kBlock, "two table entries per thread");
            const uint32_t k0 = threadIdx.x, k1 = threadIdx.x + kBlock;
            uint64_t a0 = 0, a1 = 0;
            int64_t z0 = 0, z1 = 0;
            if (k0 < g.n_chrom) { a0 = g.chrom_start[k0]; z0 = g.chrom_size[k0]; }
            if (k1 < g.n_chrom) { a1 = g.chrom_start[k1]; z1 = g.chrom_size[k1]; }
            s_cstart[k0] = a0; s_csize[k0] = z0;
            s_cstart[k1] = a1; s_csize[k1] = z1;
        }
        if (lds_tab || lds_super) __syncthreads();
        if constexpr (NQ == 4) {
            // cooperative unit loads need every window inside the genome arrays' reach: the dummy
            // genome has none (uniform branch)
            __shared__ ulonglong2 s_xchg[kBlock / 64][4 * 64];
            if (!g.dummy) {
                if (g.wt)          // word-pair layout present (fc2_wtab_launch): uniform branch
                    scan_pair<NQ, NT, true, true>(p, g, bv, out, tiemask, tw, i, s_cstart, s_csize, lds_tab,
                                                  lds_super ? s_nsuper_buf : nullptr, s_xchg[threadIdx.x >> 6]);
                else
                    scan_pair<NQ, NT, true>(p, g, bv, out, tiemask, tw, i, s_cstart, s_csize, lds_tab,
                                            lds_super ? s_nsuper_buf : nullptr, s_xchg[threadIdx.x >> 6]);
                return;
            }
        }
        scan_pair<NQ, NT, false>(p, g, bv, out, tiemask, tw, i, s_cstart, s_csize, lds_tab,
                                 lds_super ? s_nsuper_buf : nullptr, nullptr);
    } else {
        if constexpr (NQ == 4) {
            if (g.wt && !g.dummy) {   // word-pair layout present (uniform branch)
                scan_pair<NQ, NT, false, true>(p, g, bv, out, tiemask, tw, i, nullptr, nullptr, false, nullptr,
                                               nullptr);
                return;
            }
        }
        scan_pair<NQ, NT, false>(p, g, bv, out, tiemask, tw, i, nullptr, nullptr, false, nullptr, nullptr);
    }
}

// Window-carrying batches (fc2_batch_view.win_words): one pair per lane, windows streamed with
// the record -- the design BASELINE.json's north_star sketches (windows gathered on the host
// from the mmap'd FASTA).  No genome gather, no LDS.
template <int PW, bool NT>
__global__ __launch_bounds__(kBlock) void bp_scan32_win_kernel(fc2_params p, fc2_genome_view g, fc2::ScanView bv,
                                                               uint64_t *__restrict__ out,
                                                               uint64_t *__restrict__ tiemask, uint32_t tw) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    scan_pair<4, NT, false, false, PW>(p, g, bv, out, tiemask, tw, i, nullptr, nullptr, false, nullptr, nullptr);
}

// Device gather of the window rows from the resident genome (fc2_gather_windows_launch): the plain
// word-pair window path of the scan, written out instead of searched.
template <int PW>
__global__ __launch_bounds__(kBlock) void gather_windows_kernel(fc2_params p, fc2_genome_view g, uint64_t n,
                                                                uint64_t stride, fc2_pair *__restrict__ pairs,
                                                                uint64_t *__restrict__ win_words,
                                                                uint64_t *__restrict__ win_nwords) {
    constexpr uint32_t pw = PW;
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    fc2_pair pr = pairs[i];
    uint32_t w32[16], n32[8];
#pragma unroll
    for (int j = 0; j < 16; ++j) w32[j] = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) n32[j] = 0u;
    const int e = p.asize - p.margin;
    const int l = (int)pr.read_len - 2 * e;
    const int W = l + 2;
    bool anyN = false;
    if (!(pr.flags & (FC2_PAIR_SKIP | FC2_PAIR_BYTEPATH)) && l >= 0 && W <= 32 * (int)pw && pr.chrom < g.n_chrom) {
        const uint64_t cstart = g.chrom_start[pr.chrom];
        const int64_t csize = g.chrom_size[pr.chrom];
        const int64_t wsA = (int64_t)pr.a_pos + e, wsB = (int64_t)pr.b_aend - e - W;
        if (!(wsA > csize || wsA + W < 0 || wsB > csize || wsB + W < 0)) {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void *)g.wt, 0, (int)(uint32_t)g.wt_bytes, 0x00020000);
            const uint64_t nb = g.n_units * 8;
            const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
                (void *)g.nplane, 0, (int)(uint32_t)(nb > 0xFFFFFFFFull ? 0xFFFFFFFFull : nb), 0x00020000);
            WinW wA, wB;
            uint64_t cwA = 0, cwB = 0;
            window_issue_w_plain(g, rs, cstart, wsA, W, g.units_twin != nullptr, wA, cwA);
            window_issue_w_plain(g, rs, cstart, wsB, W, g.units_twin != nullptr, wB, cwB);
            window_nwords_plain(g, rn, cwA, wA);
            window_nwords_plain(g, rn, cwB, wB);
            P32<4> A, B;
            window_finish_w<4>(wA, csize, wsA, W, A);
            window_finish_w<4>(wB, csize, wsB, W, B);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t m = rmask32(0, W, k);
                if (k < (int)pw) {
                    w32[0 * pw + k] = A.lo[k] & m;
                    w32[1 * pw + k] = A.hi[k] & m;
                    w32[2 * pw + k] = B.lo[k] & m;
                    w32[3 * pw + k] = B.hi[k] & m;
                    n32[k] = A.n[k] & m;
                    n32[pw + k] = B.n[k] & m;
                    anyN |= (n32[k] | n32[pw + k]) != 0u;
                }
            }
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < 2 * pw; ++j)
        win_words[(uint64_t)j * stride + i] = (uint64_t)w32[2 * j] | ((uint64_t)w32[2 * j + 1] << 32);
#pragma unroll
    for (uint32_t j = 0; j < pw; ++j)
        win_nwords[(uint64_t)j * stride + i] = (uint64_t)n32[2 * j] | ((uint64_t)n32[2 * j + 1] << 32);
    const uint8_t f = (uint8_t)((pr.flags & ~FC2_PAIR_WIN_N) | (anyN ? FC2_PAIR_WIN_N : 0u));
    if (f != pr.flags) pairs[i].flags = f;
}

// The STAGE + cooperative word-pair form with BT-thread blocks (FC2_TUNE_STAGE_BLOCK): the LDS
// tables are staged once per BT pairs instead of once per 256 (each staging is ~60 L2 requests).
template <int BT, bool NT, int TRI>
__global__ __launch_bounds__(BT) void bp_scan32_stage_bt_kernel(fc2_params p, fc2_genome_view g, fc2::ScanView bv,
                                                                uint64_t *__restrict__ out,
                                                                uint64_t *__restrict__ tiemask, uint32_t tw) {
    __shared__ uint64_t s_cstart[kChromLds];
    __shared__ int64_t s_csize[kChromLds];
    __shared__ __attribute__((aligned(16))) uint32_t s_nsuper_buf[kSuperLds];
    __shared__ ulonglong2 s_xchg[BT / 64][4 * 64];
    // the launcher guarantees: genome not dummy, word-pair table, tables fit in LDS
    for (uint32_t w = 4 * threadIdx.x; w < (uint32_t)kSuperLds; w += 4 * BT) {
        uint4 q = uint4{0u, 0u, 0u, 0u};
        if (w < g.nsuper_words) q = *reinterpret_cast<const uint4 *>(g.nsuper + w);
        *reinterpret_cast<uint4 *>(s_nsuper_buf + w) = q;
    }
    for (uint32_t k = threadIdx.x; k < (uint32_t)kChromLds; k += BT) {
        const bool in = k < g.n_chrom;
        s_cstart[k] = in ? g.chrom_start[k] : 0ull;
        s_csize[k] = in ? g.chrom_size[k] : 0ll;
    }
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * BT + threadIdx.x;
    scan_pair<4, NT, true, true, 0, TRI>(p, g, bv, out, tiemask, tw, i, s_cstart, s_csize, true, s_nsuper_buf,
                                         s_xchg[threadIdx.x >> 6]);
}

#if FC2_AB_FORMS
// Persistent form of the STAGE + cooperative kernel (read-order batch over a large genome, l + 2
// <= 128): the grid is sized to the resident capacity of the chip, each block stages the LDS
// tables ONCE and then walks the batch's 256-pair tiles t = blockIdx.x + k * gridDim.x.  At
// 50M pairs that removes ~195k block dispatches, each followed by a 7.5 KB LDS fill from L2 and a
// barrier before the block's first window request.  The loop bound is uniform per block.
template <bool NT>
__global__ __launch_bounds__(kBlock) void bp_scan32_persist_kernel(fc2_params p, fc2_genome_view g,
                                                                   fc2::ScanView bv, uint64_t *__restrict__ out,
                                                                   uint64_t *__restrict__ tiemask, uint32_t tw,
                                                                   uint64_t n_tiles) {
    constexpr int NQ = 4;
    __shared__ uint64_t s_cstart[kChromLds];
    __shared__ int64_t s_csize[kChromLds];
    __shared__ __attribute__((aligned(16))) uint32_t s_nsuper_buf[kSuperLds];
    __shared__ ulonglong2 s_xchg[kBlock / 64][4 * 64];
    // the launcher guarantees: genome not dummy, chromosome table and nsuper fit in LDS
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const uint32_t w = c * (kSuperLds / 2) + 4 * threadIdx.x;
        uint4 q = uint4{0u, 0u, 0u, 0u};
        if (w < g.nsuper_words) q = *reinterpret_cast<const uint4 *>(g.nsuper + w);
        *reinterpret_cast<uint4 *>(s_nsuper_buf + c * (kSuperLds / 2) + 4 * threadIdx.x) = q;
    }
    {
        const uint32_t k0 = threadIdx.x, k1 = threadIdx.x + kBlock;
        uint64_t a0 = 0, a1 = 0;
        int64_t z0 = 0, z1 = 0;
        if (k0 < g.n_chrom) { a0 = g.chrom_start[k0]; z0 = g.chrom_size[k0]; }
        if (k1 < g.n_chrom) { a1 = g.chrom_start[k1]; z1 = g.chrom_size[k1]; }
        s_cstart[k0] = a0; s_csize[k0] = z0;
        s_cstart[k1] = a1; s_csize[k1] = z1;
    }
    __syncthreads();
    if (g.wt) {                 // word-pair windows (uniform branch)
        for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x)
            scan_pair<NQ, NT, true, true>(p, g, bv, out, tiemask, tw, t * kBlock + threadIdx.x, s_cstart, s_csize,
                                          true, s_nsuper_buf, s_xchg[threadIdx.x >> 6]);
    } else {
        for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x)
            scan_pair<NQ, NT, true, false>(p, g, bv, out, tiemask, tw, t * kBlock + threadIdx.x, s_cstart, s_csize,
                                           true, s_nsuper_buf, s_xchg[threadIdx.x >> 6]);
    }
}

#endif

// Speed-of-light probe of the read-order scan (measurement only, fc2_probe_pattern_launch): the
// kernel's exact memory pattern on the same batch and genome -- NT-streamed 16-B records and read
// rows, chromosome table staged in LDS, both windows' word pairs loaded by lane pairs from the same
// table offsets (main or shifted copy), 8-B result stored -- with none of the search's arithmetic
// and no N words (`tri`, windows > 97 bases: the three-lane 48-B loads).  Its time bounds what
// any kernel with this access pattern can reach on this GPU (bench.py: roofline.access_pattern_ceiling).
__global__ __launch_bounds__(kBlock) void probe_pattern_kernel(fc2_params p, fc2_genome_view g, fc2_batch_view bv,
                                                               uint64_t *__restrict__ out, int tri) {
    __shared__ uint64_t s_cstart[kChromLds];
    const bool lds_tab = g.n_chrom <= (uint32_t)kChromLds;
    if (lds_tab) {
        const uint32_t k0 = threadIdx.x, k1 = threadIdx.x + kBlock;
        s_cstart[k0] = k0 < g.n_chrom ? g.chrom_start[k0] : 0ull;
        s_cstart[k1] = k1 < g.n_chrom ? g.chrom_start[k1] : 0ull;
        __syncthreads();
    }
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool live = i < bv.n;
    u64x2 prv = {0ull, 0ull};
    uint64_t acc = 0;
    if (live) {
        prv = ld_pair_raw<true>(bv.pairs + i);
        for (uint32_t j = 0; j < bv.rw; ++j) acc += ld_stream<true>(bv.read_words + (uint64_t)j * bv.stride + i);
    }
    fc2_pair pr;
    __builtin_memcpy(&pr, &prv, sizeof pr);
    const int e = p.asize - p.margin;
    const int l = (int)pr.read_len - 2 * e;
    const bool active = live && l >= 0 && l <= 126 && pr.chrom < g.n_chrom;
    const int W = active ? l + 2 : 2;
    const uint32_t c = active ? pr.chrom : 0u;
    const uint64_t cstart = lds_tab ? s_cstart[c] : g.chrom_start[c];
    WinW wA, wB;
    window_geom_w(g, active ? cstart : 0, active ? (int64_t)pr.a_pos + e : 0, W, wA, tri);
    window_geom_w(g, active ? cstart : 0, active ? (int64_t)pr.b_aend - e - W : 0, W, wB, tri);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)g.wt, 0, (int)(uint32_t)g.wt_bytes,
                                                                         0x00020000);
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t offs[2] = {wA.off, wB.off};
    if (tri == 2) {                            // the five-lane form (windows_issue_w5): 40 B per window
#pragma unroll
        for (int c = 0; c < 11; ++c) {
            const int w = 12 * c + lane / 5;
            const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute((w & 63) << 2, (int)offs[0]);
            const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute((w & 63) << 2, (int)offs[1]);
            if (lane < 60 && w < 128) {
                const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, ((w >> 6) ? b : a) + 8u * (uint32_t)(lane % 5),
                                                                     0, 0);
                acc ^= (uint64_t)v.x | ((uint64_t)v.y << 32);
            }
        }
    } else if (tri) {                          // the scan's three-lane form (windows_issue_w3): 48 B per window
#pragma unroll
        for (int c = 0; c < 7; ++c) {
            const int w = 21 * c + lane / 3;
            const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute((w & 63) << 2, (int)offs[0]);
            const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute((w & 63) << 2, (int)offs[1]);
            if (lane < 63 && w < 128) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ((w >> 6) ? b : a) + 16u * (uint32_t)(lane % 3),
                                                                      0, 0);
                acc ^= (uint64_t)(v.x + v.y) | ((uint64_t)(v.z ^ v.w) << 32);
            }
        }
    } else {
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) {
                const uint32_t src = (uint32_t)__builtin_amdgcn_ds_bpermute((32 * cc + (lane >> 1)) << 2, (int)offs[x]);
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, src + 16u * (uint32_t)(lane & 1), 0, 0);
                acc ^= (uint64_t)(v.x + v.y) | ((uint64_t)(v.z ^ v.w) << 32);
            }
    }
    if (live) st_stream<true>(out + i, acc);
}

// ---------------------------------------------------------------------------------------------
// bp_wave_kernel: BASELINE.json north_star's kernel shape, run as a per-call form
// (FC2_BATCH_FORM_WAVE) so that DESIGN.md §4's choice of one pair per lane is measured against it
// rather than estimated.  ONE wavefront per anchor pair: a wave takes kWavePairs consecutive pairs,
// loads their records and read rows (round trip 1) and both genome windows of each -- the same
// 2-bit word pairs of g.wt as the staged form, one 128-B line per window, plus the N words of the
// windows the super map flags (round trip 2) -- cooperatively into LDS, then evaluates the pairs
// one after another with lane t on the positions x = t and x = t + 64 (find_circ.py:906-954):
// per-position mismatches of I against Af and Bf[x+2:], their wavefront prefix sums (a ballot and
// a popcount below the lane), the GT/AG - CT/AC masks, and a wavefront argmax of the score whose
// ties keep the stable-sort order (x ascending, '+' before '-', find_circ.py:961-974).  Every
// comparison uses the staged form's plane bits (low, high, N), so results are identical.
constexpr int kWavePairs = 16;         // pairs per wave, their loads in flight together
constexpr int kWaveSlot = 53;          // u32 of LDS per pair
// record at 0; read rows; read N rows; per window (A, B): lo, hi, n x 5; one pad word (the N-plane
// funnel's high word); the chromosome's start and size (2 x u64)
constexpr int kWsRead = 4, kWsReadN = 14, kWsWin = 18, kWsChrom = 49;

struct WaveGeo {
    uint64_t cstart;
    int64_t csize, ws[2];
    int l, W;
    bool ok, err;
};

// cstart / csize: the pair's chromosome (0, 0 when unknown), from g.chrom_start / chrom_size
__device__ __forceinline__ void wave_geo(const fc2_params &p, const fc2_genome_view &g, const fc2_pair &pr,
                                         uint64_t cstart, int64_t csize, WaveGeo &G) {
    const int e = p.asize - p.margin;
    G.l = (int)pr.read_len - 2 * e;
    G.W = G.l + 2;                             // flank, find_circ.py:900
    const bool known = pr.chrom < g.n_chrom;
    G.cstart = known ? cstart : 0ull;
    G.csize = known ? csize : 0;
    G.ws[0] = (int64_t)pr.a_pos + e;
    G.ws[1] = (int64_t)pr.b_aend - e - G.W;
    const bool bad = (pr.flags & FC2_PAIR_SKIP) || G.l < 0 || G.l > 126 || !known || G.ws[0] > G.csize ||
                     G.ws[0] + G.W < 0 || G.ws[1] > G.csize || G.ws[1] + G.W < 0;
    G.ok = !bad;
    G.err = bad && !(pr.flags & FC2_PAIR_SKIP) && G.l >= 0;   // as scan_pair: ERR_WIN
}

// may the window [cstart + ws, + W) touch an 'N'? (super map; without one, always load the N words)
__device__ __forceinline__ bool wave_nflag(const fc2_genome_view &g, uint64_t cstart, int64_t ws, int W) {
    const int64_t top = (int64_t)(g.n_units * 64) - 1;
    int64_t lo = (int64_t)cstart + ws, hi = lo + W - 1;
    lo = lo < 0 ? 0 : lo;
    hi = hi > top ? top : hi;
    if (lo > hi) return false;
    if (!g.nsuper) return true;
    const uint32_t k0 = (uint32_t)((uint64_t)lo >> g.nsuper_shift), k1 = (uint32_t)((uint64_t)hi >> g.nsuper_shift);
    return (((g.nsuper[k0 >> 5] >> (k0 & 31u)) | (g.nsuper[k1 >> 5] >> (k1 & 31u))) & 1u) != 0;
}

__device__ __forceinline__ fc2_pair wave_record(const uint32_t *P) {
    fc2_pair pr;
    __builtin_memcpy(&pr, P, sizeof pr);
    return pr;
}

__global__ __launch_bounds__(kBlock) void bp_wave_kernel(fc2_params p, fc2_genome_view g, fc2::ScanView bv,
                                                         uint64_t *__restrict__ out, uint64_t *__restrict__ tiemask,
                                                         uint32_t tw) {
    __shared__ uint32_t s_w[(kBlock / 64) * kWavePairs * kWaveSlot];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    uint32_t *S = s_w + wv * kWavePairs * kWaveSlot;
    const uint64_t i0 = ((uint64_t)blockIdx.x * (kBlock / 64) + wv) * kWavePairs;
    if (i0 >= bv.n) return;                    // the whole wave
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)g.wt, 0, (int)(uint32_t)g.wt_bytes,
                                                                         0x00020000);
    const uint64_t nb = g.n_units * 8;
    const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
        (void *)g.nplane, 0, (int)(uint32_t)(nb > 0xFFFFFFFFull ? 0xFFFFFFFFull : nb), 0x00020000);

    // round trip 1: records (slots 0 .. kWavePairs-1) and read rows (pair k, row j < 5) into LDS
    for (int s = lane; s < 6 * kWavePairs; s += 64) {
        if (s < kWavePairs) {
            u64x2 v = {0ull, 0ull};
            if (i0 + s < bv.n) v = ld_pair_raw<false>(bv.pairs + i0 + s);
            uint32_t *P = S + s * kWaveSlot;
            P[0] = (uint32_t)v.x; P[1] = (uint32_t)(v.x >> 32); P[2] = (uint32_t)v.y; P[3] = (uint32_t)(v.y >> 32);
        } else {
            const int t = s - kWavePairs, k = t / 5, j = t - 5 * k;
            uint64_t v = 0;
            if (i0 + k < bv.n && (uint32_t)j < bv.rw) v = bv.read_words[(uint64_t)j * bv.stride + i0 + k];
            S[k * kWaveSlot + kWsRead + 2 * j] = (uint32_t)v;
            S[k * kWaveSlot + kWsRead + 2 * j + 1] = (uint32_t)(v >> 32);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // round trip 2: both windows of every pair (slot: pair s / 10, window (s / 5) & 1, word pair
    // s % 5) with the N words of flagged windows, then the N rows of READ_N pairs
    for (int s = lane; s < 10 * kWavePairs; s += 64) {
        const int k = s / 10, x = (s / 5) & 1, j = s % 5;
        uint32_t *Q = S + k * kWaveSlot + kWsWin + 15 * x;
        uint32_t lo = 0, hi = 0, nn = 0;
        if (i0 + k < bv.n) {
            const fc2_pair pr = wave_record(S + k * kWaveSlot);
            const bool known = pr.chrom < g.n_chrom;
            const uint64_t cstart = known ? g.chrom_start[pr.chrom] : 0ull;
            const int64_t csize = known ? g.chrom_size[pr.chrom] : 0;
            if (s % 10 == 0) {                 // kept for the evaluation loop
                uint32_t *C = S + k * kWaveSlot + kWsChrom;
                C[0] = (uint32_t)cstart; C[1] = (uint32_t)(cstart >> 32);
                C[2] = (uint32_t)(uint64_t)csize; C[3] = (uint32_t)((uint64_t)csize >> 32);
            }
            WaveGeo G;
            wave_geo(p, g, pr, cstart, csize, G);
            if (G.ok && !(pr.flags & FC2_PAIR_BYTEPATH)) {
                WinW R;
                window_geom_w(g, G.cstart, G.ws[x], G.W, R);
                if (j < R.nwd) {
                    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, R.off + 8u * (uint32_t)j, 0, 0);
                    lo = v.x;
                    hi = v.y;
                    const int32_t w = (int32_t)R.q0 + j;
                    if (w >= 0 && wave_nflag(g, G.cstart, G.ws[x], G.W))
                        nn = __builtin_amdgcn_raw_buffer_load_b32(rn, (uint32_t)w * 4u, 0, 0);
                }
            }
        }
        Q[j] = lo;
        Q[5 + j] = hi;
        Q[10 + j] = nn;
    }
    for (int s = lane; s < 2 * kWavePairs; s += 64) {
        const int k = s >> 1, j = s & 1;
        uint64_t v = 0;
        if (i0 + k < bv.n) {
            const fc2_pair pr = wave_record(S + k * kWaveSlot);
            if ((pr.flags & (FC2_PAIR_READ_N | FC2_PAIR_READ_N1)) == FC2_PAIR_READ_N && bv.read_nwords &&
                (uint32_t)j < bv.nw)
                v = bv.read_nwords[(uint64_t)j * bv.stride + i0 + k];
        }
        S[k * kWaveSlot + kWsReadN + 2 * j] = (uint32_t)v;
        S[k * kWaveSlot + kWsReadN + 2 * j + 1] = (uint32_t)(v >> 32);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // evaluation, one pair at a time over the whole wave; lane t holds positions x = t, t + 64
    const bool want_ties = p.allhits != 0;
    const uint64_t lt = (1ull << lane) - 1ull;  // lanes below this one
    uint64_t myres = 0;
    bool mine = false;
    for (int k = 0; k < kWavePairs; ++k) {
        const uint64_t i = i0 + k;
        if (i >= bv.n) break;
        const uint32_t *P = S + k * kWaveSlot;
        // the pair's record and chromosome are the same for every lane: into SGPRs, so the
        // per-pair geometry runs on the scalar unit
        auto rfl = [](uint32_t v) -> uint32_t { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
        uint32_t rec[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) rec[j] = rfl(P[j]);
        fc2_pair pr;
        __builtin_memcpy(&pr, rec, sizeof pr);
        if (pr.flags & FC2_PAIR_BYTEPATH) {           // left for the byte-exact kernel
            if (bv.c_words && threadIdx.x % 64 == 0) mark_unscanned(bv, i);
            continue;
        }
        const uint32_t *C = P + kWsChrom;
        WaveGeo G;
        wave_geo(p, g, pr, (uint64_t)rfl(C[0]) | ((uint64_t)rfl(C[1]) << 32),
                 (int64_t)((uint64_t)rfl(C[2]) | ((uint64_t)rfl(C[3]) << 32)), G);
        uint64_t res;
        uint64_t tie[2][2] = {{0ull, 0ull}, {0ull, 0ull}};   // [strand][x / 64]
        if (!G.ok) {
            Best32 none;
            res = pack_result(none, 0, G.err ? FC2_RES_ERR_WIN : 0u);
        } else {
            const int l = G.l;
            const bool n1 = (pr.flags & (FC2_PAIR_READ_N | FC2_PAIR_READ_N1)) == (FC2_PAIR_READ_N | FC2_PAIR_READ_N1);
            const bool nrow = !n1 && (pr.flags & FC2_PAIR_READ_N);
            // per window (uniform): bit offset of position 0 in its first word pair, and the window
            // positions inside the chromosome, [vlo, vhi) (window_finish_w's masking), clamped
            int sh[2], vlo[2], vhi[2];
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                sh[w] = (int)(((int64_t)G.cstart + G.ws[w]) & 31);
                const int64_t a = -G.ws[w], z = G.csize - G.ws[w];
                vlo[w] = (int)(a < -256 ? -256 : (a > 256 ? 256 : a));
                vhi[w] = (int)(z < -256 ? -256 : (z > 256 ? 256 : z));
            }
            // per lane and h: window w's plane bits from position x_h on (bit j = position x_h + j),
            // positions outside the chromosome as 'N'
            uint32_t wlo[2][2], whi[2][2], wn[2][2];
            uint32_t ilo[2], ihi[2], inn[2];       // I[x_h] (bit 0)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int x = lane + 64 * h;
#pragma unroll
                for (int w = 0; w < 2; ++w) {
                    const int t = sh[w] + (x < 127 ? x : 127);
                    const int kw = t >> 5;
                    const unsigned sb = (unsigned)(t & 31);
                    const uint32_t *Q = P + kWsWin + 15 * w;
                    const uint32_t lo = alignr(Q[kw + 1], Q[kw], sb), hi = alignr(Q[kw + 6], Q[kw + 5], sb),
                                   nn = alignr(Q[kw + 11], Q[kw + 10], sb);
                    int v0 = vlo[w] - x, v1 = vhi[w] - x;          // valid j in [v0, v1)
                    v0 = v0 < 0 ? 0 : (v0 > 3 ? 3 : v0);
                    v1 = v1 < 0 ? 0 : (v1 > 3 ? 3 : v1);
                    const uint32_t vm = ((1u << v1) - 1u) & ~((1u << v0) - 1u);
                    wlo[h][w] = lo & vm;
                    whi[h][w] = hi & vm;
                    wn[h][w] = (nn & vm) | (7u & ~vm);
                }
                const int y = l + x;
                ilo[h] = (P[kWsRead + (x >> 5)] >> (x & 31)) & 1u;
                ihi[h] = (P[kWsRead + ((y >> 5) & 7)] >> (y & 31)) & 1u;
                inn[h] = n1 ? (x == (int)pr.npos ? 1u : 0u) : (nrow ? (P[kWsReadN + ((x >> 5) & 3)] >> (x & 31)) & 1u : 0u);
            }
            auto at = [&](int h, int w, int j) -> unsigned {   // plane bits of window w at position x_h + j
                return ((wlo[h][w] >> j) & 1u) | (((whi[h][w] >> j) & 1u) << 1) | (((wn[h][w] >> j) & 1u) << 2);
            };
            bool mA[2], mB[2], cp[2], cm[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int x = lane + 64 * h;
                // mismatches: A[x] vs I[x], B[x + 2] vs I[x] on all three planes
                const uint32_t dA = (wlo[h][0] ^ ilo[h]) | (whi[h][0] ^ ihi[h]) | (wn[h][0] ^ inn[h]);
                const uint32_t dB = (wlo[h][1] ^ (ilo[h] << 2)) | (whi[h][1] ^ (ihi[h] << 2)) | (wn[h][1] ^ (inn[h] << 2));
                mA[h] = x < l && (dA & 1u);
                mB[h] = x < l && (dB & 4u);
                // the staged form's masks: G = hi & ~lo, C = lo & ~hi, T = hi & lo (N bit ignored), A = no bit
                const uint32_t aT = whi[h][0] & wlo[h][0];
                const uint32_t bA = ~(wlo[h][1] | whi[h][1] | wn[h][1]);
                const uint32_t common = (aT >> 1) & bA;
                const uint32_t plus = (whi[h][0] & ~wlo[h][0]) & ((whi[h][1] & ~wlo[h][1]) >> 1) & common;
                const uint32_t minus = (wlo[h][0] & ~whi[h][0]) & ((wlo[h][1] & ~whi[h][1]) >> 1) & common;
                cp[h] = x <= l && (plus & 1u);
                cm[h] = x <= l && (minus & 1u);
            }
            // wavefront prefix sums of the mismatch flags
            const uint64_t bA0 = __ballot(mA[0]), bA1 = __ballot(mA[1]);
            const uint64_t bB0 = __ballot(mB[0]), bB1 = __ballot(mB[1]);
            const int totB = __popcll(bB0) + __popcll(bB1);
            int d[2];
            d[0] = __popcll(bA0 & lt) + totB - __popcll(bB0 & lt);
            d[1] = __popcll(bA0) + __popcll(bA1 & lt) + totB - __popcll(bB0) - __popcll(bB1 & lt);
            const int prim_minus = (pr.flags & FC2_PAIR_PRIMARY_REV) ? 1 : 0;
            const int sp_plus = p.strandpref ? (prim_minus ? 0 : 100) : 0;     // find_circ.py:796-797
            const int sp_minus = p.strandpref ? (prim_minus ? 100 : 0) : 0;
            bool hp[2], hm[2];
            int sp[2], sm[2];
            int best = INT32_MIN;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int x = lane + 64 * h;
                const bool q = x <= l && d[h] <= p.maxdist;
                const int ov = ov_of(x, l, p.margin);
                if (p.noncanonical) {
                    hp[h] = hm[h] = q;
                    sp[h] = 20 * (int)cp[h] - 10 * d[h] - ov + sp_plus;
                    sm[h] = 20 * (int)cm[h] - 10 * d[h] - ov + sp_minus;
                } else {
                    hp[h] = q && cp[h];
                    hm[h] = q && cm[h];
                    sp[h] = 20 - 10 * d[h] - ov + sp_plus;
                    sm[h] = 20 - 10 * d[h] - ov + sp_minus;
                }
                if (hp[h] && sp[h] > best) best = sp[h];
                if (hm[h] && sm[h] > best) best = sm[h];
            }
            const uint64_t hb[4] = {__ballot(hp[0]), __ballot(hp[1]), __ballot(hm[0]), __ballot(hm[1])};
            const int n_hits = __popcll(hb[0]) + __popcll(hb[1]) + __popcll(hb[2]) + __popcll(hb[3]);
            Best32 B;
            if (n_hits) {
                // wavefront argmax of the score
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const int v = __shfl_xor(best, o);
                    best = v > best ? v : best;
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    tie[0][h] = __ballot(hp[h] && sp[h] == best);
                    tie[1][h] = __ballot(hm[h] && sm[h] == best);
                }
                // first tie in stable-sort order: lowest x, '+' before '-'
                const int h = (tie[0][0] | tie[1][0]) ? 0 : 1;
                const uint64_t any = h ? (tie[0][1] | tie[1][1]) : (tie[0][0] | tie[1][0]);
                const int xl = __ffsll((unsigned long long)any) - 1;
                const int x = 64 * h + xl;
                B.n_hits = n_hits;
                B.best_score = best;
                B.best_x = x;
                B.best_minus = (((h ? tie[0][1] : tie[0][0]) >> xl) & 1ull) ? 0 : 1;
                B.best_dist = __shfl(h ? d[1] : d[0], xl);
                B.best_ov = ov_of(x, l, p.margin);
                B.n_ties = __popcll(tie[0][0]) + __popcll(tie[0][1]) + __popcll(tie[1][0]) + __popcll(tie[1][1]);
            }
            unsigned gtag12 = 0;
            if (B.n_hits) {
                if (!p.noncanonical) {
                    constexpr unsigned kGTAG = 2u | (3u << 3) | (0u << 6) | (2u << 9);
                    constexpr unsigned kCTAC = 1u | (3u << 3) | (0u << 6) | (1u << 9);
                    gtag12 = B.best_minus ? kCTAC : kGTAG;
                } else {
                    // the best x's four bases, from the lane that holds it
                    const int h = B.best_x >> 6, xl = B.best_x & 63;
                    auto code = [](unsigned v) -> unsigned { return (v & 4u) ? 4u : (v & 3u); };
                    const unsigned mine4 = code(at(h, 0, 0)) | (code(at(h, 0, 1)) << 3) | (code(at(h, 1, 0)) << 6) |
                                           (code(at(h, 1, 1)) << 9);
                    gtag12 = (unsigned)__shfl((int)mine4, xl);
                }
            }
            res = pack_result(B, gtag12, 0);
        }
        if (lane == k) { myres = res; mine = true; }
        if (want_ties && (uint32_t)lane < tw) {
            const uint32_t half = tw / 2, j = (uint32_t)lane;
            const uint32_t s = j < half ? 0u : 1u, w = j < half ? j : j - half;
            const uint64_t t0 = w ? tie[0][1] : tie[0][0], t1 = w ? tie[1][1] : tie[1][0];
            tiemask[(uint64_t)j * bv.stride + i] = w < 2 ? (s ? t1 : t0) : 0ull;
        }
    }
    if (mine) emit<false>(bv, out, i0 + lane, myres);
}

}  // namespace

namespace fc2 {

int launch_probe_pattern(hipStream_t s, const fc2_params &p, const fc2_genome_view &g, const fc2_batch_view &b,
                         uint64_t *out, int tri) {
    hipLaunchKernelGGL(probe_pattern_kernel, dim3((unsigned)((b.n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, p, g,
                       b, out, tri);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

void launch_scan32_win(int pw, bool nt, hipStream_t s, const fc2_params &p, const fc2_genome_view &g,
                       const ScanView &b, uint64_t *out, uint64_t *tiemask, uint32_t tw) {
    const unsigned grid = (unsigned)((b.n + kBlock - 1) / kBlock);
#if FC2_AB_FORMS
#define FC2_LW(PWV)                                                                                          \
    do {                                                                                                     \
        if (nt) hipLaunchKernelGGL((bp_scan32_win_kernel<PWV, true>), dim3(grid), dim3(kBlock), 0, s, p, g, b,  \
                                   out, tiemask, tw);                                                        \
        else hipLaunchKernelGGL((bp_scan32_win_kernel<PWV, false>), dim3(grid), dim3(kBlock), 0, s, p, g, b,    \
                                out, tiemask, tw);                                                           \
    } while (0)
#else
    (void)nt;
#define FC2_LW(PWV) hipLaunchKernelGGL((bp_scan32_win_kernel<PWV, true>), dim3(grid), dim3(kBlock), 0, s, p, g, b, \
                                       out, tiemask, tw)
#endif
    switch (pw) {
        case 1: FC2_LW(1); break;
        case 2: FC2_LW(2); break;
        case 3: FC2_LW(3); break;
        default: FC2_LW(4); break;
    }
#undef FC2_LW
}

void launch_gather_windows(hipStream_t s, const fc2_params &p, const fc2_genome_view &g, uint64_t n, uint64_t stride,
                           fc2_pair *pairs, uint64_t *win_words, uint64_t *win_nwords, uint32_t pw) {
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    switch (pw) {
        case 1: hipLaunchKernelGGL(gather_windows_kernel<1>, grid, dim3(kBlock), 0, s, p, g, n, stride, pairs, win_words,
                                   win_nwords); break;
        case 2: hipLaunchKernelGGL(gather_windows_kernel<2>, grid, dim3(kBlock), 0, s, p, g, n, stride, pairs, win_words,
                                   win_nwords); break;
        case 3: hipLaunchKernelGGL(gather_windows_kernel<3>, grid, dim3(kBlock), 0, s, p, g, n, stride, pairs, win_words,
                                   win_nwords); break;
        default: hipLaunchKernelGGL(gather_windows_kernel<4>, grid, dim3(kBlock), 0, s, p, g, n, stride, pairs,
                                    win_words, win_nwords); break;
    }
}

bool wave_ok(int ml, const fc2_genome_view &g) {
    return ml + 2 <= 128 && !g.dummy && g.wt && g.wt_bytes && g.chrom_start && g.chrom_size && g.nplane;
}

void launch_wave(hipStream_t s, const fc2_params &p, const fc2_genome_view &g, const ScanView &b, uint64_t *out,
                 uint64_t *tiemask, uint32_t tw) {
    constexpr uint64_t per_block = (kBlock / 64) * kWavePairs;
    hipLaunchKernelGGL(bp_wave_kernel, dim3((unsigned)((b.n + per_block - 1) / per_block)), dim3(kBlock), 0, s, p, g, b,
                       out, tiemask, tw);
}

bool stage_bt_ok(int nq, const fc2_genome_view &g) {
    return nq <= 4 && !g.dummy && g.wt && g.n_chrom <= (uint32_t)kChromLds && g.nsuper &&
           g.nsuper_words <= (uint32_t)kSuperLds;
}

void launch_scan32_stage_bt(int bt, int tri, bool nt, hipStream_t s, const fc2_params &p, const fc2_genome_view &g,
                            const ScanView &b, uint64_t *out, uint64_t *tiemask, uint32_t tw) {
#if FC2_AB_FORMS
#define FC2_LBT(BTV, TRV)                                                                                     \
    do {                                                                                                      \
        const dim3 grid((unsigned)((b.n + BTV - 1) / BTV));                                                   \
        if (nt) hipLaunchKernelGGL((bp_scan32_stage_bt_kernel<BTV, true, TRV>), grid, dim3(BTV), 0, s, p, g, b,  \
                                   out, tiemask, tw);                                                         \
        else hipLaunchKernelGGL((bp_scan32_stage_bt_kernel<BTV, false, TRV>), grid, dim3(BTV), 0, s, p, g, b,    \
                                out, tiemask, tw);                                                            \
    } while (0)
    if (tri == 2) {
        if (bt >= 1024) FC2_LBT(1024, 2);
        else if (bt >= 512) FC2_LBT(512, 2);
        else FC2_LBT(256, 2);
    } else if (tri) {
        if (bt >= 1024) FC2_LBT(1024, 1);
        else if (bt >= 512) FC2_LBT(512, 1);
        else FC2_LBT(256, 1);
    } else {
        if (bt >= 1024) FC2_LBT(1024, 0);
        else if (bt >= 512) FC2_LBT(512, 0);
        else FC2_LBT(256, 0);
    }
#undef FC2_LBT
#else
    (void)bt;
    (void)nt;
    const dim3 grid((unsigned)((b.n + 511) / 512));      // 512-pair blocks, non-temporal streaming
    if (tri == 2) hipLaunchKernelGGL((bp_scan32_stage_bt_kernel<512, true, 2>), grid, dim3(512), 0, s, p, g, b, out,
                                     tiemask, tw);
    else if (tri) hipLaunchKernelGGL((bp_scan32_stage_bt_kernel<512, true, 1>), grid, dim3(512), 0, s, p, g, b, out,
                                     tiemask, tw);
    else hipLaunchKernelGGL((bp_scan32_stage_bt_kernel<512, true, 0>), grid, dim3(512), 0, s, p, g, b, out,
                            tiemask, tw);
#endif
}

#if FC2_AB_FORMS
bool persist_ok(int nq, const fc2_genome_view &g) {
    return nq <= 4 && !g.dummy && g.n_chrom <= (uint32_t)kChromLds && g.nsuper &&
           g.nsuper_words <= (uint32_t)kSuperLds;
}

void launch_scan32_persist(bool nt, hipStream_t s, const fc2_params &p, const fc2_genome_view &g,
                           const ScanView &b, uint64_t *out, uint64_t *tiemask, uint32_t tw, int blocks_per_cu) {
    static int cus = 0, occ[2] = {0, 0};
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[0], bp_scan32_persist_kernel<false>, kBlock, 0) !=
            hipSuccess)
            occ[0] = 1;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[1], bp_scan32_persist_kernel<true>, kBlock, 0) !=
            hipSuccess)
            occ[1] = 1;
    }
    int per = blocks_per_cu > 0 ? blocks_per_cu : occ[nt ? 1 : 0];
    if (per <= 0) per = 1;
    const uint64_t n_tiles = (b.n + kBlock - 1) / kBlock;
    uint64_t grid = (uint64_t)cus * per;
    if (grid > n_tiles) grid = n_tiles;
    if (nt)
        hipLaunchKernelGGL(bp_scan32_persist_kernel<true>, dim3((unsigned)grid), dim3(kBlock), 0, s, p, g, b, out,
                           tiemask, tw, n_tiles);
    else
        hipLaunchKernelGGL(bp_scan32_persist_kernel<false>, dim3((unsigned)grid), dim3(kBlock), 0, s, p, g, b, out,
                           tiemask, tw, n_tiles);
}

#endif

void launch_scan32(int nq, bool nt, int opts, bool stage, unsigned grid, hipStream_t s, const fc2_params &p,
                   const fc2_genome_view &g, const ScanView &b, uint64_t *out, uint64_t *tiemask, uint32_t tw,
                   unsigned extra_lds) {
#define FC2_L32(NQV, NTV, STV)                                                                                   \
    hipLaunchKernelGGL((bp_scan32_kernel<NQV, NTV, STV>), dim3(grid), dim3(kBlock), extra_lds, s, p, g, b, out, tiemask, \
                       tw, opts)
#define FC2_L32S(NQV, NTV) do { if (stage) FC2_L32(NQV, NTV, true); else FC2_L32(NQV, NTV, false); } while (0)
#if FC2_AB_FORMS
    if (nq <= 4) { if (nt) FC2_L32S(4, true); else FC2_L32S(4, false); }
    else if (nq <= 8) { if (nt) FC2_L32S(8, true); else FC2_L32S(8, false); }
    else { if (nt) FC2_L32S(16, true); else FC2_L32S(16, false); }
#else
    (void)nt;
    if (nq <= 4) FC2_L32S(4, true);
    else if (nq <= 8) FC2_L32S(8, true);
    else FC2_L32S(16, true);
#endif
#undef FC2_L32S
#undef FC2_L32
}

}  // namespace fc2
