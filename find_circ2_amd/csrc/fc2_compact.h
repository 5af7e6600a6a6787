// The 4- and 2-byte transfer forms of fc2_result (include/fc2_bp.h, "compact results"): shared by
// the device kernel that packs a batch's results and the host code that expands them.
//
// Canonical mode only: there a hit's signal is implied by its strand -- 'GTAG' for '+' and 'CTAC'
// for '-' (find_circ.py:924-954) -- so the 12 gtag bits need not travel.  A word that does not
// survive pack -> unpack unchanged (4 B: x > 254, n_ties > 255, dist or ov > 15, ...; 2 B: x > 125,
// n_ties > 16, dist or ov > 3, any error bit) travels whole in the escape list instead.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fc2_bp.h"

namespace fc2 {

// gtag codes of the two canonical signals (A0 C1 G2 T3, first base lowest)
constexpr unsigned kGtagGTAG = 2u | (3u << 3) | (0u << 6) | (2u << 9);
constexpr unsigned kGtagCTAC = 1u | (3u << 3) | (0u << 6) | (1u << 9);

__host__ __device__ inline uint32_t r32_pack(uint64_t w) {
    const int16_t x = (int16_t)(uint16_t)(w & 0xFFFF);
    const unsigned dist = (unsigned)(w >> 16) & 0xFF, ov = (unsigned)(w >> 24) & 0xFF;
    const unsigned nt = (unsigned)(w >> 32) & 0xFFFF, info = (unsigned)(w >> 48) & 0xFFFF;
    return (uint32_t)((unsigned)(x + 1) & 0xFF) | ((nt & 0xFF) << 8) | ((dist & 0xF) << 16) | ((ov & 0xF) << 20) |
           ((info & FC2_RES_MINUS) ? (1u << 24) : 0u) | ((info & FC2_RES_ERR_KEY) ? (1u << 25) : 0u) |
           ((info & FC2_RES_ERR_WIN) ? (1u << 26) : 0u) | ((info & FC2_RES_DONE) ? (1u << 27) : 0u);
}

// branch-free, so the host's expansion loop vectorizes
__host__ __device__ inline uint64_t r32_unpack(uint32_t c) {
    const uint64_t x1 = c & 0xFFu;
    const uint64_t minus = (c >> 24) & 1u;
    const uint64_t errs = (uint64_t)((c >> 25) & 7u) << 13;          // ERR_KEY, ERR_WIN, DONE
    const uint64_t gtag = minus ? (uint64_t)kGtagCTAC : (uint64_t)kGtagGTAG;
    const uint64_t hit = ((x1 - 1) & 0xFFFFu) | ((uint64_t)((c >> 16) & 0xFu) << 16) |
                         ((uint64_t)((c >> 20) & 0xFu) << 24) | ((uint64_t)((c >> 8) & 0xFFu) << 32) |
                         ((errs | minus | (gtag << FC2_RES_GTAG_SHIFT)) << 48);
    const uint64_t miss = 0xFFFFu | (errs << 48);
    return x1 ? hit : miss;
}

// 2 bytes: bits 0-6 x + 1 (0: no hit, 0x7F: escaped), 7 '-', 8-9 dist, 10-11 ov, 12-15 n_ties - 1;
// no error bits (a flagged pair escapes), FC2_RES_DONE implied
constexpr uint16_t kR16Escape = 0x007Fu;

__host__ __device__ inline uint16_t r16_pack(uint64_t w) {
    const int16_t x = (int16_t)(uint16_t)(w & 0xFFFF);
    const unsigned dist = (unsigned)(w >> 16) & 0xFF, ov = (unsigned)(w >> 24) & 0xFF;
    const unsigned nt = (unsigned)(w >> 32) & 0xFFFF, info = (unsigned)(w >> 48) & 0xFFFF;
    if (x < 0) return 0;
    return (uint16_t)(((unsigned)(x + 1) & 0x7Fu) | ((info & FC2_RES_MINUS) ? 0x80u : 0u) | ((dist & 3u) << 8) |
                      ((ov & 3u) << 10) | (((nt - 1u) & 15u) << 12));
}

__host__ __device__ inline uint64_t r16_unpack(uint16_t c) {
    const uint64_t x1 = c & 0x7Fu;
    const uint64_t minus = (c >> 7) & 1u;
    const uint64_t gtag = minus ? (uint64_t)kGtagCTAC : (uint64_t)kGtagGTAG;
    const uint64_t hit = ((x1 - 1) & 0xFFFFu) | ((uint64_t)((c >> 8) & 3u) << 16) | ((uint64_t)((c >> 10) & 3u) << 24) |
                         ((uint64_t)(((c >> 12) & 15u) + 1u) << 32) |
                         (((uint64_t)FC2_RES_DONE | minus | (gtag << FC2_RES_GTAG_SHIFT)) << 48);
    const uint64_t miss = 0xFFFFu | ((uint64_t)FC2_RES_DONE << 48);
    return x1 ? hit : miss;
}

// the word a result travels as in `width` bytes and whether it must escape instead
__host__ __device__ inline uint32_t compact_pack(uint64_t w, int width, bool &escape) {
    if (width == 2) {
        const uint16_t c = r16_pack(w);
        escape = (c & 0x7Fu) == kR16Escape || r16_unpack(c) != w;
        return escape ? kR16Escape : c;
    }
    const uint32_t c = r32_pack(w);
    escape = r32_unpack(c) != w;
    return escape ? FC2_R32_ESCAPE : c;
}

}  // namespace fc2
