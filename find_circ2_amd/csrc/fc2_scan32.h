// Launcher of the 32-bit-word breakpoint-search kernel (fc2_scan32.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fc2_bp.h"
#include "fc2_common.h"

namespace fc2 {
// What the scan kernels take: the caller's batch view plus, for fc2_bp_scan_compact_launch, where
// the scan's epilogue writes the compact result words (c_words == nullptr: 8-byte words to `out`).
struct ScanView : fc2_batch_view {
    void *c_words = nullptr;
    fc2_result_escape *c_esc = nullptr;
    uint32_t *c_count = nullptr;
    uint32_t c_cap = 0;
    int32_t c_width = 0;
    ScanView() = default;
    ScanView(const fc2_batch_view &v) : fc2_batch_view(v) {}   // NOLINT: implicit on purpose
};
// nq: 32-bit words per plane needed by the batch (rounded up to 4/8/16 inside); grid: one
// 256-pair tile per block; stage: the LDS-staging kernel variant (see bp_scan32_kernel);
// opts: kOptSwizzle.
constexpr int kOptSwizzle = 1;     // XCD-contiguous block order
void launch_scan32(int nq, bool nt, int opts, bool stage, unsigned grid, hipStream_t s, const fc2_params &p,
                   const fc2_genome_view &g, const ScanView &b, uint64_t *out, uint64_t *tiemask, uint32_t tw,
                   unsigned extra_lds = 0);   // occupancy experiments only (FC2_TUNE_EXTRA_LDS)
#if FC2_AB_FORMS
// Persistent STAGE + cooperative form (grid = CUs x resident blocks); usable when persist_ok().
// Measured and rejected (profiles/r01/ab_persist*.jsonl): A/B builds only.
bool persist_ok(int nq, const fc2_genome_view &g);
void launch_scan32_persist(bool nt, hipStream_t s, const fc2_params &p, const fc2_genome_view &g,
                           const ScanView &b, uint64_t *out, uint64_t *tiemask, uint32_t tw,
                           int blocks_per_cu);   // 0: the occupancy limit
#endif
// STAGE + cooperative word-pair form with bt-thread blocks (256/512/1024); usable when stage_bt_ok().
bool stage_bt_ok(int nq, const fc2_genome_view &g);
// tri: 0 = two-lane window loads, 1 = three-lane 16-B loads, 2 = five-lane 8-B loads (the default for
// batches with windows longer than 97 bases)
void launch_scan32_stage_bt(int bt, int tri, bool nt, hipStream_t s, const fc2_params &p, const fc2_genome_view &g,
                            const ScanView &b, uint64_t *out, uint64_t *tiemask, uint32_t tw);
// Window-carrying batches (b.win_words): PW = plane words, 1..4.
void launch_scan32_win(int pw, bool nt, hipStream_t s, const fc2_params &p, const fc2_genome_view &g,
                       const ScanView &b, uint64_t *out, uint64_t *tiemask, uint32_t tw);
void launch_gather_windows(hipStream_t s, const fc2_params &p, const fc2_genome_view &g, uint64_t n, uint64_t stride,
                           fc2_pair *pairs, uint64_t *win_words, uint64_t *win_nwords, uint32_t pw);
// BASELINE north_star's shape (one wavefront per pair, FC2_BATCH_FORM_WAVE); usable when wave_ok().
bool wave_ok(int ml, const fc2_genome_view &g);
void launch_wave(hipStream_t s, const fc2_params &p, const fc2_genome_view &g, const ScanView &b, uint64_t *out,
                 uint64_t *tiemask, uint32_t tw);
// Measurement kernel: the read-order scan's memory pattern without its arithmetic (needs g.wt).
int launch_probe_pattern(hipStream_t s, const fc2_params &p, const fc2_genome_view &g, const fc2_batch_view &b,
                         uint64_t *out, int tri);   // tri: the scan's window form, as above
}  // namespace fc2
