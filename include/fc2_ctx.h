/* fc2_ctx.h -- a per-device context over the breakpoint search: the torch-free form of the drop-in
 * boundary SURVEY.md §8(b) sketches (fc2_ctx_create / genome load / scan_async + sync / last error),
 * for hosts that bind the C ABI directly (cgo, JNI, N-API, ctypes without PyTorch).
 *
 * A context owns one HIP device and stream, the device-resident genome (the tables the Python layer
 * builds in find_circ2_amd/genome.py: 2-bit planes, N maps, the half-line twin, the LDS super map and
 * the word-pair layout), and page-locked staging plus device buffers for one batch of pairs, grown
 * as batches grow.  fc2_ctx_scan_async packs the batch on the host (fc2_pack_pairs, with the byte
 * path for pairs that need the FASTA bytes, fc2_bytepath_fill), copies it to the device, runs
 * fc2_bp_scan_launch / fc2_bp_scan_bytes_launch on the context's stream and copies the results back;
 * fc2_ctx_sync waits and hands them to the caller's buffers.  One batch is in flight per context; use
 * one context per device (any number of contexts, on any threads, may run at once).
 *
 * Reference: the call JunctionSpan.find_breakpoints() (find_circ.py:854-974) for every pair of the
 * batch, its windows fetched through Track.get -> GenomeAccessor.get_data -> indexed_fasta.get_data
 * (find_circ.py:310-312, 362-368, 189-215); the results are fc2_result words of include/fc2_bp.h.  There is no
 * CPU fallback: without a usable MI355X fc2_ctx_create fails with FC2_E_HIP.
 */
#ifndef FC2_CTX_H
#define FC2_CTX_H

#include "fc2_bp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fc2_ctx fc2_ctx;

/* A context on HIP device `device` (>= 0): its own non-blocking stream.  FC2_E_PARAM for a negative
 * device, FC2_E_HIP when the device cannot be used. */
int  fc2_ctx_create(int device, fc2_ctx **out);
/* A second context on src's device with its own stream and staging that scans against src's resident
 * genome (shared, not copied): two contexts per device keep one batch on the GPU while the host packs
 * the next.  src must outlive it and keep its genome (no fc2_ctx_genome_load on src meanwhile). */
int  fc2_ctx_create_sibling(const fc2_ctx *src, fc2_ctx **out);
/* Waits for the context's work, frees its device and pinned memory (the FASTA stays the caller's). */
void fc2_ctx_destroy(fc2_ctx *ctx);

/* The genome the scans read: fa (fc2_fasta_open) indexed, packed on the host and made resident on the
 * context's device with every table of fc2_genome_view.  fa must stay open while the context scans
 * (pairs on irregular FASTA layout or exotic bytes read their windows from it).  fa == NULL selects
 * the reference's dummy genome (no -G: every window all 'N', find_circ.py:340-345, 370-371).
 * Replaces a previously loaded genome.  The context keeps the host copy of the 2-bit planes it
 * uploaded (24 bytes per 64 bases, ~1.2 GB for hg19) until its genome is replaced or it is destroyed:
 * releasing them inside this call would hold the process's memory map while the caller waits. */
int  fc2_ctx_genome_load(fc2_ctx *ctx, const fc2_fasta *fa, int n_threads);
/* The resident genome as fc2_bp_scan_launch takes it (device pointers owned by the context). */
int  fc2_ctx_genome_view(const fc2_ctx *ctx, fc2_genome_view *out);

/* Queue the breakpoint search of n pairs: reads + read_off[i] holds pair i's read_part
 * (pairs[i].read_len bytes, find_circ.py:844); pairs[i] carries a_pos, b_aend, chrom (the genome's
 * chromosome index, fc2_fasta_find; 0xFFFFFFFF = not in the genome), read_len and flags
 * (FC2_PAIR_BACKSPLICE | FC2_PAIR_PRIMARY_REV | FC2_PAIR_SKIP).  Host packing runs in the call
 * (n_threads workers, 0 = automatic); the copies and kernels run on the context's stream.  results
 * (n words) and, with p->allhits, tiemask ([tw][n] words, tw >= the tie width fc2_batch_geometry
 * gives for the batch's longest read) are written at fc2_ctx_sync.  Input buffers may be reused once
 * the call returns.  FC2_E_PARAM while a previous batch has not been synced. */
int  fc2_ctx_scan_async(fc2_ctx *ctx, const fc2_params *p, uint64_t n, const uint8_t *reads,
                        const uint64_t *read_off, const fc2_pair *pairs, fc2_result *results,
                        uint64_t *tiemask, uint32_t tw, int n_threads);
/* Wait for the queued batch and write its results; FC2_OK when nothing is queued. */
int  fc2_ctx_sync(fc2_ctx *ctx);

/* The breakpoint search of n long pairs (read parts over FC2_MAX_READ_LEN, fc2_caller_batch.long_pairs;
 * read parts at reads + pairs[i].read_off), synchronously: results [n] and, with p->allhits, the tie
 * words (fc2_long_geometry's layout and length).  FC2_E_PARAM while a batch is queued. */
int  fc2_ctx_scan_long(fc2_ctx *ctx, const fc2_params *p, uint64_t n, const uint8_t *reads, const fc2_long_pair *pairs,
                       fc2_long_result *results, uint64_t *ties);

/* The context's hipStream_t (to order other work after or before its scans). */
void *fc2_ctx_stream(const fc2_ctx *ctx);
/* The last error a call on this context reported ("" if none); stays valid until the next call. */
const char *fc2_ctx_last_error(const fc2_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* FC2_CTX_H */
