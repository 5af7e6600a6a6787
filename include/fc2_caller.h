/*
 * fc2_caller.h -- native find_circ read loop around the breakpoint search (libfc2.so).
 *
 * The per-fragment logic of find_circ.py 1.99 after the alignments are grouped
 * (include/fc2_ingest.h): anchor-pair formation (JunctionSpan, :821-852,
 * adjacent_segment_pairs :1058-1140, process_mate :1492-1527), the junction logic
 * of record_hits (:1276-1439), junction aggregation and naming (Hit /
 * SpliceSiteStorage, :486-730), MultiEventRecorder (:733-763), write_read
 * (:1442-1447) and the --test validator (:1148-1273), with Python-2 output
 * formatting.  find_circ2_amd/caller.py is the same logic in Python (kept as the
 * reference path: --python-caller); tests/test_native_caller.py checks both write
 * identical files.
 *
 * The breakpoint search stays outside: fc2_caller_next collects the anchor pairs
 * of up to `chunksize` fragments (the spans record_hits would evaluate) in the
 * layout fc2_pack_pairs takes; the caller evaluates them (fc2_bp_scan_launch) and
 * returns the raw per-pair results with fc2_caller_submit, which runs
 * record_hits for those fragments in input order.
 *
 * Errors the reference raises (KeyError at :927 / :193, undefined windows,
 * --stranded AttributeError, TypeError on reads without SEQ, ValueError for
 * unknown reference ids) end the run: the call returns FC2_E_FORMAT / FC2_E_KEY
 * and fc2_last_error() holds "ExceptionType: message".
 */
#ifndef FC2_CALLER_H
#define FC2_CALLER_H
#include <stdint.h>

#include "fc2_bp.h"
#include "fc2_ingest.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fc2_caller fc2_caller;

typedef struct fc2_caller_opts {     /* find_circ.py:383-413 */
    const char *name;                /* -n (tissue name) */
    const char *known_circ;          /* --known-circ BED6 path or NULL */
    const char *known_lin;           /* --known-lin BED6 path or NULL */
    int32_t min_uniq_qual, asize, margin, maxdist, short_threshold, huge_threshold;
    uint8_t noncanonical, allhits, stranded, strandpref, halfunique, report_nobridges, test, nolinear;
    uint8_t multi_events, noop, write_reads, write_multi;   /* write_*: that output file exists */
    uint32_t _pad;
    uint64_t chunksize;              /* fragments per evaluation batch */
} fc2_caller_opts;

/* Anchor pairs to evaluate (host memory, valid until the next call). pairs[i].chrom
 * is the genome chromosome index (tid_to_chrom of fc2_caller_open); pairs whose
 * chromosome is missing from the genome carry FC2_PAIR_SKIP and fail when
 * record_hits evaluates them.  Pairs whose read part is longer than FC2_MAX_READ_LEN
 * come in long_pairs instead (their read parts in the same `reads` buffer); their
 * results go back with fc2_caller_submit_long before the chunk's fc2_caller_submit. */
typedef struct fc2_caller_batch {
    uint64_t n;
    const uint8_t *reads;            /* read_part bytes (JunctionSpan.read_part, :844) */
    const uint64_t *read_off;        /* [n]; lengths are pairs[i].read_len */
    const fc2_pair *pairs;           /* [n] */
    uint64_t n_long;
    const fc2_long_pair *long_pairs; /* [n_long] */
} fc2_caller_batch;

/* path / is_bam as fc2_ingest_open.  tid_to_chrom [n_tid]: genome chromosome index
 * of each reference id of the alignment file, -1 if absent; fasta: the genome
 * FASTA (4-mers of --all-hits --non-canonical ties), NULL = dummy genome (all N).
 * *n_known_circ / *n_known_lin (may be NULL): known sites loaded. */
int  fc2_caller_open(const char *path, int is_bam, const fc2_caller_opts *opts, fc2_caller **out);
int  fc2_caller_set_genome(fc2_caller *h, const int32_t *tid_to_chrom, int32_t n_tid, const fc2_fasta *fasta,
                           uint64_t *n_known_circ, uint64_t *n_known_lin);
fc2_ingest *fc2_caller_ingest(fc2_caller *h);    /* reference names, header (NULL after the rows, below) */
/* BGZF blocks the input's GPU inflate took and left to the CPU (fc2_ingest_inflate_counts; kept
 * after the input is released). */
int fc2_caller_inflate_counts(const fc2_caller *h, uint64_t *gpu_blocks, uint64_t *cpu_blocks);
void fc2_caller_close(fc2_caller *h);

/* Read on until `chunksize` fragments carry pairs (or the input ends); *b = the pairs
 * to evaluate (n may be 0), *eof = 1 once the input is exhausted.  fc2_caller_next and
 * fc2_caller_submit may run concurrently on two threads (one caller of each): they share only
 * the chunk queue.  fc2_last_error() is per thread.  The chunk stays queued
 * (and *b valid) until fc2_caller_submit records it, so a caller may read ahead: form
 * chunk k+1 while chunk k is being searched (at most FC2_CALLER_MAX_QUEUED chunks).
 * Reading ahead changes nothing in the outputs, which submit writes in input order;
 * if next fails, the caller submits the chunks it holds first, then raises (the
 * reference reaches those fragments' record_hits before the failing one).  An input or
 * process_mate error met after some fragments of a chunk were formed ends that chunk there:
 * it is handed out as usual and the error is returned by the following call. */
#define FC2_CALLER_MAX_QUEUED 64
int fc2_caller_next(fc2_caller *h, fc2_caller_batch *b, int *eof);
/* Chunks handed out by fc2_caller_next and not yet submitted. */
int fc2_caller_queued(fc2_caller *h);
/* Results of the OLDEST queued batch, in its order: fc2_result [n] and, with --all-hits,
 * the tie mask [tw][stride] (x-major 64-bit words, '+' rows then '-' rows). */
int fc2_caller_submit(fc2_caller *h, const fc2_result *results, const uint64_t *tiemask, uint32_t tw,
                      uint64_t stride);
/* Results of the OLDEST queued batch's long pairs (fc2_bp_scan_long_launch), in their order:
 * results [n_long] and, with --all-hits, the tie words [tie words of fc2_long_geometry] (copied;
 * NULL without --all-hits).  Required before fc2_caller_submit(_compact) of a batch with long pairs. */
int fc2_caller_submit_long(fc2_caller *h, const fc2_long_result *results, uint64_t n_long, const uint64_t *ties,
                           uint64_t n_tie_words);
/* The same with the results in a compact transfer form (include/fc2_bp.h "compact results",
 * canonical mode, width 4 or 2 bytes): words [n_words] and the n_esc escapes (indices into this
 * batch), expanded here.  FC2_E_PARAM unless n_words is the oldest queued batch's pair count. */
int fc2_caller_submit_compact(fc2_caller *h, const void *words, int width, uint64_t n_words,
                              const fc2_result_escape *esc, uint64_t n_esc, const uint64_t *tiemask, uint32_t tw,
                              uint64_t stride);

/* Output text produced since the last call: 0 = spliced_reads.fastq, 1 =
 * multi_events.tsv rows, 2 = test_results.tsv rows. */
int fc2_caller_take(fc2_caller *h, int stream, const char **text, uint64_t *len);
/* Write spliced_reads.fastq.gz here instead (find_circ.py:445): the text of stream 0 is cut into
 * pieces of `piece` bytes (0: 4 MiB), each compressed at `level` as its own gzip member on
 * `threads` worker threads and written in order (one valid gzip stream); stream 0 of
 * fc2_caller_take then stays empty.  Call before the first fc2_caller_submit. */
int fc2_caller_set_reads_gz(fc2_caller *h, const char *path, int level, int threads, uint64_t piece);
/* Compress and write what is left and close the file (also done, errors ignored, by
 * fc2_caller_close); FC2_E_IO if a write failed. */
int fc2_caller_close_reads(fc2_caller *h);
/* The BED rows (no header) of 0 = circ_splice_sites.bed, 1 = lin_splice_sites.bed
 * (call once, at the end).  Once the input was read to its end and every chunk submitted, the first
 * call releases the read side -- the input (so finish -B output with fc2_ingest_close_bam_out
 * before), its parse blocks, the chunk buffers -- on a thread of its own: fc2_caller_ingest returns
 * NULL from then on, fc2_caller_next reports the end, the counters keep their final values. */
int fc2_caller_rows(fc2_caller *h, int kind, const char **text, uint64_t *len);
/* The same rows written to the file descriptor fd at its current offset (the CLI's BED files; the
 * ranges are formatted on the workers and written in order as each is done, never joined in memory);
 * *len (may be NULL) = bytes written.  FC2_E_IO if a write failed.  Call once per kind, instead of
 * fc2_caller_rows. */
int fc2_caller_write_rows(fc2_caller *h, int kind, int fd, uint64_t *len);
/* The reference's N[...] counters in sorted key order: i-th name and value;
 * FC2_E_RANGE past the end. */
int fc2_caller_counter(fc2_caller *h, int i, const char **name, double *value);
/* fragments read (n_reads) and anchor pairs evaluated so far, as of the last fc2_caller_next to
 * return (safe to call from a thread other than the one calling fc2_caller_next). */
int fc2_caller_stats(fc2_caller *h, uint64_t *n_reads, uint64_t *n_pairs);

#ifdef __cplusplus
}
#endif
#endif /* FC2_CALLER_H */
