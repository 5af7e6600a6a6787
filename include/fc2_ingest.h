/*
 * fc2_ingest.h -- native SAM/BAM ingest for the find_circ2 caller (libfc2.so).
 *
 * Replaces the per-record Python work of find_circ.py's read loop
 * (pysam iteration find_circ.py:461-469, collected_bwa_mem_segments
 * :1450-1486, MateSegments :976-1140, process_mate :1492-1527) for the records
 * that never reach the breakpoint search: every record is parsed and grouped
 * into fragments (mate pairs / single reads) here, adjacent segment pairs are
 * formed with the reference's rules, and only fragments that carry at least
 * one anchor pair are handed back (as SAM text) for the per-fragment logic.
 * Counters the reference keeps for the others are accumulated here.
 *
 * Reads a path or "-" (stdin).  The format is detected from the bytes, never
 * from the file name, as htslib's hts_open does for the reference's
 * pysam.Samfile(path | '-', 'r' | 'rb') (find_circ.py:461-469): the byte source
 * is plain, BGZF (parallel block inflate) or any other gzip stream, and what it
 * holds is BAM ("BAM\1") or SAM text.  CRAM is rejected (FC2_E_FORMAT).
 */
#ifndef FC2_INGEST_H
#define FC2_INGEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fc2_ingest fc2_ingest;

typedef struct fc2_ingest_params {
    int32_t asize;      /* -a: minimal segment length of an anchor (find_circ.py:1125) */
    uint8_t nolinear;   /* --no-linear: fragments without backsplice spans are skipped (:1568-1569) */
    uint8_t noop;       /* --noop: count reads only (:1554-1558) */
    uint8_t _pad[2];
} fc2_ingest_params;

typedef struct fc2_ingest_counts {  /* cumulative since open (the reference's N[...] keys) */
    uint64_t n_reads;               /* fragments yielded (n_reads, :1536) */
    uint64_t total_mates;           /* N['total_mates'] (:978) */
    uint64_t unmapped_reads;        /* N['unmapped_reads'] (:1467) */
    uint64_t unspliced_mates;       /* N['unspliced_mates'] of skipped fragments (:1494) */
    uint64_t seg_too_short_skip;    /* N['seg_too_short_skip'] of skipped fragments (:1127) */
    uint64_t records;               /* alignment records read */
    uint64_t handed_back;           /* fragments returned to the caller */
} fc2_ingest_counts;

/* path "-" reads stdin.  is_bam is the reference's mode hint ('rb' unless the name ends in
 * "sam", find_circ.py:463-466) and, as in htslib, does not decide anything: a BAM named x.sam,
 * SAM named x.bam, bgzip'ed or gzip'ed SAM and BAM on stdin are all read by what they are. */
int  fc2_ingest_open(const char *path, int is_bam, fc2_ingest **out);

/* What fc2_ingest_open found: FC2_INGEST_SAM or FC2_INGEST_BAM (-1 for a null handle);
 * *compression (optional) = FC2_INGEST_PLAIN / _BGZF / _GZIP. */
enum { FC2_INGEST_SAM = 0, FC2_INGEST_BAM = 1 };
enum { FC2_INGEST_PLAIN = 0, FC2_INGEST_BGZF = 1, FC2_INGEST_GZIP = 2 };
int  fc2_ingest_format(const fc2_ingest *h, int *compression);
void fc2_ingest_close(fc2_ingest *h);
int  fc2_ingest_n_refs(const fc2_ingest *h);
const char *fc2_ingest_ref_name(const fc2_ingest *h, int tid);
/* SAM header text (one line per @ record). */
const char *fc2_ingest_header(const fc2_ingest *h);

/* Process up to max_frags fragments.  *text / *text_len: SAM lines of the
 * returned fragments, each fragment's records consecutive and followed by an
 * empty line; valid until the next call.  *n_handed: fragments in *text.
 * *eof = 1 when the input is exhausted.  Returns FC2_OK or a negative status
 * (FC2_E_FORMAT for malformed input; the reference's UnboundLocalError on
 * single-record input is FC2_E_FORMAT with that message).  An error met after some fragments
 * of the call were formed is returned by the following call, after those fragments. */
int fc2_ingest_next(fc2_ingest *h, const fc2_ingest_params *p, uint64_t max_frags, fc2_ingest_counts *counts,
                    const char **text, uint64_t *text_len, uint64_t *n_handed, int *eof);

/* Counters so far (also returned by fc2_ingest_next). */
int fc2_ingest_counts_get(const fc2_ingest *h, fc2_ingest_counts *counts);

/* -B/--bam (replaces pysam.Samfile(spliced_alignments.bam, 'wb', template=sam_input) and
 * bam_out.write(seg) in adjacent_segment_pairs, find_circ.py:479-483, 1134-1140): every
 * processed mate's anchor alignments go to a BGZF BAM with the input's header, in the
 * reference's order.  BAM input records are copied byte for byte; SAM lines are encoded as
 * htslib's sam_parse1 does.  Call once, before the first fc2_ingest_next; the file is
 * finished (EOF block) by fc2_ingest_close_bam_out or fc2_ingest_close. */
int fc2_ingest_set_bam_out(fc2_ingest *h, const char *path);
int fc2_ingest_close_bam_out(fc2_ingest *h);

/* ``samtools view -b`` for SAM text (any compression): every record encoded as htslib's
 * sam_parse1 does (the -B encoder above), BGZF blocks (zlib level 1, as samtools view -1) + EOF block.  Used to make BAM inputs for
 * tests and the bench's stdin-BAM CLI run. */
int fc2_sam_to_bam(const char *sam_path, const char *bam_path);
/* The BAM input's BGZF blocks inflated on GPU `device` (fc2_inflate.hip) instead of the CPU from the
 * next batch on; call before reading (FC2_GPU_INFLATE=1 or 2 makes the CLI's read loop call this, on
 * its first device; by default it calls fc2_ingest_set_gpu_inflate_from below).  The device's
 * buffers are made now (wait != 0) or meanwhile, the batches inflated on the CPU until they are ready.
 * Batches grow to 1024 blocks (FC2_BGZF_BATCH still sets them); every block's CRC-32 and ISIZE are
 * checked (on the device), and the CPU inflates any block the GPU refused, and every block from then
 * on if the device fails.  device < 0, a non-BGZF input or FC2_GPU_INFLATE=0: the CPU inflates. */
int fc2_ingest_set_gpu_inflate(fc2_ingest *h, int device, int wait);
/* The same, with nothing made on the device until after_bytes of the input were read (0: as
 * fc2_ingest_set_gpu_inflate(h, device, 0)): smaller inputs never touch the device, and their batches
 * keep the ingest's size.  The CLI's default, with 256 MiB (DESIGN.md §5 "The BAM input inflated on the
 * GPU").  FC2_GPU_INFLATE=0 turns it off, 1 or 2 start it at once. */
int fc2_ingest_set_gpu_inflate_from(fc2_ingest *h, int device, uint64_t after_bytes);
/* Blocks of the batches the GPU inflated: those it took, and those it left to the CPU. */
int fc2_ingest_inflate_counts(const fc2_ingest *h, uint64_t *gpu_blocks, uint64_t *cpu_blocks);
/* BGZF blocks inflated on the GPU (fc2_inflate.hip; the BAM input's inflate, which pysam/htslib does for
 * the reference, find_circ.py:461-469): n blocks, block i = len[i] bytes of raw DEFLATE at src + off[i]
 * (device memory, readable 8 bytes past every payload: a BGZF block's trailer) holding isize[i] <= 65536
 * bytes, inflated into dst + i * 65536 and, when crc is not NULL, checked against crc[i] (the gzip
 * CRC-32); status[i] = 0, or why the block was refused (the host then inflates it on the CPU). */
int fc2_bgzf_inflate_launch(const uint8_t *src, const uint32_t *off, const uint32_t *len, const uint32_t *isize,
                            const uint32_t *crc, uint8_t *dst, uint32_t *status, uint32_t n, void *stream);
#ifdef __cplusplus
}
#endif
#endif /* FC2_INGEST_H */
