/*
 * fc2_bp.h -- C ABI of the MI355X breakpoint-search library (libfc2.so).
 *
 * Drop-in boundary for ONE hot path of find_circ2 (find_circ.py 1.99):
 *
 *   JunctionSpan.find_breakpoints(self) -> [Splice]   find_circ.py:854-974
 *     + its genome window fetch  Track.get -> GenomeAccessor.get_data ->
 *       indexed_fasta.get_data                         find_circ.py:310-312, 362-368, 189-215
 *
 * The reference has no FFI: the path is a Python method called from
 * record_hits (find_circ.py:1303 circ spans, 1355 linear spans).  This header
 * is what a ctypes binding of that method binds; the
 * Python host layer find_circ2_amd/hotpath.py mirrors the method itself.
 *
 * Conventions
 *  - plain C types, no torch types; every function returns an int status
 *    (FC2_OK = 0, negative = error class) and never throws;
 *    fc2_last_error() gives the message of the last failure on this thread.
 *  - device pointers are HIP device pointers owned by the caller (the Python
 *    layer allocates them as torch tensors); `stream` is a hipStream_t.
 *    fc2_*_launch functions are asynchronous on that stream.
 *  - host pointers are ordinary host memory owned by the caller.
 *  - reference errors that are fatal in find_circ.py (KeyError at :927 and
 *    :193, undefined windows at :194-211) are reported per pair in
 *    fc2_result.info, never silently dropped.
 */
#ifndef FC2_BP_H
#define FC2_BP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FC2_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------ */
#define FC2_OK        0
#define FC2_E_PARAM  -1   /* invalid argument / unsupported option value          */
#define FC2_E_HIP    -2   /* HIP runtime error (message via fc2_last_error)       */
#define FC2_E_FORMAT -3   /* malformed FASTA / index                               */
#define FC2_E_RANGE  -4   /* value outside the supported range                     */
#define FC2_E_IO     -5   /* IOError class: the file cannot be opened or read (the reference's
                             file()/open() raises IOError; GenomeAccessor then switches to its
                             all-N dummy mode, find_circ.py:338-345)                         */
#define FC2_E_KEY    -6   /* unknown chromosome (reference KeyError, find_circ.py:193) */
#define FC2_E_OS     -7   /* OS error the reference does not catch (mmap.error, OSError from
                             writing the .byo_index, find_circ.py:118, 157-179)             */

/* ---- options the hot path reads (find_circ.py:393-404) ----------------- */
typedef struct fc2_params {
    int32_t asize;        /* -a/--anchor      (default 15)  find_circ.py:394 */
    int32_t margin;       /* -m/--margin      (default 2)   find_circ.py:395 */
    int32_t maxdist;      /* -d/--max-mismatch(default 2)   find_circ.py:396 */
    uint8_t noncanonical; /* --non-canonical                find_circ.py:401 */
    uint8_t strandpref;   /* --strand-pref                  find_circ.py:404 */
    uint8_t allhits;      /* --all-hits                     find_circ.py:402 */
    uint8_t _pad;
} fc2_params;

/* ---- one anchor pair (a JunctionSpan, find_circ.py:821-852), 16 bytes ---- */
#define FC2_PAIR_BACKSPLICE  0x01u  /* align_B.pos - align_A.aend < 0   (:842, :851) */
#define FC2_PAIR_PRIMARY_REV 0x02u  /* primary.is_reverse -> span strand '-' (:834) */
#define FC2_PAIR_READ_N      0x04u  /* internal read part has 'N' bytes: N plane present */
#define FC2_PAIR_BYTEPATH    0x08u  /* evaluated by the byte-exact kernel (exotic bytes,
                                       irregular FASTA line layout, very long reads) */
#define FC2_PAIR_SKIP        0x10u  /* not evaluated (e.g. not is_uniq, :1299): no hit */
#define FC2_PAIR_WIN_N       0x20u  /* window-carrying batch: this pair's window N rows are present */
#define FC2_PAIR_READ_N1     0x40u  /* with READ_N: the read part holds exactly ONE 'N', at position npos
                                       (< 256); the scan then skips the N row (which is filled all the same) */

typedef struct fc2_pair {
    int32_t  a_pos;     /* align_A.pos  (0-based)                                    */
    int32_t  b_aend;    /* align_B.aend (exclusive)                                  */
    uint32_t chrom;     /* index into the genome's chromosome table                  */
    uint16_t read_len;  /* L = len(read_part)                                        */
    uint8_t  flags;     /* FC2_PAIR_*                                                */
    uint8_t  npos;      /* FC2_PAIR_READ_N1: position of the read part's single 'N'; else 0 */
} fc2_pair;

/* Longest read_part of a batch pair (fc2_pack_pairs fails with FC2_E_RANGE above it): every
 * breakpoint index x <= l < 2^15 fits fc2_result.best_x, and the at most 2(l+1) ties of
 * --non-canonical fit n_ties.  Longer read parts -- the reference's x-loop has no limit
 * (find_circ.py:873, :904-906) -- travel as fc2_long_pair records, below. */
#define FC2_MAX_READ_LEN 32767

/* ---- per-pair result, 8 bytes ------------------------------------------- */
/* best_x = breakpoint index x of ties[0] (the Splice record_hits keeps,
 * find_circ.py:1312-1317), -1 if find_breakpoints returned [].
 * n_ties = Splice.n_hits of the returned ties (1 if a single hit).
 * Coordinates follow from x (find_circ.py:929-945):
 *   s0 = b_aend - e - l + x,  e0 = a_pos + e + x + 1,  e = asize - margin,  l = L - 2e
 *   (start, end) = (min, max); backsplice: end -= 1, else start -= 1.          */
#define FC2_RES_MINUS       0x0001u  /* strand of ties[0] is '-'                        */
#define FC2_RES_GTAG_SHIFT  1        /* 4 x 3-bit base codes of gtag = A[x]A[x+1]B[x]B[x+1]
                                        (A0 C1 G2 T3 N4), first base in the lowest bits;
                                        a '-' Splice's signal is rev_comp(gtag)           */
#define FC2_RES_GTAG_MASK   0x1FFEu
#define FC2_RES_ERR_KEY     0x2000u  /* reference raises KeyError (find_circ.py:927)    */
#define FC2_RES_ERR_WIN     0x4000u  /* window outside the range where get_data is defined
                                        (find_circ.py:194-211); reference output undefined */
#define FC2_RES_DONE        0x8000u  /* written by a kernel                               */

typedef struct fc2_result {
    int16_t  best_x;
    uint8_t  dist;      /* mismatches of ties[0]  (Splice.dist)  */
    uint8_t  ov;        /* anchor overlap of ties[0] (Splice.ov) */
    uint16_t n_ties;
    uint16_t info;      /* FC2_RES_*                              */
} fc2_result;

/* ---- compact results: the 4- and 2-byte transfer forms ------------------------ */
/* What moves a batch's results off the device in bulk (the ordered merge of a strong-scaled
 * stream, find_circ.py:681-690 naming + :544/:563/:579 weight sums in input order) at `width` = 4
 * or 2 bytes per pair instead of 8.  Canonical mode only (no --non-canonical): a hit's signal is
 * implied by its strand ('+' GTAG, '-' CTAC, :924-954), and FC2_RES_DONE is implied.
 *   width 4, uint32 words[i] = bits 0-7 best_x + 1 (0: no hit) | 8-15 n_ties | 16-19 dist |
 *     20-23 ov | 24 '-' | 25 FC2_RES_ERR_KEY | 26 FC2_RES_ERR_WIN | 27 FC2_RES_DONE | 31 escape.
 *   width 2, uint16 words[i] = bits 0-6 best_x + 1 (0: no hit, 0x7F: escape) | 7 '-' |
 *     8-9 dist | 10-11 ov | 12-15 n_ties - 1; a result with an error bit escapes.
 * A result that would not come back unchanged (too large a field, an error bit in the 2-byte form,
 * ...) gets the escape word and travels whole as an escape (its index, its fc2_result), in no
 * particular order.  *esc_count (device) is zeroed by the launch and counts every escape; only
 * the first esc_cap are stored: a count above esc_cap means the caller must move the 8-byte
 * results instead. */
#define FC2_R32_ESCAPE 0x80000000u
#define FC2_R16_ESCAPE 0x007Fu
typedef struct fc2_result_escape {
    uint64_t   index;
    fc2_result result;
} fc2_result_escape;
int fc2_result_compact_launch(const fc2_params *p, const fc2_result *results, uint64_t n, int width, void *words,
                              fc2_result_escape *esc, uint32_t esc_cap, uint32_t *esc_count, void *stream);
/* The device address of page-locked host memory registered with fc2_host_register (or allocated
 * page-locked): what a kernel writes through to reach it. */
int fc2_host_device_pointer(void *host, void **dev);
/* Host: the 8-byte results back from words[n] (width 4 or 2) and the n_esc escapes (indices < n),
 * on n_threads threads (<= 0: all cores, at most 64).  FC2_E_FORMAT if the escapes do not match
 * the escaped words one to one. */
int fc2_result_expand(const fc2_params *p, const void *words, int width, uint64_t n, const fc2_result_escape *esc,
                      uint64_t n_esc, fc2_result *out, int n_threads);

/* ---- device-resident genome (2-bit bit-sliced + N plane) ---------------- */
/* Bases of all chromosomes are concatenated, each chromosome starting at a
 * multiple of 64.  Unit u covers global bases [64u, 64u+64):
 *   units[2u]   : low  code bit of each base (bit b = base 64u+b)
 *   units[2u+1] : high code bit            (A=00 C=01 G=10 T=11, N=00)
 *   nplane[u]   : 1 where the (uppercased) base is 'N'
 *   ncoarse     : bit k set iff any of units [16k, 16k+16) contains an N
 * Positions outside [0, chrom_size) read as 'N' (get_data's N padding). */
typedef struct fc2_genome_view {
    const uint64_t *units;       /* device [2*n_units] */
    const uint64_t *nplane;      /* device [n_units]   */
    const uint32_t *ncoarse;     /* device [ceil(n_units/16/32)] */
    const uint64_t *chrom_start; /* device [n_chrom] */
    const int64_t  *chrom_size;  /* device [n_chrom] */
    uint64_t n_units;
    uint32_t n_chrom;
    uint32_t dummy;              /* 1: every window is all 'N' (GenomeAccessor dummy mode, :340-345) */
    const uint64_t *units_twin;  /* device [2*(n_units+8)] or NULL: units shifted by half a 128-B line,
                                    units_twin[2t..2t+1] = units of unit t-4 (zero outside the genome);
                                    a window that straddles a line of `units` lies inside one line of
                                    the twin, so a random window costs one line fill instead of ~1.15
                                    (fc2_twin_launch builds it) */
    const uint32_t *nsuper;      /* device [nsuper_words rounded up to a multiple of 4] or NULL: bit k
                                    set iff global bases
                                    [k << nsuper_shift, (k+1) << nsuper_shift) contain an N; small
                                    enough (<= 2048 words) to live in LDS, so a window's N test costs
                                    no memory request (fc2_nsuper_geometry / fc2_nsuper_launch) */
    uint32_t nsuper_shift;
    uint32_t nsuper_words;
    const uint32_t *wt;          /* device or NULL: word-pair layout for the read-order scan
                                    (fc2_wtab_launch): pair q = (low-plane, high-plane) 32-bit code
                                    words of bases [32q, 32q+32) at byte 128 + 8q, then at byte wt_twin_off
                                    the same pairs shifted by 64 B (pair q at wt_twin_off + 8(q+8)), so
                                    that any run of <= 5 pairs lies inside one 128-B line of one copy */
    uint64_t wt_bytes;           /* size of wt in bytes (< 4 GiB: 32-bit buffer offsets) */
    uint64_t wt_twin_off;        /* byte offset of the shifted copy inside wt */
} fc2_genome_view;

/* ---- a batch of anchor pairs in device memory (SoA) --------------------- */
/* Internal read part I = upper(read_part[e:L-e]) (find_circ.py:895), l = L-2e
 * bases, packed per pair in rw 64-bit words stored column-major
 * (word j of pair i at read_words[j*stride + i]): low code bits at bit
 * positions [0,l), high code bits at [l,2l).  read_nwords holds the N bits
 * ([nw][stride], only read for FC2_PAIR_READ_N pairs). */
typedef struct fc2_batch_view {
    const fc2_pair *pairs;       /* device [n] */
    const uint64_t *read_words;  /* device [rw][stride] */
    const uint64_t *read_nwords; /* device [nw][stride] (may be NULL if no pair has READ_N) */
    uint64_t n;
    uint64_t stride;
    uint32_t rw;
    uint32_t nw;
    int32_t  max_l;              /* largest l = L - 2e of a non-BYTEPATH pair (selects the kernel width) */
    uint32_t layout;             /* FC2_BATCH_* hints (results never depend on them) */
    /* Optional window-carrying form (north_star's "two genome windows per pair streamed from the
     * FASTA"; SURVEY.md §8(b) win_2bit): when win_words != NULL the scan reads each pair's windows
     * Af, Bf (find_circ.py:900-902) from these rows instead of gathering them from the genome view
     * (which then needs only chrom_size / n_chrom).  pw = ceil((max_l + 2) / 32) <= 4 32-bit words
     * per plane; pair i's row is ww = 2*pw 64-bit words at win_words[j*stride + i], read as 4*pw
     * 32-bit words: plane p (0 A-low, 1 A-high, 2 B-low, 3 B-high code bits) word k at 32-bit index
     * p*pw + k, bit b = window position 32k + b (positions >= l + 2 zero).  'N' (incl. positions
     * outside the chromosome) = code 00 + a bit in the N row: wnw = pw words at
     * win_nwords[j*stride + i] (A-N words 0..pw-1, B-N words pw..2pw-1), read only for pairs
     * flagged FC2_PAIR_WIN_N.  Built by fc2_pack_windows (host, mmap'd FASTA) or
     * fc2_gather_windows_launch (device, resident genome). */
    const uint64_t *win_words;
    const uint64_t *win_nwords;
    uint32_t ww;
    uint32_t wnw;
} fc2_batch_view;
#define FC2_BATCH_LOCUS_ORDERED 0x1u  /* pairs are sorted by genome locus (fc2_reorder_launch output or a
                                         host-sorted batch): the scan deals each XCD a contiguous range */
/* Per-call form hints (results never depend on them; by default fc2_bp_scan_launch picks the form from
 * the batch and the genome -- LDS-staged for a read-order batch over a genome >= 64 MiB of code planes,
 * plain otherwise; word-pair windows when the view carries wt and l + 2 <= 128; five-lane loads for
 * windows > 97 bases).  They let a caller (the test suite) run every form on any data: */
#define FC2_BATCH_FORM_STAGED  0x02u  /* the LDS-staged form (chromosome table + N super map in LDS)   */
#define FC2_BATCH_FORM_PLAIN   0x04u  /* the plain form (tables from L2, one lane per window)           */
#define FC2_BATCH_FORM_UNITS   0x08u  /* windows from the 64-base unit planes even if wt is present      */
#define FC2_BATCH_FORM_TWOLANE 0x10u  /* staged word-pair form: two-lane window loads at any length     */
#define FC2_BATCH_FORM_TRI     0x20u  /* staged word-pair form: three-lane window loads at any length   */
#define FC2_BATCH_FORM_FIVE    0x40u  /* staged word-pair form: five-lane 8-B window loads at any length */
#define FC2_BATCH_FORM_WAVE    0x80u  /* BASELINE north_star's shape: one wavefront per pair, windows and read
                                         staged in LDS, lane = position x, ballot prefix sums, wave argmax
                                         (needs wt and l + 2 <= 128; otherwise the default form runs) */

/* ---- pairs that need byte-exact evaluation ------------------------------ */
/* Block for pair k at arena[off[k]]: int32 lenI, lenA, lenB, tailB, then
 * I (lenI bytes: read[e:-e].upper() with Python's slice rules, find_circ.py:895), then the A and B
 * windows of get_data(...).upper() (:901-902) in slots of l+3 and 2l+3 bytes (l = read_len - 2e).
 * lenA / lenB are the windows' full lengths (saturated at INT32_MAX); a window outside get_data's
 * defined range can be longer than its slot (:194-211).  The string form of :907-908 reads at most
 * B[:2l+3] when A_flank[:x] + B_flank[x+2:] has the internal part's length (A cut short past the
 * chromosome's end, B padded long before its start); only a one-base internal part that numpy
 * broadcasts over the spliced string (:861-863) reads past B's slot: tailB = the bytes of
 * B[2l+3:] that differ from I[0] when lenI == 1, else 0. */
typedef struct fc2_bytes_view {
    const uint64_t *index;       /* device [m] : pair index into results/tiemask */
    const fc2_pair *pairs;       /* device [m] */
    const uint8_t  *arena;       /* device */
    const uint64_t *off;         /* device [m] */
    uint64_t m;
} fc2_bytes_view;

/* ---- anchor pairs with read parts longer than FC2_MAX_READ_LEN ---------- */
/* fc2_pair's 16-bit read_len and fc2_result's 16-bit best_x / n_ties cannot carry them, so they go
 * in a list of their own with 32-bit fields and are evaluated byte-exactly (fc2_bp_scan_long_launch),
 * one thread per pair, with results of the same meaning as fc2_result's.  Any read length BAM allows
 * (< 2^31) is accepted. */
typedef struct fc2_long_pair {
    uint64_t read_off;  /* the read part: read_len bytes at reads + read_off      */
    uint32_t read_len;  /* L = len(read_part)                                     */
    uint32_t chrom;     /* as fc2_pair.chrom                                      */
    int32_t  a_pos;     /* align_A.pos                                            */
    int32_t  b_aend;    /* align_B.aend                                           */
    uint8_t  flags;     /* FC2_PAIR_BACKSPLICE | FC2_PAIR_PRIMARY_REV | FC2_PAIR_SKIP */
    uint8_t  _pad[7];
} fc2_long_pair;        /* 32 bytes */

typedef struct fc2_long_result {
    int32_t  best_x;    /* as in fc2_result; -1: find_breakpoints returned []    */
    uint32_t n_ties;
    uint8_t  dist, ov;  /* dist saturates at 255 (only with maxdist > 255)       */
    uint16_t info;      /* FC2_RES_*                                              */
    uint32_t _pad;
} fc2_long_result;      /* 16 bytes */

/* ======================================================================== */
/* library info                                                              */
/* ======================================================================== */
int         fc2_abi_version(void);
const char *fc2_last_error(void);
/* Returns FC2_OK and the device count (0 on a host without GPUs is not an error). */
int         fc2_device_count(int *count);
/* Page-lock (hipHostRegister, portable to every device) / release caller-owned host memory, e.g.
 * a node-local shared-memory merge buffer that several per-GPU processes copy results into
 * (find_circ2_amd/shard.py SharedResults): device-to-host copies into it then run at full PCIe rate
 * and asynchronously on a side stream.  Replaces nothing in the reference (find_circ.py is one
 * process); it backs the host-side ordered merge of SURVEY.md 8(e). */
int         fc2_host_register(void *ptr, uint64_t bytes);
int         fc2_host_unregister(void *ptr);

/* Device side of the window-carrying form: the same rows as fc2_pack_windows, gathered from the
 * resident genome (needs g->wt); b supplies pairs/n/stride/max_l, pairs (device, = b->pairs) get
 * FC2_PAIR_WIN_N set or cleared. */
int         fc2_gather_windows_launch(const fc2_params *p, const fc2_genome_view *g, const fc2_batch_view *b,
                                      fc2_pair *pairs, uint64_t *win_words, uint64_t *win_nwords, uint32_t pw,
                                      void *stream);

/* Measurement only: the read-order scan's memory pattern (16-B records and read rows streamed, both
 * windows' word pairs gathered exactly where the scan gathers them, 8-B word per pair stored into
 * out[n]) with none of its arithmetic; its duration is the access-pattern speed of light that
 * bench.py reports next to the scan.  Needs g->wt.  out receives meaningless checksums. */
int         fc2_probe_pattern_launch(const fc2_params *p, const fc2_genome_view *g, const fc2_batch_view *b,
                                     uint64_t *out, void *stream);

/* Performance knobs (results never depend on them) for A/B measurements, process-global.  They exist
 * only in A/B builds of the library (-DFC2_AB_FORMS=1: `make -C find_circ2_amd/csrc ab` ->
 * libfc2_ab.so), together with the measured-and-rejected kernel forms they select (64-bit words,
 * persistent grid, 256/1024-pair staged blocks, cached streaming, extra LDS, forced swizzle/twin).
 * The shipped libfc2.so keeps no mutable tuning state: fc2_set_tuning fails with FC2_E_PARAM there and
 * fc2_get_tuning reports the fixed defaults; per-call form choices go through the FC2_BATCH_FORM_*
 * hints of fc2_batch_view.layout. */
#define FC2_TUNE_STREAM_NT 1   /* 1 (default): per-pair inputs/results use non-temporal loads/stores */
#define FC2_TUNE_KERNEL32  2   /* 1 (default): 32-bit-word scan kernel; 0: 64-bit-word scan kernel */
#define FC2_TUNE_XCD_SWIZZLE 3 /* each XCD scans a contiguous range of the batch: 0 never, 1 always,
                                  2 (default) iff the batch view has FC2_BATCH_LOCUS_ORDERED */
#define FC2_TUNE_REORDER_ROUNDS 4 /* fc2_reorder: pairs per thread per 256-thread chunk (1..32), read by
                                     fc2_reorder_plan */
#define FC2_TUNE_REORDER_NT 5  /* fc2_reorder: 1 = non-temporal scatter stores (default 0) */
#define FC2_TUNE_TWIN 6        /* windows that straddle a line read the genome view's twin: 0 never,
                                  1 always, 2 (default) unless the batch is FC2_BATCH_LOCUS_ORDERED */
#define FC2_TUNE_STAGE 7       /* scan kernel stages the chromosome table and nsuper in LDS: 0 never,
                                  1 always, 2 (default) for batches not locus-ordered over a genome of
                                  >= 64 MiB of code planes */
#define FC2_TUNE_EXTRA_LDS 9   /* bytes of unused LDS added to each scan block (occupancy experiments; 0) */
#define FC2_TUNE_PERSIST 10    /* LDS-staging scan as a persistent grid that stages once per block:
                                  0 off, -1 grid = CUs x resident blocks, k > 0 = CUs x k blocks */
#define FC2_TUNE_WORDS 11      /* 1 (default): the LDS-staging scan reads windows from the view's
                                  word-pair layout (wt) when present; 0: from the unit planes */
#define FC2_TUNE_STAGE_BLOCK 13  /* threads per block of the LDS-staging word-pair scan: 256, 512 (default), 1024 */
#define FC2_TUNE_TRI 14         /* long-window loads of the LDS-staging word-pair scan: 0 two lanes always,
                                   1 three 16-B lanes always, 2 three lanes when a batch's windows exceed
                                   97 bases, 3 (default) five 8-B lanes when they exceed 97 bases */
#define FC2_TUNE_REORDER_SHIFT 12 /* fc2_reorder_plan bucket size 2^shift bases (16..40; raised until
                                     <= 1024 buckets); 0 (default): ~1024 buckets over the genome */
int         fc2_set_tuning(int key, int value);
int         fc2_get_tuning(int key, int *value);

/* Largest l the register kernel handles (longer reads go to the byte kernel). */
int         fc2_max_fast_l(void);
/* Words per pair for the chosen max l: rw (read planes), nw (read N plane),
 * tw (all-hits tie mask: tw/2 words of '+' ties then tw/2 words of '-' ties). */
int         fc2_batch_geometry(const fc2_params *p, int32_t max_read_len,
                               uint32_t *rw, uint32_t *nw, uint32_t *tw);

/* ======================================================================== */
/* device kernels (asynchronous on `stream`)                                 */
/* ======================================================================== */
/* The hot path: JunctionSpan.find_breakpoints for every pair of the batch
 * (pairs flagged FC2_PAIR_BYTEPATH are left for fc2_bp_scan_bytes_launch).
 * tiemask: device [tw][stride] (required iff p->allhits). */
int fc2_bp_scan_launch(const fc2_params *p, const fc2_genome_view *g, const fc2_batch_view *b,
                       fc2_result *results, uint64_t *tiemask, uint32_t tw, void *stream);

/* The scan writing its results straight in a compact form (no 8-byte words, no pack launch, no
 * copy): every pair's word goes to words[i] from the scan's own epilogue, escapes to esc[] through
 * the device counter *esc_count.  words and esc may be page-locked host memory mapped into the device
 * (fc2_host_register + fc2_host_device_pointer): the results then cross PCIe as the scan produces
 * them, which is the ordered merge of a strong-scaled stream without a copy.  *esc_count must be
 * zero before the launch; with count_out != NULL a one-thread kernel after the scan moves the count
 * there (host memory allowed) and zeroes *esc_count again, ready for the next launch.  Canonical
 * mode without --all-hits only, and the batch must hold no FC2_PAIR_BYTEPATH pair (their results
 * come from fc2_bp_scan_bytes_launch as 8-byte words).  Otherwise as fc2_bp_scan_launch. */
typedef struct fc2_compact_out {
    int32_t  width;              /* 2 or 4 */
    uint32_t esc_cap;
    void    *words;              /* [n] uint16 / uint32 */
    fc2_result_escape *esc;      /* [esc_cap] */
    uint32_t *esc_count;         /* device memory */
    uint32_t *count_out;         /* or NULL */
} fc2_compact_out;
int fc2_bp_scan_compact_launch(const fc2_params *p, const fc2_genome_view *g, const fc2_batch_view *b,
                               const fc2_compact_out *co, void *stream);
/* Byte-exact evaluation of the pairs listed in v (any read length, any bytes). */
int fc2_bp_scan_bytes_launch(const fc2_params *p, const fc2_bytes_view *v, fc2_result *results,
                             uint64_t *tiemask, uint32_t tw, uint64_t stride, void *stream);

/* ---- locality reorder ---------------------------------------------------- */
/* A batch in read order sends the lanes of a wave to unrelated genome loci, so
 * every window costs a full HBM line fill.  fc2_reorder_launch writes a copy of
 * the batch stably sorted by genome bucket of the A window
 * (bucket = (chrom_start + a_pos) >> shift, <= 1024 buckets); a scan of the copy
 * (view flagged FC2_BATCH_LOCUS_ORDERED) reads each genome line about once per
 * XCD.  Results of that scan are in reordered order: result i belongs to input
 * pair slot[i].  BYTEPATH / SKIP pairs are moved like any other pair. */
typedef struct fc2_reorder_info {
    uint64_t n;                  /* batch size the plan is for */
    uint64_t workspace_bytes;    /* device scratch fc2_reorder_launch needs */
    uint32_t shift;              /* log2 bases per bucket */
    uint32_t n_buckets;
    uint32_t bucket_bits;        /* ceil(log2(n_buckets)) */
    uint32_t n_chunks;           /* chunks of `chunk` pairs (one workgroup each) */
    uint32_t n_groups;           /* groups of chunks for the offset prefix (<= 128) */
    uint32_t chunk;
} fc2_reorder_info;
int fc2_reorder_plan(const fc2_genome_view *g, uint64_t n, fc2_reorder_info *info);
/* out arrays have the input's shapes: pairs_out [n], read_words_out [rw][stride],
 * read_nwords_out [nw][stride] (only READ_N pairs' rows are written; may be NULL
 * iff in->read_nwords is NULL), slot_out [n]; n < 2^32. */
int fc2_reorder_launch(const fc2_reorder_info *info, const fc2_genome_view *g, const fc2_batch_view *in,
                       fc2_pair *pairs_out, uint64_t *read_words_out, uint64_t *read_nwords_out,
                       uint32_t *slot_out, void *workspace, void *stream);
/* ======================================================================== */
/* host side: FASTA (indexed_fasta semantics, find_circ.py:103-215)         */
/* ======================================================================== */
typedef struct fc2_fasta fc2_fasta;

/* Open + mmap a (multi-)FASTA.  If <path>.byo_index is readable it is used
 * (find_circ.py:110-112); otherwise the file is indexed (:120-155) and, when
 * write_index != 0, the index is stored atomically next to it (:157-179).
 * Errors follow the exception the reference's indexed_fasta() raises:
 *   FC2_E_IO     IOError (missing or unreadable file, a directory -- the -G <folder> form of
 *                find_circ.py:386 -- or an unreadable index): GenomeAccessor catches it and
 *                runs in dummy mode (find_circ.py:338-345), so a host passes NULL to
 *                fc2_ctx_genome_load / fc2_caller_set_genome and goes on;
 *   FC2_E_OS     mmap.error or an OSError writing the index (not caught by the reference);
 *   FC2_E_FORMAT a FASTA / index the reference's index()/load_index() fail on. */
int  fc2_fasta_open(const char *path, int write_index, fc2_fasta **out);
void fc2_fasta_close(fc2_fasta *f);
int  fc2_fasta_n_chrom(const fc2_fasta *f);
/* chrom table in index order; name buffer owned by f. */
int  fc2_fasta_chrom(const fc2_fasta *f, int i, const char **name, int64_t *size,
                     int64_t *ofs, int64_t *ldata, int64_t *skip, int *regular);
int  fc2_fasta_find(const fc2_fasta *f, const char *name);   /* -1 if absent */
/* Reference get_data(chrom, start, end, '+').upper() into out (cap bytes);
 * *len = produced length (= end-start inside the defined range). */
int  fc2_fasta_get_upper(const fc2_fasta *f, int chrom, int64_t start, int64_t end,
                         uint8_t *out, int64_t cap, int64_t *len);
/* Device genome layout for this FASTA. */
int  fc2_fasta_layout(const fc2_fasta *f, uint64_t *n_units, uint64_t *n_coarse_words,
                      uint64_t *chrom_start /* [n_chrom] or NULL */);
/* Pack into host buffers sized by fc2_fasta_layout (units [2*n_units],
 * nplane [n_units], ncoarse [n_coarse_words]); *n_exotic = number of bases
 * that are neither ACGT nor N after uppercasing (they are stored as N and
 * pairs touching them take the byte path).  n_threads <= 0: all cores. */
int  fc2_fasta_pack(const fc2_fasta *f, uint64_t *units, uint64_t *nplane, uint32_t *ncoarse,
                    uint64_t *n_exotic, int n_threads);
/* fc2_fasta_pack into host memory f keeps until the next fc2_ctx_genome_load of f takes it over (that
 * call then only uploads): a host may pack on one thread while another initialises HIP
 * (fc2_ctx_create), as the CLI's start-up does.  Freed with f if no context takes it. */
int  fc2_fasta_prepack(fc2_fasta *f, int n_threads);

/* ======================================================================== */
/* host side: pair packing                                                   */
/* ======================================================================== */
/* Pack n anchor pairs into the device SoA layout (host buffers).
 * reads/read_off/read_len: the read_part strings (find_circ.py:844).
 * pairs_io: in = a_pos, b_aend, chrom, read_len, flags (BACKSPLICE,
 * PRIMARY_REV, SKIP); out = READ_N / BYTEPATH set as needed.
 * f (may be NULL = dummy genome) is used to route pairs whose windows touch
 * exotic genome bytes or irregular FASTA layout, or fall outside the defined
 * window range, to the byte path.  *n_bytepath = number of such pairs. */
int fc2_pack_pairs(const fc2_params *p, const fc2_fasta *f, uint64_t n,
                   const uint8_t *reads, const uint64_t *read_off,
                   fc2_pair *pairs_io, uint64_t *read_words, uint32_t rw,
                   uint64_t *read_nwords, uint32_t nw, uint64_t stride,
                   uint64_t *n_bytepath, int n_threads);

/* Window rows (fc2_batch_view.win_words) for reads up to max_read_len: *pw plane words,
 * *ww = 2*pw row words, *wnw = pw N-row words; FC2_E_RANGE when l + 2 > 128. */
int fc2_window_geometry(const fc2_params *p, int max_read_len, uint32_t *pw, uint32_t *ww, uint32_t *wnw);
/* Host side of the window-carrying form: Af / Bf of every packed, non-SKIP, non-BYTEPATH pair with
 * l >= 0, read from the mmap'd FASTA with get_data's semantics (find_circ.py:189-215, uppercased as
 * at :901-902), into rows of pw plane words; sets FC2_PAIR_WIN_N where a window holds an 'N'. */
int fc2_pack_windows(const fc2_params *p, const fc2_fasta *f, uint64_t n, fc2_pair *pairs_io,
                     uint64_t *win_words, uint64_t *win_nwords, uint32_t pw, uint64_t stride, int n_threads);

/* Size (bytes) of the byte-path arena for the pairs flagged BYTEPATH. */
int fc2_bytepath_size(const fc2_params *p, uint64_t n, const fc2_pair *pairs, uint64_t *m,
                      uint64_t *arena_bytes);
/* Fill index/pairs/off/arena (host) for the BYTEPATH pairs; windows come
 * from f with the reference's get_data semantics (dummy genome if f == NULL). */
int fc2_bytepath_fill(const fc2_params *p, const fc2_fasta *f, uint64_t n,
                      const uint8_t *reads, const uint64_t *read_off, const fc2_pair *pairs,
                      uint64_t *index, fc2_pair *bpairs, uint64_t *off, uint8_t *arena);

/* Long pairs (fc2_long_pair), host side: the byte arena of n long pairs (*arena_bytes) and, for --all-hits, the tie words:
 * pair j's ties are words [tie_off[j], tie_off[j+1]) of a tie array, the first half '+' ties and the
 * second half '-' ties, bit x of word k of a half = breakpoint index 64k + x (tie_off may be NULL;
 * tie_off[n] = the array's length in words). */
int fc2_long_geometry(const fc2_params *p, uint64_t n, const fc2_long_pair *pairs, uint64_t *arena_bytes,
                      uint64_t *tie_off);
/* Fill off [n] and the arena (blocks of fc2_bytes_view's layout) with the read parts and the
 * windows of get_data(...).upper() from f (dummy genome: f == NULL). */
int fc2_long_fill(const fc2_params *p, const fc2_fasta *f, uint64_t n, const uint8_t *reads, const fc2_long_pair *pairs,
                  uint64_t *off, uint8_t *arena);
/* Device: find_breakpoints of every long pair (pairs, off, arena, tie_off and the outputs in device
 * memory); ties (zeroed by the kernel) and tie_off only with p->allhits, else NULL. */
int fc2_bp_scan_long_launch(const fc2_params *p, uint64_t n, const fc2_long_pair *pairs, const uint64_t *off,
                            const uint8_t *arena, const uint64_t *tie_off, fc2_long_result *results, uint64_t *ties,
                            void *stream);

/* ======================================================================== */
/* synthetic workloads (cf. simulate_reads.py)              */
/* ======================================================================== */
typedef struct fc2_synth_cfg {
    uint64_t seed;
    int32_t  len_min, len_max;     /* read length L range                   */
    float    p_planted;            /* junction at a GT..AG / CT..AC site     */
    float    p_minus_site;         /* of planted: CT..AC instead of GT..AG   */
    float    p_backsplice;         /* backsplice vs linear                   */
    float    mut_rate;             /* per-base substitution rate             */
    float    n_rate;               /* per-base N rate in reads               */
    float    p_clip;               /* clip 0..3 bases off each read end      */
    int32_t  span_min, span_max;   /* exon (circ) / intron (linear) span     */
    int32_t  locus_ordered;        /* 1: pair i's locus is drawn from the i-th of n equal genome
                                      strata (a batch ordered by position); 0: uniform (read order) */
    float    p_three_seg;          /* of stream slots (pairs 2s, 2s+1): the two anchor pairs of one
                                      three-segment read wrapping a short circle (config 5: 0.1);
                                      always backsplice, circle length from the read length (span_*,
                                      p_backsplice, p_clip and locus_ordered do not apply to them) */
    uint64_t first;                /* pair i of the call is pair first + i of the seeded stream
                                      (each pair depends only on seed and its stream index): a
                                      rank generates just its share of a stream */
} fc2_synth_cfg;

/* Fill a synthetic genome on the device: random bases from a counter-based
 * hash of (seed, unit), 'N' over the given sorted, non-overlapping global
 * base intervals [n_lo[k], n_hi[k]) (device arrays), coarse map rebuilt. */
int fc2_synth_genome_launch(uint64_t seed, uint64_t *units, uint64_t *nplane, uint32_t *ncoarse,
                            uint64_t n_units, const int64_t *n_lo, const int64_t *n_hi,
                            uint32_t n_intervals, void *stream);
/* Word-pair layout (fc2_genome_view.wt) for a genome of n_units 64-base units: its size and the
 * byte offset of the shifted copy (FC2_E_RANGE if it would not fit 32-bit offsets, > ~8 Gbp), and
 * the kernel that builds it (device [bytes / 4] words) from the unit planes. */
int fc2_wtab_geometry(uint64_t n_units, uint64_t *bytes, uint64_t *twin_off);
int fc2_wtab_launch(const uint64_t *units, uint64_t n_units, uint32_t *wt, void *stream);
/* Build units_twin (device [2*(n_units+8)]) from units (device [2*n_units]). */
int fc2_twin_launch(const uint64_t *units, uint64_t n_units, uint64_t *units_twin, void *stream);
/* Super-coarse N map for n_units: *shift (>= 10) and *words (<= 2048). */
int fc2_nsuper_geometry(uint64_t n_units, uint32_t *shift, uint32_t *words);
/* Build nsuper (device [words]) from the coarse N map ncoarse (device). */
int fc2_nsuper_launch(const uint32_t *ncoarse, uint64_t n_units, uint32_t *nsuper, void *stream);
/* Rebuild the coarse N map from nplane (device). */
int fc2_coarse_launch(const uint64_t *nplane, uint32_t *ncoarse, uint64_t n_units, void *stream);

/* Generate n anchor pairs from the device genome, packed for fc2_bp_scan_launch.
 * chrom_cum: device [n_chrom+1] cumulative chrom sizes used to draw loci.
 * truth (optional, device [2n] int32): planted junction (start, end). */
int fc2_synth_pairs_launch(const fc2_params *p, const fc2_synth_cfg *cfg, const fc2_genome_view *g,
                           const int64_t *chrom_cum, uint64_t n, fc2_pair *pairs,
                           uint64_t *read_words, uint32_t rw, uint64_t *read_nwords, uint32_t nw,
                           uint64_t stride, int32_t *truth, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* FC2_BP_H */
