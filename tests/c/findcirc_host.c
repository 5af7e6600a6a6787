/* find_circ2 as a C program over the C ABI alone -- no Python, no PyTorch: the read loop of
 * include/fc2_caller.h (SAM/BAM ingest, anchor pairs, record_hits, junction tables, writers) with
 * the breakpoint search on the GPU through include/fc2_ctx.h.
 *
 *   findcirc_host -G genome.fa -o outdir [-n name] alignments.{sam,bam}|-
 *
 * The reference's default options (find_circ.py:383-413); writes circ_splice_sites.bed,
 * lin_splice_sites.bed, multi_events.tsv and spliced_reads.fastq.gz as the Python CLI does with its
 * native loop (tests/test_ctx_c_host.py compares them).  Sequential: next -> scan -> submit. */
#define _POSIX_C_SOURCE 200809L   /* fileno */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "fc2_caller.h"
#include "fc2_ctx.h"

static const char *kBedHeader =
    "#chrom\tstart\tend\tname\tn_frags\tstrand\tn_weight\tn_spanned\tn_uniq\tuniq_bridges\tbest_qual_left\t"
    "best_qual_right\ttissues\ttiss_counts\tedits\tanchor_overlap\tbreakpoints\tsignal\tstrandmatch\tcategory\t"
    "flags\tflag_counts\n";
static const char *kMultiHeader =
    "#chrom\tstart\tend\tname\tscore\tstrand\tfragment_name\tlin_cons\tlin_incons\tunspliced_cons\t"
    "unspliced_incons\n";

static int fail(const char *what, const char *msg) {
    fprintf(stderr, "%s: %s\n", what, msg ? msg : "");
    return 2;
}

static FILE *out_file(const char *dir, const char *name) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    return fopen(path, "wb");
}

int main(int argc, char **argv) {
    const char *genome = NULL, *outdir = "find_circ_run", *name = "unknown", *input = NULL;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-G") && i + 1 < argc) genome = argv[++i];
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) outdir = argv[++i];
        else if (!strcmp(argv[i], "-n") && i + 1 < argc) name = argv[++i];
        else input = argv[i];
    }
    if (!genome || !input) {
        fprintf(stderr, "usage: %s -G genome.fa -o outdir [-n name] alignments|-\n", argv[0]);
        return 1;
    }
    mkdir(outdir, 0755);
    fc2_fasta *fa = NULL;
    const int frc = fc2_fasta_open(genome, 1, &fa);
    if (frc == FC2_E_IO) {   /* the reference's IOError: GenomeAccessor's all-N dummy mode (find_circ.py:338-345) */
        fprintf(stderr, "Could not access '%s'. Switching to dummy mode (only Ns)\n", genome);
        fa = NULL;
    } else if (frc != FC2_OK) {
        return fail("fc2_fasta_open", fc2_last_error());
    }
    fc2_ctx *ctx = NULL;
    if (fc2_ctx_create(0, &ctx) != FC2_OK) return fail("fc2_ctx_create", fc2_last_error());
    if (fc2_ctx_genome_load(ctx, fa, 0) != FC2_OK) return fail("fc2_ctx_genome_load", fc2_ctx_last_error(ctx));

    fc2_caller_opts o;
    memset(&o, 0, sizeof o);
    o.name = name;
    o.min_uniq_qual = 2; o.asize = 15; o.margin = 2; o.maxdist = 2;
    o.short_threshold = 100; o.huge_threshold = 100000;
    o.multi_events = 1; o.write_reads = 1; o.write_multi = 1;
    o.chunksize = 100000;
    fc2_caller *c = NULL;
    if (fc2_caller_open(input, 0, &o, &c) != FC2_OK) return fail("fc2_caller_open", fc2_last_error());
    fc2_ingest *ing = fc2_caller_ingest(c);
    const int n_ref = fc2_ingest_n_refs(ing);
    int32_t *t2c = (int32_t *)malloc(sizeof(int32_t) * (n_ref > 0 ? n_ref : 1));
    for (int t = 0; t < n_ref; ++t) t2c[t] = fa ? fc2_fasta_find(fa, fc2_ingest_ref_name(ing, t)) : 0;
    if (fc2_caller_set_genome(c, t2c, n_ref, fa, NULL, NULL) != FC2_OK) return fail("fc2_caller_set_genome", fc2_last_error());
    char gz[4096];
    snprintf(gz, sizeof gz, "%s/spliced_reads.fastq.gz", outdir);
    if (fc2_caller_set_reads_gz(c, gz, 2, 4, 0) != FC2_OK) return fail("fc2_caller_set_reads_gz", fc2_last_error());
    FILE *multi = out_file(outdir, "multi_events.tsv");
    if (!multi) return fail("open", "multi_events.tsv");
    fputs(kMultiHeader, multi);

    const fc2_params params = {o.asize, o.margin, o.maxdist, 0, 0, 0, 0};
    fc2_result *results = NULL;
    uint64_t cap = 0;
    for (int eof = 0; !eof;) {
        fc2_caller_batch b;
        if (fc2_caller_next(c, &b, &eof) != FC2_OK) return fail("fc2_caller_next", fc2_last_error());
        if (b.n > cap) {
            free(results);
            cap = b.n;
            results = (fc2_result *)malloc(sizeof(fc2_result) * cap);
        }
        if (b.n && (fc2_ctx_scan_async(ctx, &params, b.n, b.reads, b.read_off, b.pairs, results, NULL, 0, 0) != FC2_OK ||
                    fc2_ctx_sync(ctx) != FC2_OK))
            return fail("fc2_ctx_scan", fc2_ctx_last_error(ctx));
        if (b.n_long) {                        /* read parts over FC2_MAX_READ_LEN: the long path */
            fc2_long_result *lr = (fc2_long_result *)malloc(sizeof(fc2_long_result) * b.n_long);
            if (fc2_ctx_scan_long(ctx, &params, b.n_long, b.reads, b.long_pairs, lr, NULL) != FC2_OK)
                return fail("fc2_ctx_scan_long", fc2_ctx_last_error(ctx));
            if (fc2_caller_submit_long(c, lr, b.n_long, NULL, 0) != FC2_OK) return fail("fc2_caller_submit_long", fc2_last_error());
            free(lr);
        }
        if (fc2_caller_submit(c, b.n ? results : NULL, NULL, 0, b.n) != FC2_OK) return fail("fc2_caller_submit", fc2_last_error());
        const char *t;
        uint64_t len;
        if (fc2_caller_take(c, 1, &t, &len) == FC2_OK && len) fwrite(t, 1, len, multi);
    }
    fclose(multi);
    if (fc2_caller_close_reads(c) != FC2_OK) return fail("fc2_caller_close_reads", fc2_last_error());
    const char *files[2] = {"circ_splice_sites.bed", "lin_splice_sites.bed"};
    for (int kind = 0; kind < 2; ++kind) {
        const char *t;
        uint64_t len;
        FILE *f = out_file(outdir, files[kind]);
        if (!f) return fail("open", files[kind]);
        fputs(kBedHeader, f);
        if (kind == 0) {                       /* the rows as text ... */
            if (fc2_caller_rows(c, kind, &t, &len) != FC2_OK) return fail("fc2_caller_rows", fc2_last_error());
            if (len) fwrite(t, 1, len, f);
        } else {                               /* ... or written to the file by the library (the CLI's way) */
            fflush(f);
            if (fc2_caller_write_rows(c, kind, fileno(f), &len) != FC2_OK)
                return fail("fc2_caller_write_rows", fc2_last_error());
        }
        fclose(f);
    }
    fc2_caller_close(c);
    fc2_ctx_destroy(ctx);
    if (fa) fc2_fasta_close(fa);
    free(results);
    free(t2c);
    return 0;
}
