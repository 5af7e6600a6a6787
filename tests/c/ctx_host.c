/* A C host of the breakpoint search through include/fc2_ctx.h only -- what a cgo / JNI / N-API
 * binding does (the same calls as printed there).
 *
 *   ctx_host FASTA|- BATCH RESULTS asize margin maxdist
 *
 * BATCH: uint64 n, then n fc2_pair records (a_pos, b_aend, chrom, read_len, flags), then uint64 read
 * offsets [n], then the read_part bytes.  RESULTS: the n fc2_result words.  FASTA '-' selects the
 * dummy genome.  Exit status: 0, or 2 with fc2_ctx_last_error / fc2_last_error on stderr. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fc2_ctx.h"

static int die(fc2_ctx *ctx, const char *what) {
    fprintf(stderr, "%s: %s\n", what, ctx ? fc2_ctx_last_error(ctx) : fc2_last_error());
    return 2;
}

int main(int argc, char **argv) {
    if (argc != 7) {
        fprintf(stderr, "usage: %s FASTA|- BATCH RESULTS asize margin maxdist\n", argv[0]);
        return 1;
    }
    FILE *in = fopen(argv[2], "rb");
    if (!in) return 1;
    uint64_t n = 0;
    if (fread(&n, 8, 1, in) != 1) return 1;
    fc2_pair *pairs = (fc2_pair *)malloc(sizeof(fc2_pair) * (n ? n : 1));
    uint64_t *read_off = (uint64_t *)malloc(8 * (n ? n : 1));
    if (fread(pairs, sizeof(fc2_pair), n, in) != n || fread(read_off, 8, n, in) != n) return 1;
    long here = ftell(in);
    fseek(in, 0, SEEK_END);
    const long nbytes = ftell(in) - here;
    fseek(in, here, SEEK_SET);
    uint8_t *reads = (uint8_t *)malloc((size_t)nbytes + 16);
    if (fread(reads, 1, (size_t)nbytes, in) != (size_t)nbytes) return 1;
    fclose(in);

    fc2_params params = {atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), 0, 0, 0, 0};
    fc2_fasta *fa = NULL;
    if (strcmp(argv[1], "-") != 0 && fc2_fasta_open(argv[1], 0, &fa) != FC2_OK) return die(NULL, "fc2_fasta_open");
    fc2_ctx *ctx = NULL;
    if (fc2_ctx_create(0, &ctx) != FC2_OK) return die(NULL, "fc2_ctx_create");
    if (fc2_ctx_genome_load(ctx, fa, 0) != FC2_OK) return die(ctx, "fc2_ctx_genome_load");
    fc2_result *results = (fc2_result *)calloc(n ? n : 1, sizeof(fc2_result));
    if (fc2_ctx_scan_async(ctx, &params, n, reads, read_off, pairs, results, NULL, 0, 0) != FC2_OK ||
        fc2_ctx_sync(ctx) != FC2_OK)
        return die(ctx, "fc2_ctx_scan");
    FILE *out = fopen(argv[3], "wb");
    if (!out || fwrite(results, sizeof(fc2_result), n, out) != n) return 1;
    fclose(out);
    fc2_ctx_destroy(ctx);
    if (fa) fc2_fasta_close(fa);
    free(results); free(reads); free(read_off); free(pairs);
    return 0;
}
