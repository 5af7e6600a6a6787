/*
 * gen_reads.c -- fast generator of the CLI's steady-state input (scripts/cli_steady.py).
 *
 * The same model as scripts/cli_scale_check.py's make_genome / write_sam (the bench's 2M-read CLI
 * input), in C so that tens of millions of reads take seconds: an hg19-shaped genome (the @SQ names
 * and lengths given, random ACGT, one N run of 1,000..140,000 bases per 2 Mbp) and bwa-mem-shaped
 * single-end 100 bp reads -- 60 % unspliced, 20 % backsplice, 20 % linear splice (anchor kA in
 * [20, L-20), intron / circle span in [200, 20000)), GT/AG or CT/AC planted at every junction, one
 * substitution in 30 % of spliced reads, AS = segment length, XS random -- as a primary (kAM(L-kA)S)
 * plus a hard-clipped supplementary ((kA)H(L-kA)M).  Seeded (splitmix64): the same arguments give the
 * same files.  Test/measurement infrastructure, not part of the product.
 *
 * usage: gen_reads SQ_TABLE N_READS SEED OUT.fa OUT.sam [SITES]
 *        SQ_TABLE: one "name<TAB>length" line per chromosome
 *        SITES: 0 (default) plants a junction of its own for every spliced read (every junction is
 *        supported by one read: the junction tables grow with the input); K > 0 plants K junctions
 *        (half backsplice, half linear) and every spliced read crosses one of them, drawn uniformly,
 *        with its own anchor length (junctions supported by many reads, as in real libraries)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t S;
static uint64_t next64(void) {                 /* splitmix64 */
    uint64_t z = (S += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static uint64_t below(uint64_t n) { return n ? next64() % n : 0; }           /* [0, n) */
static int64_t range(int64_t a, int64_t b) { return a + (int64_t)below((uint64_t)(b - a)); }   /* [a, b) */
static double unif(void) { return (double)(next64() >> 11) * (1.0 / 9007199254740992.0); }

#define MAXC 4096
static char *names[MAXC];
static int64_t lens[MAXC];
static unsigned char *seq[MAXC];

static char *out;                               /* output buffer of the SAM writer */
static size_t olen, ocap;
static FILE *fsam;
static void flush_out(void) {
    if (olen && fwrite(out, 1, olen, fsam) != olen) { perror("write sam"); exit(1); }
    olen = 0;
}
static void put(const void *p, size_t n) {
    if (olen + n > ocap) flush_out();
    memcpy(out + olen, p, n);
    olen += n;
}
static void puts_(const char *s) { put(s, strlen(s)); }
static void putc_(char c) { put(&c, 1); }
static void putu(uint64_t v) {
    char b[24];
    int k = 24;
    do { b[--k] = (char)('0' + v % 10); v /= 10; } while (v);
    put(b + k, (size_t)(24 - k));
}

int main(int argc, char **argv) {
    if (argc != 6 && argc != 7) {
        fprintf(stderr, "usage: %s SQ_TABLE N_READS SEED OUT.fa OUT.sam [SITES]\n", argv[0]);
        return 2;
    }
    const uint64_t n_sites = argc == 7 ? strtoull(argv[6], NULL, 10) : 0;
    FILE *t = fopen(argv[1], "r");
    if (!t) { perror(argv[1]); return 1; }
    int nc = 0;
    char nm[1024];
    long long ln;
    while (nc < MAXC && fscanf(t, "%1023s %lld", nm, &ln) == 2) {
        names[nc] = strdup(nm);
        lens[nc] = ln;
        ++nc;
    }
    fclose(t);
    const uint64_t n_reads = strtoull(argv[2], NULL, 10);
    S = strtoull(argv[3], NULL, 10) * 0x2545f4914f6cdd1dull + 1;
    /* genome: 4 random bases per byte of randomness, then the N runs */
    static const unsigned char acgt[4] = {'A', 'C', 'G', 'T'};
    for (int c = 0; c < nc; ++c) {
        seq[c] = (unsigned char *)malloc((size_t)lens[c] + 1);
        if (!seq[c]) { fprintf(stderr, "out of memory\n"); return 1; }
        for (int64_t i = 0; i < lens[c]; i += 32) {
            uint64_t r = next64();
            for (int k = 0; k < 32 && i + k < lens[c]; ++k, r >>= 2) seq[c][i + k] = acgt[r & 3];
        }
        const int64_t runs = lens[c] / 2000000 > 1 ? lens[c] / 2000000 : 1;
        for (int64_t k = 0; k < runs; ++k) {
            const int64_t a = (int64_t)below((uint64_t)lens[c]);
            int64_t e = a + range(1000, 140000);
            if (e > lens[c]) e = lens[c];
            memset(seq[c] + a, 'N', (size_t)(e - a));
        }
    }
    /* reads: chromosomes over 200 kbp, drawn by length */
    int big[MAXC], nb = 0;
    double cum[MAXC], tot = 0;
    for (int c = 0; c < nc; ++c)
        if (lens[c] > 200000) { big[nb] = c; tot += (double)lens[c]; cum[nb++] = tot; }
    if (!nb) { fprintf(stderr, "no chromosome over 200 kbp\n"); return 1; }
    fsam = fopen(argv[5], "wb");
    if (!fsam) { perror(argv[5]); return 1; }
    ocap = 64u << 20;
    out = (char *)malloc(ocap);
    puts_("@HD\tVN:1.5\n");
    for (int c = 0; c < nc; ++c) {
        puts_("@SQ\tSN:");
        puts_(names[c]);
        puts_("\tLN:");
        putu((uint64_t)lens[c]);
        putc_('\n');
    }
    enum { L = 100 };
    /* SITES > 0: the junction sites, planted up front (anchor lengths are drawn per read) */
    typedef struct { int c, back, minus; int64_t lo, hi; } Site;   /* back: E = hi, S = lo; linear: D = lo, D + span = hi */
    Site *sites = NULL;
    if (n_sites) {
        sites = (Site *)malloc(sizeof(Site) * n_sites);
        for (uint64_t k = 0; k < n_sites; ++k) {
            const double x = unif() * tot;
            int lo = 0, hi = nb - 1;
            while (lo < hi) { const int m = (lo + hi) / 2; if (cum[m] <= x) lo = m + 1; else hi = m; }
            Site st;
            st.c = big[lo];
            unsigned char *g = seq[st.c];
            const int64_t G = lens[st.c];
            const int64_t span = range(200, 20000);
            st.back = k % 2 == 0;
            st.minus = unif() < 0.5;
            if (st.back) {                      /* reads take A = G[E-kA:E], B = G[S:S+kB], kA, kB < L */
                st.hi = range(span + L + 10, G - L - 10);
                st.lo = st.hi - span;
                memcpy(g + st.hi, st.minus ? "CT" : "GT", 2);
                memcpy(g + st.lo - 2, st.minus ? "AC" : "AG", 2);
            } else {                            /* A = G[D-kA:D], B = G[D+span:D+span+kB] */
                st.lo = range(L + 10, G - span - L - 10);
                st.hi = st.lo + span;
                memcpy(g + st.lo, st.minus ? "CT" : "GT", 2);
                memcpy(g + st.hi - 2, st.minus ? "AC" : "AG", 2);
            }
            sites[k] = st;
        }
    }
    char qual[L + 1];
    memset(qual, 'I', L);
    qual[L] = 0;
    unsigned char read[L];
    for (uint64_t i = 0; i < n_reads; ++i) {
        const double x = unif() * tot;
        int lo = 0, hi = nb - 1;
        while (lo < hi) { const int m = (lo + hi) / 2; if (cum[m] <= x) lo = m + 1; else hi = m; }
        const int c = big[lo];
        unsigned char *g = seq[c];
        const int64_t G = lens[c];
        const double kind = unif();
        if (kind < 0.6) {                       /* unspliced */
            const int64_t p = range(0, G - L);
            putc_('u'); putu(i); puts_("\t0\t"); puts_(names[c]); putc_('\t'); putu((uint64_t)p + 1);
            puts_("\t60\t100M\t*\t0\t0\t"); put(g + p, L); putc_('\t'); puts_(qual);
            puts_("\tAS:i:100\tXS:i:"); putu(below(40)); putc_('\n');
            continue;
        }
        const int kA = (int)range(20, L - 20);
        const int64_t span = range(200, 20000);
        const int minus = unif() < 0.5;
        int64_t a_pos, b_pos;
        int cr = c;                             /* the read's chromosome */
        if (n_sites) {                          /* a read across one of the planted junctions */
            const Site *st = &sites[below(n_sites)];
            cr = st->c;
            g = seq[cr];
            if (st->back) { a_pos = st->hi - kA; b_pos = st->lo; }
            else { a_pos = st->lo - kA; b_pos = st->hi; }
            memcpy(read, g + a_pos, (size_t)kA);
            memcpy(read + kA, g + b_pos, (size_t)(L - kA));
            (void)span; (void)minus;
            goto emit;
        }
        if (kind < 0.8) {                       /* backsplice: A = G[E-kA:E], B = G[S:S+kB] */
            const int64_t E = range(span + kA + 10, G - 10);
            const int64_t Sx = E - span;
            memcpy(g + E, minus ? "CT" : "GT", 2);
            memcpy(g + Sx - 2, minus ? "AC" : "AG", 2);
            a_pos = E - kA;
            b_pos = Sx;
        } else {                                /* linear: A = G[D-kA:D], B = G[D+span:...] */
            const int64_t D = range(kA + 10, G - span - L - 10);
            memcpy(g + D, minus ? "CT" : "GT", 2);
            memcpy(g + D + span - 2, minus ? "AC" : "AG", 2);
            a_pos = D - kA;
            b_pos = D + span;
        }
        memcpy(read, g + a_pos, (size_t)kA);
        memcpy(read + kA, g + b_pos, (size_t)(L - kA));
    emit:
        if (unif() < 0.3) {
            const int k = (int)below(L);
            const char *q = memchr("ACGT", read[k], 4);
            if (q) read[k] = acgt[(q - "ACGT" + 1) % 4];
        }
        const uint64_t xs = below(12);
        putc_('s'); putu(i); puts_("\t0\t"); puts_(names[cr]); putc_('\t'); putu((uint64_t)a_pos + 1);
        puts_("\t60\t"); putu((uint64_t)kA); putc_('M'); putu((uint64_t)(L - kA)); puts_("S\t*\t0\t0\t");
        put(read, L); putc_('\t'); puts_(qual); puts_("\tAS:i:"); putu((uint64_t)kA); puts_("\tXS:i:"); putu(xs);
        putc_('\n');
        putc_('s'); putu(i); puts_("\t2048\t"); puts_(names[cr]); putc_('\t'); putu((uint64_t)b_pos + 1);
        puts_("\t60\t"); putu((uint64_t)kA); putc_('H'); putu((uint64_t)(L - kA)); puts_("M\t*\t0\t0\t");
        put(read + kA, (size_t)(L - kA)); puts_("\t*\tAS:i:"); putu((uint64_t)(L - kA)); putc_('\n');
    }
    flush_out();
    if (fclose(fsam) != 0) { perror("close sam"); return 1; }
    /* the genome as FASTA, 50 bases a line (UCSC hg19's layout) */
    FILE *fa = fopen(argv[4], "wb");
    if (!fa) { perror(argv[4]); return 1; }
    fsam = fa;
    for (int c = 0; c < nc; ++c) {
        putc_('>'); puts_(names[c]); putc_('\n');
        for (int64_t p = 0; p < lens[c]; p += 50) {
            put(seq[c] + p, (size_t)(lens[c] - p < 50 ? lens[c] - p : 50));
            putc_('\n');
        }
    }
    flush_out();
    if (fclose(fa) != 0) { perror("close fasta"); return 1; }
    return 0;
}
