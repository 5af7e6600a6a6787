/*
 * CPU oracle for the breakpoint-search hot path -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's per-anchor-pair breakpoint search
 * (/root/reference/find_circ.py:854-974) and of its genome window fetch
 * (indexed_fasta.index / get_data, find_circ.py:120-155, 189-215), used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg to CHECK the
 * HIP product path.  It is never linked into find_circ2_amd/.
 *
 *   orc_find_breakpoints_naive : literal O(l^2) form -- for every x build the
 *                                spliced string A[:x]+B[x+2:] and byte-compare
 *                                it with the internal read (find_circ.py:906-908)
 *   orc_find_breakpoints_fast  : O(l) prefix/suffix-sum form of the same
 *                                function; used as the multi-core CPU baseline
 *                                and cross-checked against the naive form.
 *
 * Parity: pinned by the reference's known answers (cdr1as_reference.bed row 2,
 * test_reads.fa truth strings) through tests/test_oracle_known_answers.py, and
 * cross-checked against the literal Python restatement oracle/bp_oracle.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>

#define ORC_OK 0
#define ORC_ERR_KEY 1     /* fast_4mer_RC KeyError, find_circ.py:927            */
#define ORC_ERR_SHAPE 2   /* numpy compare of unequal lengths, find_circ.py:863 */
#define ORC_ERR_CHROM 3   /* chrom missing from index, find_circ.py:193          */

typedef struct {
    int32_t asize, margin, maxdist;
    uint8_t noncanonical, strandpref, allhits, _pad;
} orc_params;

/* one returned Splice (a tie) */
typedef struct {
    int32_t x;
    int32_t start, end;    /* after the backsplice/linear correction, before coord ordering */
    int32_t dist, ov, score;
    int32_t n_hits;
    char strand;           /* '+' / '-' */
    char gtag[5];          /* signal string of the Splice (rc for '-' hits) */
} orc_hit;

/* ------------------------------------------------------------------ */
/* splice-signal helpers (find_circ.py:21-74)                           */
/* ------------------------------------------------------------------ */
static int is_acgtn(unsigned char c) { return c == 'A' || c == 'C' || c == 'G' || c == 'T' || c == 'N'; }
static char comp_upper(char c) {
    switch (c) { case 'A': return 'T'; case 'T': return 'A'; case 'C': return 'G'; case 'G': return 'C'; default: return 'N'; }
}
static void rc4(const char *g, char *out) {  /* rev_comp of a 4-mer over ACGTN */
    for (int i = 0; i < 4; i++) out[i] = comp_upper(g[3 - i]);
    out[4] = 0;
}
static unsigned char up(unsigned char c) { return (c >= 'a' && c <= 'z') ? (unsigned char)(c - 32) : c; }

/* ------------------------------------------------------------------ */
/* indexed FASTA, reference semantics (find_circ.py:120-155, 189-215)   */
/* ------------------------------------------------------------------ */
typedef struct {
    char name[256];
    int64_t ofs, ldata, skip, size;
    char skipchar[8];
    int skiplen;
} orc_chrom;

typedef struct {
    const unsigned char *data;
    int64_t n;
    orc_chrom *chroms;
    int n_chrom;
    int dummy;             /* GenomeAccessor dummy mode (find_circ.py:338-345, 370-371) */
} orc_fasta;

static int is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

/* index(): one pass over lines split after '\n' (Python 2 file iteration). */
orc_fasta *orc_fasta_index(const unsigned char *data, int64_t n) {
    orc_fasta *f = (orc_fasta *)calloc(1, sizeof(orc_fasta));
    int cap = 16;
    f->data = data; f->n = n;
    f->chroms = (orc_chrom *)calloc(cap, sizeof(orc_chrom));
    int64_t ofs = 0, chrom_ofs = 0, size = 0;
    int cur = -1;          /* index of current chrom, -1 = "undef" not yet created */
    char curname[256] = "undef";
    int cur_created = 0;
    int64_t i = 0;
    while (i < n) {
        int64_t j = i;
        while (j < n && data[j] != '\n') j++;
        int64_t len = (j < n) ? (j - i + 1) : (j - i);
        const unsigned char *line = data + i;
        ofs += len;
        /* strip() extent */
        int64_t a = 0, b = len;
        while (a < b && is_space(line[a])) a++;
        while (b > a && is_space(line[b - 1])) b--;
        int64_t stripped = b - a;
        if (len > 0 && line[0] == '>') {
            if (size && cur >= 0) f->chroms[cur].size = size;
            /* chrom = line[1:].split()[0] */
            int64_t s = 1;
            while (s < len && is_space(line[s])) s++;
            int64_t e = s;
            while (e < len && !is_space(line[e])) e++;
            int64_t nl = e - s; if (nl > 255) nl = 255;
            memcpy(curname, line + s, (size_t)nl); curname[nl] = 0;
            chrom_ofs = ofs;
            cur_created = 0;
            /* an existing chrom of the same name (duplicate header) is re-used like the dict */
            cur = -1;
            for (int k = 0; k < f->n_chrom; k++) if (!strcmp(f->chroms[k].name, curname)) { cur = k; cur_created = 1; }
        } else {
            if (!cur_created) {
                if (f->n_chrom == cap) { cap *= 2; f->chroms = (orc_chrom *)realloc(f->chroms, cap * sizeof(orc_chrom)); }
                cur = f->n_chrom++;
                memset(&f->chroms[cur], 0, sizeof(orc_chrom));
                strcpy(f->chroms[cur].name, curname);
                size = 0;
                /* ldata = len(line.strip()); nl_char = len(line) - ldata; skipchar = line[ldata:] */
                f->chroms[cur].ofs = chrom_ofs;
                f->chroms[cur].ldata = stripped;
                f->chroms[cur].skip = len - stripped;
                int sl = (int)(len - stripped); if (sl > 7) sl = 7; if (sl < 0) sl = 0;
                memcpy(f->chroms[cur].skipchar, line + stripped, (size_t)sl);
                f->chroms[cur].skiplen = sl;
                cur_created = 1;
            }
            size += stripped;
        }
        i = j + 1;
    }
    if (size && cur >= 0) f->chroms[cur].size = size;
    return f;
}

/* GenomeAccessor.get_dummy (find_circ.py:370-371): "N"*int(end-start) for every chromosome, which
 * is what find_breakpoints sees once indexed_fasta() raised IOError (:338-345). */
orc_fasta *orc_fasta_dummy(void) {
    orc_fasta *f = (orc_fasta *)calloc(1, sizeof(orc_fasta));
    f->dummy = 1;
    return f;
}

/* load_index (find_circ.py:182-187): the chromosome table of an existing .byo_index replaces the one
 * index() built, since the reference reads that file instead of indexing (:110-112).  Entry k:
 * name, ofs, ldata, skip, skipchar (skiplen bytes, escapes already decoded), size. */
void orc_fasta_set_chroms(orc_fasta *f, int n, const char *const *names, const int64_t *ofs, const int64_t *ldata,
                          const int64_t *skip, const char *const *skipchar, const int32_t *skiplen,
                          const int64_t *size) {
    free(f->chroms);
    f->chroms = (orc_chrom *)calloc((size_t)(n > 0 ? n : 1), sizeof(orc_chrom));
    f->n_chrom = n;
    for (int k = 0; k < n; k++) {
        orc_chrom *c = &f->chroms[k];
        strncpy(c->name, names[k], sizeof c->name - 1);
        c->ofs = ofs[k];
        c->ldata = ldata[k];
        c->skip = skip[k];
        c->size = size[k];
        int sl = skiplen[k] < 0 ? 0 : skiplen[k] > 7 ? 7 : skiplen[k];
        memcpy(c->skipchar, skipchar[k], (size_t)sl);
        c->skiplen = sl;
    }
}

void orc_fasta_free(orc_fasta *f) { if (f) { free(f->chroms); free(f); } }
int orc_fasta_n_chrom(const orc_fasta *f) { return f->n_chrom; }
const char *orc_fasta_chrom_name(const orc_fasta *f, int i) { return f->chroms[i].name; }
int64_t orc_fasta_chrom_size(const orc_fasta *f, int i) { return f->chroms[i].size; }
int orc_fasta_find(const orc_fasta *f, const char *name) {
    for (int k = 0; k < f->n_chrom; k++) if (!strcmp(f->chroms[k].name, name)) return k;
    return -1;
}

static int64_t pyslice_clip(int64_t idx, int64_t n) {  /* Python slice index normalisation */
    if (idx < 0) { idx += n; if (idx < 0) idx = 0; }
    if (idx > n) idx = n;
    return idx;
}

static int64_t floordiv(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b != 0) && ((a < 0) != (b < 0))) q--; return q; }

/* get_data(chrom, start, end, '+') followed by .upper() (find_circ.py:189-215, 901-902).
 * Writes up to cap bytes into out, returns the produced length (may differ from end-start
 * outside the reference's well-defined range). */
int64_t orc_get_upper(const orc_fasta *f, int ci, int64_t start, int64_t end, unsigned char *out, int64_t cap) {
    if (f->dummy) {
        int64_t k = end > start ? end - start : 0;
        for (int64_t q = 0; q < k && q < cap; q++) out[q] = 'N';
        return k;
    }
    const orc_chrom *c = &f->chroms[ci];
    int64_t pad_start = 0, pad_end = 0;
    if (start < 0) { pad_start = -start; start = 0; }
    if (end > c->size) { pad_end = end - c->size; end = c->size; }
    int64_t l_start = floordiv(start, c->ldata), l_end = floordiv(end, c->ldata);
    int64_t os = l_start * c->skip + start + c->ofs;
    int64_t oe = l_end * c->skip + end + c->ofs;
    os = pyslice_clip(os, f->n); oe = pyslice_clip(oe, f->n);
    int64_t k = 0;
    for (int64_t p = 0; p < pad_start && k < cap; p++) out[k++] = 'N';
    /* slice with skip_char removed (str.replace, non-overlapping left-to-right) */
    int64_t p = os;
    while (p < oe) {
        if (c->skiplen > 0 && p + c->skiplen <= oe && !memcmp(f->data + p, c->skipchar, (size_t)c->skiplen)) { p += c->skiplen; continue; }
        if (k < cap) out[k] = up(f->data[p]);
        k++; p++;
    }
    for (int64_t q = 0; q < pad_end; q++) { if (k < cap) out[k] = 'N'; k++; }
    return k;
}

/* ------------------------------------------------------------------ */
/* the hot path                                                          */
/* ------------------------------------------------------------------ */
static int ov_of(int x, int l, int margin) {
    int ov = 0;
    if (margin) {
        if (x < margin) ov = margin - x;
        if (l - x < margin) ov = margin - (l - x);
    }
    return ov;
}

/* Emit candidate hits in the reference's append order and keep the ties.
 * hits_tmp must hold 2*(l+1) entries.  Returns number of ties (= returned Splices). */
static int finish_hits(orc_hit *hits, int nh, orc_hit *ties, int max_ties) {
    if (nh == 0) return 0;
    if (nh < 2) { hits[0].n_hits = 1; if (max_ties > 0) ties[0] = hits[0]; return 1; }
    int best = hits[0].score;
    for (int i = 1; i < nh; i++) if (hits[i].score > best) best = hits[i].score;
    int nt = 0;
    for (int i = 0; i < nh; i++) if (hits[i].score == best) nt++;
    int k = 0;
    for (int i = 0; i < nh; i++) if (hits[i].score == best) { if (k < max_ties) { ties[k] = hits[i]; ties[k].n_hits = nt; } k++; }
    return nt;
}

static void push_hit(orc_hit *h, int x, int start, int end, char strand, int dist, int ov,
                     const char *gtag, int primary_rev, const orc_params *p) {
    h->x = x; h->start = start; h->end = end; h->strand = strand; h->dist = dist; h->ov = ov;
    memcpy(h->gtag, gtag, 4); h->gtag[4] = 0;
    int s = (!strcmp(h->gtag, "GTAG")) * 20 - dist * 10 - ov;
    if (p->strandpref) s += 100 * (strand == (primary_rev ? '-' : '+'));
    h->score = s; h->n_hits = 1;
}

/* One byte of a window whose first `stored` bytes are in W: past them lies the 'N' padding that
 * get_data appends to a window starting past the chromosome end (find_circ.py:194-211). */
static unsigned char win_byte(const unsigned char *W, int64_t stored, int64_t j) { return j < stored ? W[j] : 'N'; }

/* Literal O(l^2) restatement (find_circ.py:854-974).
 * read: read_part (L bytes, any case); Af/Bf: uppercased windows of true lengths la/lb as
 * produced by get_data (normally l+2), of which the first sa/sb bytes are stored.  Returns number
 * of ties written (<= max_ties are stored), or -ORC_ERR_*.  hits_tmp: scratch of >= 2*(l+1) entries.
 *
 * mismatches(a, b) = (fromstring(a) != fromstring(b)).sum() (:861-863) with numpy's rules: equal
 * lengths compare elementwise; a 1-byte operand is broadcast against the other (a 0-byte one
 * against a 1-byte one gives an empty comparison, sum 0); any other pair of lengths makes `!=` the
 * scalar True (numpy 1.x) and .sum() raises -> ORC_ERR_SHAPE.  simple_match (-d 0, :865-866) is the
 * plain string inequality. */
int orc_find_breakpoints_naive(const orc_params *p, const unsigned char *read, int L,
                               const unsigned char *Af, int64_t la, int64_t sa,
                               const unsigned char *Bf, int64_t lb, int64_t sb,
                               int32_t a_pos, int32_t b_aend, int is_backsplice, int primary_rev,
                               orc_hit *hits_tmp, orc_hit *ties, int max_ties) {
    int e = p->asize - p->margin;
    int l = L - 2 * e;
    /* internal = read[e:-e].upper(): Python slice semantics */
    int64_t s0 = e, s1 = -e;
    if (s0 < 0) { s0 += L; if (s0 < 0) s0 = 0; } if (s0 > L) s0 = L;
    if (s1 < 0) { s1 += L; if (s1 < 0) s1 = 0; } else if (e == 0) s1 = 0; if (s1 > L) s1 = L;
    int ilen = (s1 > s0) ? (int)(s1 - s0) : 0;
    unsigned char *internal = (unsigned char *)malloc((size_t)(ilen + 1));
    for (int i = 0; i < ilen; i++) internal[i] = up(read[s0 + i]);
    int nh = 0, err = 0;
    for (int x = 0; x <= l; x++) {
        int64_t n1 = x < la ? x : la;                 /* A_flank[:x] */
        int64_t n2 = (x + 2 < lb) ? lb - (x + 2) : 0; /* B_flank[x+2:] */
        int64_t slen = n1 + n2;
        /* byte j of spliced = A_flank[:x] + B_flank[x+2:] */
#define SPLICED(j) ((j) < n1 ? win_byte(Af, sa, (j)) : win_byte(Bf, sb, x + 2 + (j) - n1))
        int64_t dist;
        if (p->maxdist == 0) {
            /* simple_match: a != b  (bool) */
            int eq = slen == ilen;
            for (int64_t j = 0; eq && j < slen; j++) eq = SPLICED(j) == internal[j];
            dist = !eq;
        } else if (slen == ilen) {
            dist = 0;
            for (int64_t j = 0; j < slen; j++) dist += SPLICED(j) != internal[j];
        } else if (ilen == 1) {
            dist = 0;
            for (int64_t j = 0; j < slen; j++) dist += SPLICED(j) != internal[0];
        } else if (slen == 1) {
            dist = 0;
            for (int j = 0; j < ilen; j++) dist += SPLICED(0) != internal[j];
        } else { err = ORC_ERR_SHAPE; break; }
#undef SPLICED
        if (dist <= p->maxdist) {
            int ov = ov_of(x, l, p->margin);
            char gtag[5] = {0, 0, 0, 0, 0};
            int gl = 0;
            for (int i = x; i < x + 2 && i < la; i++) gtag[gl++] = (char)win_byte(Af, sa, i);
            for (int i = x; i < x + 2 && i < lb; i++) gtag[gl++] = (char)win_byte(Bf, sb, i);
            if (gl != 4) { err = ORC_ERR_KEY; break; }
            for (int i = 0; i < 4; i++) if (!is_acgtn((unsigned char)gtag[i])) { err = ORC_ERR_KEY; }
            if (err) break;
            char rc[5]; rc4(gtag, rc);
            int start = b_aend - e - l + x, end = a_pos + e + x + 1;
            int lo = start < end ? start : end, hi = start < end ? end : start;
            start = lo; end = hi;
            if (is_backsplice) end -= 1; else start -= 1;
            if (p->noncanonical) {
                push_hit(&hits_tmp[nh++], x, start, end, '+', (int)dist, ov, gtag, primary_rev, p);
                push_hit(&hits_tmp[nh++], x, start, end, '-', (int)dist, ov, rc, primary_rev, p);
            } else if (!strcmp(gtag, "GTAG")) {
                push_hit(&hits_tmp[nh++], x, start, end, '+', (int)dist, ov, gtag, primary_rev, p);
            } else if (!strcmp(gtag, "CTAC")) {
                push_hit(&hits_tmp[nh++], x, start, end, '-', (int)dist, ov, rc, primary_rev, p);
            }
        }
    }
    free(internal);
    if (err) return -err;
    return finish_hits(hits_tmp, nh, ties, max_ties);
}

/* O(l) form: mismatch prefix over A and suffix over B (same outputs as naive for
 * windows of the regular length l+2). */
int orc_find_breakpoints_fast(const orc_params *p, const unsigned char *read, int L,
                              const unsigned char *Af, const unsigned char *Bf,
                              int32_t a_pos, int32_t b_aend, int is_backsplice, int primary_rev,
                              orc_hit *hits_tmp, orc_hit *ties, int max_ties) {
    int e = p->asize - p->margin;
    int l = L - 2 * e;
    if (e <= 0) return -ORC_ERR_SHAPE;
    if (l < 0) return 0;
    const unsigned char *I = read + e;
    int totB = 0;
    for (int i = 0; i < l; i++) totB += Bf[i + 2] != up(I[i]);
    int dist = totB, nh = 0;
    for (int x = 0; x <= l; x++) {
        if (x > 0) { unsigned char c = up(I[x - 1]); dist += (Af[x - 1] != c) - (Bf[x + 1] != c); }
        if (dist <= p->maxdist) {
            int ov = ov_of(x, l, p->margin);
            char gtag[5] = {(char)Af[x], (char)Af[x + 1], (char)Bf[x], (char)Bf[x + 1], 0};
            for (int i = 0; i < 4; i++) if (!is_acgtn((unsigned char)gtag[i])) return -ORC_ERR_KEY;
            char rc[5]; rc4(gtag, rc);
            int start = b_aend - e - l + x, end = a_pos + e + x + 1;
            int lo = start < end ? start : end, hi = start < end ? end : start;
            start = lo; end = hi;
            if (is_backsplice) end -= 1; else start -= 1;
            int dd = (p->maxdist == 0) ? 0 : dist;
            if (p->noncanonical) {
                push_hit(&hits_tmp[nh++], x, start, end, '+', dd, ov, gtag, primary_rev, p);
                push_hit(&hits_tmp[nh++], x, start, end, '-', dd, ov, rc, primary_rev, p);
            } else if (!strcmp(gtag, "GTAG")) {
                push_hit(&hits_tmp[nh++], x, start, end, '+', dd, ov, gtag, primary_rev, p);
            } else if (!strcmp(gtag, "CTAC")) {
                push_hit(&hits_tmp[nh++], x, start, end, '-', dd, ov, rc, primary_rev, p);
            }
        }
    }
    return finish_hits(hits_tmp, nh, ties, max_ties);
}

/* ------------------------------------------------------------------ */
/* batch driver over a FASTA (used by tests and the CPU baseline)        */
/* ------------------------------------------------------------------ */
/* Per pair outputs: n_ties[i] (0 = no hit, <0 = -error), first tie in first[i].
 * If allhits, all ties are appended to all_ties (capacity cap_all); all_off[i] = start index.
 * chrom_idx[i] indexes f's chrom table (-1 -> ORC_ERR_CHROM).  use_fast selects the O(l) form. */
int64_t orc_scan_fasta(const orc_params *p, const orc_fasta *f, int64_t n,
                       const unsigned char *reads, const int64_t *read_off, const int32_t *read_len,
                       const int32_t *chrom_idx, const int32_t *a_pos, const int32_t *b_aend,
                       const uint8_t *is_bs, const uint8_t *primary_rev, int use_fast,
                       int32_t *n_ties, orc_hit *first, orc_hit *all_ties, int64_t cap_all, int64_t *all_off,
                       int n_threads) {
    int64_t total_all = 0;
    int e = p->asize - p->margin;
    (void)n_threads;
    int maxL = 0;
    for (int64_t i = 0; i < n; i++) if (read_len[i] > maxL) maxL = read_len[i];
    int wcap = maxL + 2 * (e < 0 ? -e : 0) + 8;
    int hcap = 2 * (maxL + 2 * (e < 0 ? -e : 0) + 2) + 4;
    unsigned char *Af = (unsigned char *)malloc((size_t)wcap * 2 + 64);
    unsigned char *Bf = (unsigned char *)malloc((size_t)wcap * 2 + 64);
    orc_hit *tmp = (orc_hit *)malloc(sizeof(orc_hit) * (size_t)hcap);
    orc_hit *ties = (orc_hit *)malloc(sizeof(orc_hit) * (size_t)hcap);
    for (int64_t i = 0; i < n; i++) {
        int L = read_len[i];
        int l = L - 2 * e;
        int ci = chrom_idx[i];
        if (all_off) all_off[i] = total_all;
        if (!f->dummy && (ci < 0 || ci >= f->n_chrom)) { n_ties[i] = -ORC_ERR_CHROM; continue; }
        int flank = l + 2;
        int64_t as = (int64_t)a_pos[i] + e, bs = (int64_t)b_aend[i] - e - flank;
        int64_t la = 0, lb = 0;
        if (flank > 0 && flank <= wcap) {
            /* true lengths; the buffers keep the first wcap * 2 bytes (a longer window is 'N' padding
             * past that point, win_byte) */
            la = orc_get_upper(f, ci, as, as + flank, Af, wcap * 2);
            lb = orc_get_upper(f, ci, bs, bs + flank, Bf, wcap * 2);
        }
        int r;
        if (use_fast && e > 0 && la == flank && lb == flank)
            r = orc_find_breakpoints_fast(p, reads + read_off[i], L, Af, Bf, a_pos[i], b_aend[i], is_bs[i], primary_rev[i], tmp, ties, hcap);
        else
            r = orc_find_breakpoints_naive(p, reads + read_off[i], L, Af, la, la < wcap * 2 ? la : wcap * 2, Bf, lb,
                                           lb < wcap * 2 ? lb : wcap * 2, a_pos[i], b_aend[i], is_bs[i], primary_rev[i],
                                           tmp, ties, hcap);
        n_ties[i] = r;
        if (r > 0) {
            first[i] = ties[0];
            if (all_ties) {
                for (int k = 0; k < r && k < hcap; k++) { if (total_all < cap_all) all_ties[total_all] = ties[k]; total_all++; }
            }
        }
    }
    free(Af); free(Bf); free(tmp); free(ties);
    return total_all;
}

/* Same, with caller-provided windows (Af/Bf arenas of l+2 bytes per pair at win_off[i]). */
int64_t orc_scan_windows(const orc_params *p, int64_t n,
                         const unsigned char *reads, const int64_t *read_off, const int32_t *read_len,
                         const unsigned char *wins, const int64_t *win_off, /* Af then Bf, each l+2 */
                         const int32_t *a_pos, const int32_t *b_aend,
                         const uint8_t *is_bs, const uint8_t *primary_rev, int use_fast,
                         int32_t *n_ties, orc_hit *first, orc_hit *all_ties, int64_t cap_all, int64_t *all_off) {
    int64_t total_all = 0;
    int e = p->asize - p->margin;
    int maxL = 0;
    for (int64_t i = 0; i < n; i++) if (read_len[i] > maxL) maxL = read_len[i];
    int hcap = 2 * (maxL + 2 * (e < 0 ? -e : 0) + 2) + 4;
    orc_hit *tmp = (orc_hit *)malloc(sizeof(orc_hit) * (size_t)hcap);
    orc_hit *ties = (orc_hit *)malloc(sizeof(orc_hit) * (size_t)hcap);
    for (int64_t i = 0; i < n; i++) {
        int L = read_len[i];
        int l = L - 2 * e;
        if (all_off) all_off[i] = total_all;
        int flank = l + 2;
        if (flank < 0) flank = 0;
        const unsigned char *Af = wins + win_off[i];
        const unsigned char *Bf = Af + flank;
        int r;
        if (use_fast && e > 0)
            r = orc_find_breakpoints_fast(p, reads + read_off[i], L, Af, Bf, a_pos[i], b_aend[i], is_bs[i], primary_rev[i], tmp, ties, hcap);
        else
            r = orc_find_breakpoints_naive(p, reads + read_off[i], L, Af, flank, flank, Bf, flank, flank, a_pos[i], b_aend[i], is_bs[i], primary_rev[i], tmp, ties, hcap);
        n_ties[i] = r;
        if (r > 0) {
            first[i] = ties[0];
            if (all_ties) {
                for (int k = 0; k < r && k < hcap; k++) { if (total_all < cap_all) all_ties[total_all] = ties[k]; total_all++; }
            }
        }
    }
    free(tmp); free(ties);
    return total_all;
}

/* ------------------------------------------------------------------ */
/* whole-batch check straight from the device layouts (full-size parity) */
/* ------------------------------------------------------------------ */
/* The same search, fed from the documented device layouts of include/fc2_bp.h instead of a
 * FASTA: the internal read part I is decoded from the tight bit-sliced rows (low code bits at
 * [0,l), high at [l,2l), 'N' from the N row of READ_N pairs), the windows Af/Bf from the 2-bit
 * genome unit planes + N plane (get_data's 'N' padding outside [0, size), find_circ.py:194-211),
 * and the first tie is encoded as the 8-byte fc2_result word the kernel writes (best_x, dist, ov,
 * n_ties, info = DONE | MINUS | 3-bit codes of A[x]A[x+1]B[x]B[x+1] | KEY error).  Threads split
 * the batch.  Returns the number of pairs it could not check (BYTEPATH pairs, chromosome index
 * out of range: their word is left 0). */
#include <pthread.h>

typedef struct {            /* fc2_pair */
    int32_t a_pos, b_aend;
    uint32_t chrom;
    uint16_t read_len;
    uint8_t flags, npos;
} orc_pair;

typedef struct {
    const orc_params *p;
    const uint64_t *units, *nplane, *chrom_start;
    const int64_t *chrom_size;
    int n_chrom;
    const orc_pair *pairs;
    const uint64_t *rows, *nrows;
    uint64_t stride;
    uint32_t rw, nw;
    int64_t lo, hi;
    uint64_t *out;
    int64_t skipped;
} orc_plane_job;

static unsigned char orc_base(const orc_plane_job *J, int c, int64_t pos) {
    static const unsigned char code[4] = {'A', 'C', 'G', 'T'};
    if (pos < 0 || pos >= J->chrom_size[c]) return 'N';
    const uint64_t g = J->chrom_start[c] + (uint64_t)pos, u = g >> 6, b = g & 63;
    if ((J->nplane[u] >> b) & 1) return 'N';
    return code[((J->units[2 * u] >> b) & 1) | (((J->units[2 * u + 1] >> b) & 1) << 1)];
}

static unsigned orc_code3(unsigned char c) {
    switch (c) { case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3; default: return 4; }
}

static void *orc_plane_worker(void *arg) {
    orc_plane_job *J = (orc_plane_job *)arg;
    const orc_params *p = J->p;
    const int e = p->asize - p->margin;
    int maxL = 0;
    for (int64_t i = J->lo; i < J->hi; i++) if (J->pairs[i].read_len > maxL) maxL = J->pairs[i].read_len;
    const int hcap = 2 * (maxL + 2) + 4;
    unsigned char *read = (unsigned char *)malloc((size_t)maxL + 8);
    unsigned char *Af = (unsigned char *)malloc((size_t)maxL + 8);
    unsigned char *Bf = (unsigned char *)malloc((size_t)maxL + 8);
    orc_hit *tmp = (orc_hit *)malloc(sizeof(orc_hit) * (size_t)hcap);
    orc_hit *ties = (orc_hit *)malloc(sizeof(orc_hit) * (size_t)hcap);
    const uint64_t none = 0xFFFFull | ((uint64_t)0x8000u << 48);
    for (int64_t i = J->lo; i < J->hi; i++) {
        const orc_pair pr = J->pairs[i];
        J->out[i] = 0;
        if (pr.flags & 0x10) { J->out[i] = none; continue; }                     /* SKIP */
        if ((pr.flags & 0x08) || (int)pr.chrom >= J->n_chrom) { J->skipped++; continue; }   /* BYTEPATH */
        const int L = pr.read_len, l = L - 2 * e;
        if (l < 0 || e <= 0) { J->out[i] = none; continue; }
        for (int k = 0; k < e; k++) read[k] = read[e + l + k] = 'A';
        for (int j = 0; j < l; j++) {
            const int t = l + j;
            const unsigned lo = (unsigned)(J->rows[(uint64_t)(j >> 6) * J->stride + i] >> (j & 63)) & 1u;
            const unsigned hi = (unsigned)(J->rows[(uint64_t)(t >> 6) * J->stride + i] >> (t & 63)) & 1u;
            unsigned char c = "ACGT"[lo | (hi << 1)];
            if ((pr.flags & 0x04) && ((J->nrows[(uint64_t)(j >> 6) * J->stride + i] >> (j & 63)) & 1)) c = 'N';
            read[e + j] = c;
        }
        const int W = l + 2;
        const int64_t as = (int64_t)pr.a_pos + e, bs = (int64_t)pr.b_aend - e - W;
        for (int k = 0; k < W; k++) { Af[k] = orc_base(J, (int)pr.chrom, as + k); Bf[k] = orc_base(J, (int)pr.chrom, bs + k); }
        const int r = orc_find_breakpoints_fast(p, read, L, Af, Bf, pr.a_pos, pr.b_aend, pr.flags & 1,
                                                (pr.flags >> 1) & 1, tmp, ties, hcap);
        if (r < 0) { J->out[i] = none | ((uint64_t)(r == -ORC_ERR_KEY ? 0x2000u : 0x4000u) << 48); continue; }
        if (r == 0) { J->out[i] = none; continue; }
        const orc_hit *h = &ties[0];
        const int x = h->x;
        const unsigned g12 = orc_code3(Af[x]) | (orc_code3(Af[x + 1]) << 3) | (orc_code3(Bf[x]) << 6) |
                             (orc_code3(Bf[x + 1]) << 9);
        const unsigned info = 0x8000u | (h->strand == '-' ? 1u : 0u) | ((g12 << 1) & 0x1FFEu);
        const unsigned nt = r > 0xFFFF ? 0xFFFFu : (unsigned)r;
        const unsigned dist = h->dist > 255 ? 255u : (unsigned)h->dist;
        J->out[i] = (uint64_t)(uint16_t)(int16_t)x | ((uint64_t)(dist & 0xFF) << 16) | ((uint64_t)(h->ov & 0xFF) << 24) |
                    ((uint64_t)nt << 32) | ((uint64_t)info << 48);
    }
    free(read); free(Af); free(Bf); free(tmp); free(ties);
    return NULL;
}

int64_t orc_scan_planes(const orc_params *p, const uint64_t *units, const uint64_t *nplane,
                        const uint64_t *chrom_start, const int64_t *chrom_size, int n_chrom,
                        const void *pairs, const uint64_t *read_words, const uint64_t *read_nwords,
                        uint32_t rw, uint32_t nw, uint64_t stride, int64_t n, uint64_t *out, int n_threads) {
    (void)rw; (void)nw;
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    orc_plane_job jobs[256];
    pthread_t th[256];
    const int64_t per = (n + n_threads - 1) / n_threads;
    int started = 0;
    for (int t = 0; t < n_threads; t++) {
        orc_plane_job *J = &jobs[t];
        J->p = p; J->units = units; J->nplane = nplane; J->chrom_start = chrom_start; J->chrom_size = chrom_size;
        J->n_chrom = n_chrom; J->pairs = (const orc_pair *)pairs; J->rows = read_words; J->nrows = read_nwords;
        J->stride = stride; J->rw = rw; J->nw = nw; J->out = out; J->skipped = 0;
        J->lo = t * per; J->hi = (t + 1) * per < n ? (t + 1) * per : n;
        if (J->lo >= J->hi) break;
        pthread_create(&th[t], NULL, orc_plane_worker, J);
        started++;
    }
    int64_t skipped = 0;
    for (int t = 0; t < started; t++) { pthread_join(th[t], NULL); skipped += jobs[t].skipped; }
    return skipped;
}
