// fc2_caller.cpp -- native find_circ read loop around the breakpoint search
// (include/fc2_caller.h).  Same logic and output as find_circ2_amd/caller.py,
// which cites find_circ.py line by line; the comments here point at the
// reference where the semantics are subtle.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "../../include/fc2_caller.h"
#include "fc2_common.h"
#include "fc2_ingest_impl.h"

using fc2::ing::Mate;
using fc2::ing::Rec;

namespace {

// ---- Python-2 formatting ---------------------------------------------------------
std::string py2_float(double v) {             // str(float) in Python 2: '%.12g' (+ '.0')
    if (v != v) return "nan";
    if (isinf(v)) return v > 0 ? "inf" : "-inf";
    char b[64];
    snprintf(b, sizeof b, "%.12g", v);
    std::string r(b);
    if (r.find_first_of(".en") == std::string::npos) r += ".0";
    return r;
}

std::string i2s(int64_t v) { return std::to_string(v); }

std::string py_repr(const std::string &s) {   // repr(str), for the --test rows
    const bool sq = s.find('\'') != std::string::npos, dq = s.find('"') != std::string::npos;
    const char q = (sq && !dq) ? '"' : '\'';
    std::string r(1, q);
    for (unsigned char c : s) {
        if (c == '\\') r += "\\\\";
        else if (c == (unsigned char)q) { r += '\\'; r += (char)c; }
        else if (c == '\n') r += "\\n";
        else if (c == '\r') r += "\\r";
        else if (c == '\t') r += "\\t";
        else if (c < 32 || c >= 127) { char b[8]; snprintf(b, sizeof b, "\\x%02x", c); r += b; }
        else r += (char)c;
    }
    r += q;
    return r;
}

struct Fatal {                                 // an exception the reference raises
    int code;
    std::string msg;
};

// find_circ.py:54-58 (KeyError outside the IUPAC table)
char comp(char c) {
    switch (c) {
        case 'a': return 't'; case 't': return 'a'; case 'c': return 'g'; case 'g': return 'c';
        case 'k': return 'm'; case 'm': return 'k'; case 'r': return 'y'; case 'y': return 'r';
        case 's': return 's'; case 'w': return 'w'; case 'b': return 'v'; case 'v': return 'b';
        case 'h': return 'd'; case 'd': return 'h'; case 'n': return 'n';
        case 'A': return 'T'; case 'T': return 'A'; case 'C': return 'G'; case 'G': return 'C';
        case 'K': return 'M'; case 'M': return 'K'; case 'R': return 'Y'; case 'Y': return 'R';
        case 'S': return 'S'; case 'W': return 'W'; case 'B': return 'V'; case 'V': return 'B';
        case 'H': return 'D'; case 'D': return 'H'; case 'N': return 'N';
        default: return 0;
    }
}

void rev_comp_into(const std::string &s, std::string &r) {
    r.resize(s.size());
    for (size_t k = 0; k < s.size(); ++k) {
        const char c = comp(s[s.size() - 1 - k]);
        if (!c) throw Fatal{FC2_E_KEY, std::string("KeyError: ") + py_repr(std::string(1, s[s.size() - 1 - k]))};
        r[k] = c;
    }
}

std::string rev_comp(const std::string &s) {
    std::string r;
    rev_comp_into(s, r);
    return r;
}

// ---- data ----------------------------------------------------------------------
struct Align {                                 // what record_hits and the writers read of an alignment
    std::string qname, seq, qual;
    bool has_seq = false, has_qual = false;
    int32_t tid = -1;
    int64_t pos = -1, aend = -1;               // aend -1: None
    bool rev = false;
};

Align make_align(const Rec &r) {
    Align a;
    a.qname = r.qname;
    a.seq = r.seq;
    a.qual = r.qual;
    a.has_seq = r.has_seq;
    a.has_qual = r.has_qual;
    a.tid = r.tid;
    a.pos = r.pos;
    a.aend = r.aend;
    a.rev = r.reverse();
    return a;
}

struct Span {                                  // JunctionSpan (:821-852)
    int mate;                                  // 0 = mate1, 1 = mate2 of the fragment
    int32_t tid;                               // chromosome (reference id of the segments)
    bool circ;                                 // is_backsplice: B.pos - A.aend < 0
    int64_t a_pos, b_aend;
    double weight;
    int64_t uniq;
    int64_t qA, qB;                            // Hit.add's anchor qualities (after the backsplice swap)
    bool a_rev;                                // A.is_reverse after the swap
    uint64_t read_off;
    uint32_t read_len;
    int64_t eval = -1;                         // index in the evaluation batch
};

struct Frag {
    std::string name;
    bool has[2] = {false, false};
    Align prim[2];
    std::vector<int> circ, lin;                // indices into the chunk's spans
    std::vector<Align> unspliced, broken;
};

using Coord = std::tuple<std::string, int64_t, int64_t, std::string>;   // (chrom, start, end, strand)

// SpliceSiteStorage's dict key (the coord tuple), without building a string: the chromosome and the
// strand interned to small ids, the two positions as they are
struct CKey {
    int64_t start, end;
    uint32_t chrom, strand;
    bool operator==(const CKey &o) const {
        return start == o.start && end == o.end && chrom == o.chrom && strand == o.strand;
    }
};
struct CKeyHash {
    size_t operator()(const CKey &k) const {
        uint64_t x = (uint64_t)k.start * 0x9E3779B97F4A7C15ull ^ ((uint64_t)k.end + 0x632BE59BD9B4E019ull);
        x ^= ((uint64_t)k.chrom << 32 | k.strand) * 0xD6E8FEB86659FD93ull;
        return (size_t)(x ^ (x >> 29));
    }
};

// Open-addressing CKey -> index table (linear probing, power-of-two capacity, load <= 1/2): one flat
// array instead of a node per junction
class CIndex {
  public:
    // the index of k, inserting v for a new key; second = inserted
    std::pair<size_t, bool> try_emplace(const CKey &k, size_t v) {
        if (2 * (n_ + 1) > slots_.size()) grow();
        size_t i = CKeyHash()(k) & (slots_.size() - 1);
        for (;; i = (i + 1) & (slots_.size() - 1)) {
            Slot &s = slots_[i];
            if (!s.used) { s.used = true; s.k = k; s.v = v; ++n_; return {v, true}; }
            if (s.k == k) return {s.v, false};
        }
    }
    const size_t *find(const CKey &k) const {
        if (slots_.empty()) return nullptr;
        for (size_t i = CKeyHash()(k) & (slots_.size() - 1);; i = (i + 1) & (slots_.size() - 1)) {
            const Slot &s = slots_[i];
            if (!s.used) return nullptr;
            if (s.k == k) return &s.v;
        }
    }
    size_t at(const CKey &k) const {
        const size_t *p = find(k);
        if (!p) throw std::out_of_range("CIndex::at");
        return *p;
    }
  private:
    struct Slot { CKey k; size_t v; bool used = false; };
    std::vector<Slot> slots_;
    size_t n_ = 0;
    void grow() {
        std::vector<Slot> old;
        old.swap(slots_);
        slots_.assign(old.empty() ? 1024 : 2 * old.size(), Slot{});
        n_ = 0;
        for (const Slot &s : old)
            if (s.used) try_emplace(s.k, s.v);
    }
};

struct Splice {                                // Splice (:766-806)
    int span = -1;                             // -1: a known site (junc_span None)
    int64_t cid = -1;                          // interned chrom (fc2_caller::ids), -1: not yet
    std::string chrom, strand, gtag;
    int64_t start = 0, end = 0;
    int64_t dist = 0;
    bool dist_bool = false;                    // -d 0: simple_match returns a bool (:865-871)
    int64_t ov = 0;
    int64_t n_hits = 1;
    Coord coord() const {
        return start < end ? Coord(chrom, start, end, strand) : Coord(chrom, end, start, strand);
    }
};

// min() over a Python list that may mix bools and ints: first minimal element wins
struct PyMin {
    bool has = false, is_bool = false;
    int64_t v = 0;
    void add(int64_t x, bool b) {
        if (!has || x < v) { has = true; v = x; is_bool = b; }
    }
    std::string str() const { return is_bool ? (v ? "True" : "False") : i2s(v); }
};

// A set of strings of which only the size is read (Hit.readnames / Hit.uniq): a short vector
// for the usual handful of members, a hash set past 16 (no per-hit hash table otherwise).
struct StrSet {
    std::vector<std::string> v;
    std::unique_ptr<std::unordered_set<std::string>> big;
    void insert(const std::string &s) {
        if (big) { big->insert(s); return; }
        for (const std::string &x : v)
            if (x == s) return;
        v.push_back(s);
        if (v.size() > 16) {
            big.reset(new std::unordered_set<std::string>(v.begin(), v.end()));
            v.clear();
            v.shrink_to_fit();
        }
    }
    size_t size() const { return big ? big->size() : v.size(); }
};

// Hit.uniq (:579-580, :590): the set of (read, rc(read)) of every spliced read; only
// len(uniq) / 2 is read.  Stored as the set C of canonical forms min(read, rc(read)) plus the number
// of palindromic members (read == rc(read)), so len(uniq) = 2|C| - palindromes exactly, with one
// string per distinct read instead of two.
struct CanonSet {
    StrSet canon;
    int64_t palindromes = 0;
    void insert(const std::string &read, const std::string &rc) {
        const bool pal = read == rc;
        const std::string &c = pal || read < rc ? read : rc;
        const size_t before = canon.size();
        canon.insert(c);
        if (pal && canon.size() != before) palindromes += 1;
    }
    int64_t size() const { return 2 * (int64_t)canon.size() - palindromes; }
};

struct Hit {                                   // Hit (:486-654)
    std::string name;
    Coord coord;
    int64_t n_reads = 0;
    StrSet readnames;
    CanonSet uniq;
    bool has_mq = false;
    int64_t mq_a = 0, mq_b = 0;                // max of mapquals_A / _B
    double n_weighted = 0.;
    int64_t n_spanned = 0;
    double n_uniq_bridges = 0.;
    PyMin edits, overlaps, n_hits;
    std::string signal = "NNNN", strandmatch = "NA";
    std::map<std::string, int64_t> flags;
    std::unordered_map<std::string, std::set<std::string>> read_flags;
    bool has_tissue = false;
    double tissue = 0.;
};

}  // namespace

struct fc2_caller {
    fc2_ingest *ing = nullptr;
    fc2_ingest_params ip{};
    std::string name, known_circ, known_lin;
    fc2_caller_opts o{};
    std::vector<int32_t> tid2chrom;
    const fc2_fasta *fasta = nullptr;
    bool eof = false;
    // Two sides that may run on two threads at once: fc2_caller_next forms chunks (ingest,
    // process_mate, the pairs) into the bf_* fields, fc2_caller_submit records the oldest queued chunk
    // (record_hits, tables, writers) from the plain fields.  They share only the queue (mutex) and
    // read-only state (options, genome map, reference names); each side has its own counters.
    std::vector<Frag> bf_frags;                 // the chunk being formed (next)
    std::vector<Span> bf_spans;
    std::string bf_arena;                       // read_part bytes
    std::vector<uint64_t> bf_off;
    std::vector<fc2_pair> bf_pairs;
    std::vector<Frag> frags;                    // the chunk being recorded (submit)
    std::vector<Span> spans;
    std::string arena;
    std::vector<uint64_t> b_off;
    std::vector<fc2_pair> b_pairs;
    // chunks handed out by fc2_caller_next and not yet submitted, oldest first: the caller may
    // read ahead (form chunk k+1 while chunk k is on the GPU or being recorded)
    struct Chunk {
        std::vector<Frag> frags;
        std::vector<Span> spans;
        std::string arena;
        std::vector<uint64_t> b_off;
        std::vector<fc2_pair> b_pairs;
    };
    std::deque<Chunk> queued;
    std::mutex qmu;
    // aggregation
    struct Storage {
        std::string prefix;
        std::deque<Hit> hits;                   // insertion (= dict) order; never relocated
        CIndex index;
        int64_t novel = 0;
    } st[2];                                    // 0 circ, 1 lin
    std::unordered_map<std::string, uint32_t> ids;    // interned chromosome / strand strings (submit side)
    std::vector<int64_t> tid_cid;                     // reference id -> interned chromosome (submit side)
    std::vector<std::pair<const char *, double>> N;   // the reference's counters, keyed by literal
                                                      // (merged by name into sorted keys on output)
    std::vector<std::pair<const char *, double>> N_in; // the same for the counters the next side bumps
    std::string out[3];                         // reads, multi, test text since the last take
    std::string rows_text;
    std::vector<std::pair<std::string, double>> counters_snapshot;
    uint64_t n_pairs = 0;
};

namespace {

void incN_into(std::vector<std::pair<const char *, double>> &N, const char *k, double v) {
    for (auto &kv : N)
        if (kv.first == k) { kv.second += v; return; }
    N.emplace_back(k, v);
}
// record side (fc2_caller_submit and the output functions)
void incN(fc2_caller *h, const char *k, double v = 1.) { incN_into(h->N, k, v); }
// next side (process_mate)
void incN_in(fc2_caller *h, const char *k, double v = 1.) { incN_into(h->N_in, k, v); }

uint32_t intern(fc2_caller *h, const std::string &v) {
    auto it = h->ids.find(v);
    if (it != h->ids.end()) return it->second;
    const uint32_t id = (uint32_t)h->ids.size();
    h->ids.emplace(v, id);
    return id;
}

uint32_t strand_id(fc2_caller *h, const std::string &strand) {
    if (strand.size() == 1 && (strand[0] == '+' || strand[0] == '-')) return strand[0] == '-' ? 1u : 0u;
    return 2u + intern(h, strand);
}

CKey coord_key(fc2_caller *h, const Coord &c) {
    return CKey{std::get<1>(c), std::get<2>(c), intern(h, std::get<0>(c)), strand_id(h, std::get<3>(c))};
}

// the same key straight from a Splice (Splice.coord, :801-806), without building the tuple
CKey coord_key(fc2_caller *h, const Splice &sp) {
    const uint32_t c = sp.cid >= 0 ? (uint32_t)sp.cid : intern(h, sp.chrom);
    return sp.start < sp.end ? CKey{sp.start, sp.end, c, strand_id(h, sp.strand)}
                             : CKey{sp.end, sp.start, c, strand_id(h, sp.strand)};
}

// ---- Hit / SpliceSiteStorage ----------------------------------------------------------
void hit_add(fc2_caller *h, Hit &t, const Splice &sp) {
    t.signal = sp.gtag;
    t.strandmatch = "N/A";
    if (h->o.stranded)   // Splice has no strandmatch attribute (:532-533)
        throw Fatal{FC2_E_FORMAT, "AttributeError: 'Splice' object has no attribute 'strandmatch'"};
    t.edits.add(sp.dist, sp.dist_bool);
    t.overlaps.add(sp.ov, false);
    t.n_hits.add(sp.n_hits, false);
    if (sp.span < 0) return;
    const Span &s = h->spans[sp.span];
    t.n_spanned += 1;
    t.n_weighted += s.weight;
    if (s.qA && s.qB) t.n_uniq_bridges += s.weight;
    if (!t.has_mq) { t.has_mq = true; t.mq_a = s.qA; t.mq_b = s.qB; }
    else { t.mq_a = std::max(t.mq_a, s.qA); t.mq_b = std::max(t.mq_b, s.qB); }
    return;
}

// the span-dependent part of Hit.add that needs the fragment's primary
void hit_add_read(fc2_caller *h, Hit &t, const Span &s, const Align &prim) {
    t.readnames.insert(prim.qname);
    const std::string &read = prim.seq;
    static thread_local std::string rc;
    rev_comp_into(read, rc);
    t.n_reads += 1;
    (void)h;
    t.has_tissue = true;
    t.tissue += s.weight;
    t.uniq.insert(read, rc);
}

Hit make_hit(fc2_caller *h, const std::string &name, const Splice &sp) {
    Hit t;
    t.name = name;
    t.coord = sp.coord();
    hit_add(h, t, sp);
    return t;
}

size_t storage_add(fc2_caller *h, int kind, const Splice &sp, const Align *prim) {
    auto &S = h->st[kind];
    const auto ins = S.index.try_emplace(coord_key(h, sp), S.hits.size());
    const size_t k = ins.first;
    if (ins.second) {                           // a new junction: named by first appearance (:684-686)
        S.novel += 1;
        char nm[64];
        snprintf(nm, sizeof nm, "_%s_%06lld", S.prefix.c_str(), (long long)S.novel);
        Hit &t = S.hits.emplace_back();
        t.name = h->name + nm;
        t.coord = sp.coord();
        hit_add(h, t, sp);
    } else {
        hit_add(h, S.hits[k], sp);
    }
    if (sp.span >= 0) hit_add_read(h, S.hits[k], h->spans[sp.span], *prim);
    return k;
}

void add_flag(Hit &t, const std::string &flag, const std::string &frag) {
    t.flags[flag] += 1;
    t.read_flags[frag].insert(flag);
}

std::vector<std::string> categories(fc2_caller *h, const Hit &t) {   // :601-654
    const auto &o = h->o;
    std::vector<std::string> cats;
    if (t.signal != "GTAG") cats.push_back("NON_CANONICAL");
    if (t.mq_a == 0 || t.mq_b == 0) cats.push_back("WARN_NON_UNIQUE_ANCHOR");
    if (t.n_uniq_bridges == 0) cats.push_back("WARN_NO_UNIQ_BRIDGES");
    if (t.n_hits.v > 1) cats.push_back("WARN_AMBIGUOUS_BP");
    const int64_t mov = t.overlaps.v, med = t.edits.v;
    if (mov == 0 && med == 0) {
    } else if (mov < 2 && med < 2) {
        cats.push_back("WARN_EXT_1MM");
    } else if (mov >= 2 || med >= 2) {
        cats.push_back("WARN_EXT_2MM+");
    }
    const int64_t start = std::get<1>(t.coord), end = std::get<2>(t.coord);
    if (end - start < o.short_threshold) cats.push_back("SHORT");
    else if (end - start > o.huge_threshold) cats.push_back("HUGE");
    int64_t unbroken = 0, unwarned = 0;
    double total = 0.;
    for (const auto &kv : t.read_flags) {
        total += 1.;
        if (!kv.second.count("BROKEN_SEGMENTS")) unbroken += 1;
        for (const auto &w : kv.second)
            if (w.compare(0, 4, "WARN") != 0) unwarned += 1;
    }
    if (total) {
        if (!unbroken) cats.push_back("WARN_ALWAYS_BROKEN");
        if (!unwarned) cats.push_back("WARN_ALWAYS_WARN");
    }
    return cats;
}

std::string join(const std::vector<std::string> &v, const char *sep) {
    std::string r;
    for (size_t k = 0; k < v.size(); ++k) {
        if (k) r += sep;
        r += v[k];
    }
    return r;
}

void storage_rows(fc2_caller *h, int kind, std::string &outs) {           // :690-730
    const auto &o = h->o;
    for (const Hit &t : h->st[kind].hits) {
        if (!t.n_reads) continue;
        const int64_t qa = t.mq_a, qb = t.mq_b;
        if (o.halfunique) {
            if (qa < o.min_uniq_qual && qb < o.min_uniq_qual) { incN(h, "anchor_not_uniq"); continue; }
        } else if (qa < o.min_uniq_qual || qb < o.min_uniq_qual) {
            incN(h, "anchor_not_uniq");
            continue;
        }
        if (t.n_uniq_bridges == 0 && !o.report_nobridges) { incN(h, "no_uniq_bridges"); continue; }
        // the 22 columns of find_circ.py:712-730, appended in place
        auto col = [&](const std::string &v) { outs += v; outs += '\t'; };
        col(std::get<0>(t.coord));
        col(i2s(std::get<1>(t.coord)));
        col(i2s(std::get<2>(t.coord)));
        col(t.name);
        col(i2s((int64_t)t.readnames.size()));
        col(std::get<3>(t.coord));
        col(py2_float(t.n_weighted));
        col(i2s(t.n_spanned));
        col(i2s(t.uniq.size() / 2));
        col(py2_float(t.n_uniq_bridges));
        col(i2s(qa));
        col(i2s(qb));
        col(t.has_tissue ? h->name : std::string());
        col(t.has_tissue ? py2_float(t.tissue) : std::string());
        col(t.edits.str());
        col(t.overlaps.str());
        col(t.n_hits.str());
        col(t.signal);
        col(t.strandmatch);
        std::vector<std::string> cats = categories(h, t);
        std::sort(cats.begin(), cats.end());
        col(join(cats, ","));
        if (!t.flags.empty()) {
            bool first = true;
            for (const auto &kv : t.flags) { if (!first) outs += ','; outs += kv.first; first = false; }
            outs += '\t';
            first = true;
            for (const auto &kv : t.flags) { if (!first) outs += ','; outs += i2s(kv.second); first = false; }
        } else {
            outs += "N/A\t0";
        }
        outs += '\n';
    }
}

// known sites (:657-689): Splice(None, chrom, start, end, sense, 10, 10, 'NNNN')
uint64_t load_known(fc2_caller *h, int kind, const std::string &path) {
    if (path.empty()) return 0;
    FILE *f = fopen(path.c_str(), "r");
    if (!f) throw Fatal{FC2_E_IO, "IOError: [Errno 2] No such file or directory: " + py_repr(path)};
    auto &S = h->st[kind];
    uint64_t n = 0;
    std::string line;
    char buf[65536];
    while (fgets(buf, sizeof buf, f)) {
        line = buf;
        if (!line.empty() && line[0] == '#') continue;
        while (!line.empty() && isspace((unsigned char)line.back())) line.pop_back();   // rstrip()
        std::vector<std::string> fl;
        size_t p = 0;
        for (;;) {
            const size_t t = line.find('\t', p);
            fl.push_back(line.substr(p, t == std::string::npos ? std::string::npos : t - p));
            if (t == std::string::npos) break;
            p = t + 1;
        }
        if (fl.size() < 6) {
            fclose(f);
            throw Fatal{FC2_E_FORMAT, "ValueError: need more than " + i2s((int64_t)fl.size()) + " values to unpack"};
        }
        Splice sp;
        sp.chrom = fl[0];
        char *e1 = nullptr, *e2 = nullptr;
        sp.start = strtoll(fl[1].c_str(), &e1, 10);
        sp.end = strtoll(fl[2].c_str(), &e2, 10);
        if (fl[1].empty() || *e1 || fl[2].empty() || *e2) {
            fclose(f);
            throw Fatal{FC2_E_FORMAT, "ValueError: invalid literal for int() with base 10"};
        }
        sp.strand = fl[5];
        sp.dist = 10;
        sp.ov = 10;
        sp.gtag = "NNNN";
        const CKey key = coord_key(h, sp);
        Hit t = make_hit(h, fl[3], sp);
        const auto ins = S.index.try_emplace(key, S.hits.size());
        if (ins.second)                         // a repeated coordinate keeps its first dict position
            S.hits.push_back(std::move(t));
        else
            S.hits[ins.first] = std::move(t);
        ++n;
    }
    fclose(f);
    return n;
}

// ---- fragments ----------------------------------------------------------------------
std::string chrom_of(fc2_caller *h, int32_t tid) {               // fast_chrom_lookup (:471-477)
    const char *nm = fc2_ingest_ref_name(h->ing, tid);
    if (tid < 0 || !nm) throw Fatal{FC2_E_FORMAT, "ValueError: reference id " + i2s(tid) + " out of range"};
    return nm;
}

int64_t uniqness(const Rec &a) {                                  // :809-819
    if (!a.has_as) throw Fatal{FC2_E_KEY, "KeyError: \"tag 'AS' not present\""};
    if (!a.as_int || (a.has_xs && !a.xs_int))
        throw Fatal{FC2_E_FORMAT, "native caller: AS / XS tags must be integers (use --python-caller)"};
    return a.as - (a.has_xs ? a.xs : 0);
}

const char *kNoneLen = "TypeError: object of type 'NoneType' has no len()";

// process_mate (:1492-1527) with adjacent_segment_pairs (:1058-1140)
void process_mate(fc2_caller *h, const Mate &m, int mi, Frag &fr) {
    const Rec &prim = m.recs[0];
    if (m.proper.size() < 2) {
        incN_in(h, "unspliced_mates");
        fr.unspliced.push_back(make_align(prim));
        return;
    }
    if (!prim.has_seq) throw Fatal{FC2_E_FORMAT, kNoneLen};      // L = len(mate.full_seq)
    const int64_t L = (int64_t)prim.seq.size();
    const size_t n = m.proper.size();
    const double weight = 1. / ((double)n - 1.);
    std::vector<int64_t> starts(n), ends(n);
    for (size_t k = 0; k < n; ++k) {
        const Rec &s = m.recs[m.proper[k]];
        if (s.qlen < 0) throw Fatal{FC2_E_FORMAT, kNoneLen};     // len(s.query)
        starts[k] = s.astart;
        ends[k] = s.astart + s.qlen;
    }
    std::vector<size_t> order(n);
    for (size_t k = 0; k < n; ++k) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return starts[a] < starts[b]; });
    int64_t min_s = L, max_e = 0;
    for (size_t k = 0; k + 1 < n; ++k) {
        const size_t a = order[k], b = order[k + 1];
        if (ends[a] - starts[a] < h->o.asize || ends[b] - starts[b] < h->o.asize) {
            incN_in(h, "seg_too_short_skip");
            continue;
        }
        const Rec &A = m.recs[m.proper[a]], &B = m.recs[m.proper[b]];
        const int64_t q_start = std::min(starts[a], starts[b]), q_end = std::max(ends[a], ends[b]);
        (void)chrom_of(h, A.tid);
        Span s;
        s.mate = mi;
        s.tid = A.tid;
        const int64_t ua = uniqness(A), ub = uniqness(B);
        if (A.aend < 0) throw Fatal{FC2_E_FORMAT, "TypeError: unsupported operand type(s) for -: 'int' and 'NoneType'"};
        s.circ = B.pos - A.aend < 0;
        s.a_pos = A.pos;
        s.b_aend = B.aend;
        s.weight = weight;
        s.uniq = std::min(ua, ub);
        s.qA = s.circ ? ub : ua;
        s.qB = s.circ ? ua : ub;
        s.a_rev = s.circ ? B.reverse() : A.reverse();
        // read_part = primary.seq[q_start:q_end] (Python slice)
        const int64_t lo = std::max<int64_t>(0, std::min(q_start, L)), hi = std::max(lo, std::min(q_end, L));
        s.read_off = h->bf_arena.size();
        s.read_len = (uint32_t)(hi - lo);
        h->bf_arena.append(prim.seq, (size_t)lo, (size_t)(hi - lo));
        h->bf_spans.push_back(s);
        (s.circ ? fr.circ : fr.lin).push_back((int)h->bf_spans.size() - 1);
        min_s = std::min(min_s, q_start);
        max_e = std::max(max_e, q_end);
    }
    if (max_e < L - h->o.asize || min_s > h->o.asize) {
        for (size_t k = 1; k < m.recs.size(); ++k)
            if (m.recs[k].tid != prim.tid) fr.broken.push_back(make_align(m.recs[k]));
        for (size_t k = 1; k < m.recs.size(); ++k)
            if (m.recs[k].tid == prim.tid && m.recs[k].reverse() != prim.reverse())
                fr.broken.push_back(make_align(m.recs[k]));
    }
}

int on_fragment(fc2_caller *h, const Mate *m1, const Mate *m2) {
    Frag fr;
    fr.name = m2->recs[0].qname;               // Fragment(mate2.primary.qname, ...)
    const Mate *ms[2] = {m1, m2};
    const size_t span0 = h->bf_spans.size(), arena0 = h->bf_arena.size();
    for (int k = 0; k < 2; ++k) {
        if (!ms[k]) continue;
        fr.has[k] = true;
        fr.prim[k] = make_align(ms[k]->recs[0]);
        process_mate(h, *ms[k], k, fr);
    }
    if ((fr.circ.empty() && h->o.nolinear) || (fr.circ.empty() && fr.lin.empty())) {
        h->bf_spans.resize(span0);                // not pending: its spans are never evaluated
        h->bf_arena.resize(arena0);
        return FC2_OK;
    }
    h->bf_frags.push_back(std::move(fr));
    return FC2_OK;
}

// ---- evaluation results -> Splice lists (hotpath.decode_splices) -------------------------
const char kCode[] = "ACGTN";

std::string rev_comp4(const std::string &g) { return rev_comp(g); }

struct Eval {
    int err = 0;                               // 0 ok, else a Fatal raised by find_breakpoints
    std::string msg;
    std::vector<Splice> ties;
};

int score_of(const fc2_caller *h, const std::string &sig, int64_t dist, int64_t ov, const std::string &strand,
             bool prim_rev) {
    int64_t sc = (sig == "GTAG" ? 20 : 0) - dist * 10 - ov;
    if (h->o.strandpref && strand == (prim_rev ? "-" : "+")) sc += 100;
    return (int)sc;
}

Eval decode(fc2_caller *h, int si, const fc2_result &r, const uint64_t *tiemask, uint32_t tw, uint64_t stride) {
    Eval ev;
    const Span &s = h->spans[si];
    const fc2_pair &pr = h->b_pairs[(size_t)s.eval];
    const std::string chrom = chrom_of(h, s.tid);
    if ((size_t)s.tid >= h->tid_cid.size()) h->tid_cid.resize((size_t)s.tid + 1, -1);
    int64_t &cid = h->tid_cid[(size_t)s.tid];
    if (cid < 0) cid = intern(h, chrom);
    if (pr.flags & FC2_PAIR_SKIP) {            // chromosome missing from the genome (get_data, :193)
        ev.err = FC2_E_KEY;
        ev.msg = "KeyError: " + py_repr(chrom);
        return ev;
    }
    if (r.info & FC2_RES_ERR_KEY) {
        ev.err = FC2_E_KEY;
        ev.msg = "KeyError: splice signal with a byte outside ACGTN (find_circ.py:927)";
        return ev;
    }
    if (r.info & FC2_RES_ERR_WIN) {
        ev.err = FC2_E_FORMAT;
        // numpy 1.x (Python 2): unequal-length `!=` gives the scalar True, whose .sum() fails (:861-863)
        ev.msg = "AttributeError: 'bool' object has no attribute 'sum'";
        return ev;
    }
    if (r.best_x < 0) return ev;
    const int64_t e = h->o.asize - h->o.margin;
    const int64_t L = pr.read_len, l = L - 2 * e, x = r.best_x;
    const bool bs = pr.flags & FC2_PAIR_BACKSPLICE, prim_rev = pr.flags & FC2_PAIR_PRIMARY_REV;
    auto coords = [&](int64_t xx, int64_t &st, int64_t &en) {
        const int64_t s0 = pr.b_aend - e - l + xx, e0 = pr.a_pos + e + xx + 1;
        st = std::min(s0, e0);
        en = std::max(s0, e0);
        if (bs) en -= 1; else st -= 1;
    };
    std::string g;
    for (int k = 0; k < 4; ++k) g += kCode[((r.info & FC2_RES_GTAG_MASK) >> FC2_RES_GTAG_SHIFT >> (3 * k)) & 7];
    Splice best;
    best.span = si;
    best.chrom = chrom;
    best.cid = cid;
    coords(x, best.start, best.end);
    best.strand = (r.info & FC2_RES_MINUS) ? "-" : "+";
    best.gtag = best.strand == "-" ? rev_comp4(g) : g;
    best.dist = r.dist;
    best.dist_bool = h->o.maxdist == 0;
    if (best.dist_bool) best.dist = 0;
    best.ov = r.ov;
    best.n_hits = r.n_ties;
    const int best_score = score_of(h, best.gtag, r.dist, r.ov, best.strand, prim_rev);
    if (!(h->o.allhits && r.n_ties > 1)) {
        ev.ties.push_back(best);
        return ev;
    }
    // all ties in (x asc, '+' before '-') order from the tie mask (hotpath._expand_ties)
    const uint32_t half = tw / 2;
    for (int64_t xx = 0; xx <= l; ++xx) {
        const uint32_t k = (uint32_t)(xx >> 6), b = (uint32_t)(xx & 63);
        for (int strand = 0; strand < 2; ++strand) {
            const uint32_t row = strand ? half + k : k;
            if (!((tiemask[(uint64_t)row * stride + (uint64_t)s.eval] >> b) & 1ull)) continue;
            Splice t;
            t.span = si;
            t.chrom = chrom;
            t.cid = cid;
            coords(xx, t.start, t.end);
            t.strand = strand ? "-" : "+";
            int64_t ov = 0;
            if (h->o.margin) {
                if (xx < h->o.margin) ov = h->o.margin - xx;
                if (l - xx < h->o.margin) ov = h->o.margin - (l - xx);
            }
            t.ov = ov;
            std::string sig;
            if (h->o.noncanonical) {
                std::string wg;
                if (!h->fasta) {
                    wg = "NNNN";
                } else {
                    const int64_t a0 = pr.a_pos + e, b1 = pr.b_aend - e;
                    auto window = [&](int64_t lo, int64_t hi) {
                        std::string w((size_t)std::max<int64_t>(0, hi - lo) + 16, '\0');
                        int64_t len = 0;
                        int rc = fc2_fasta_get_upper(h->fasta, (int)pr.chrom, lo, hi, (uint8_t *)&w[0],
                                                     (int64_t)w.size(), &len);
                        if (rc == FC2_OK && len > (int64_t)w.size()) {
                            w.assign((size_t)len, '\0');
                            rc = fc2_fasta_get_upper(h->fasta, (int)pr.chrom, lo, hi, (uint8_t *)&w[0],
                                                     (int64_t)w.size(), &len);
                        }
                        if (rc != FC2_OK) throw Fatal{rc, fc2_last_error()};
                        w.resize((size_t)len);
                        return w;
                    };
                    const std::string A = window(a0, a0 + l + 2), B = window(b1 - l - 2, b1);
                    auto sl = [](const std::string &w, int64_t p) {   // w[p:p+2]
                        if (p >= (int64_t)w.size()) return std::string();
                        return w.substr((size_t)p, 2);
                    };
                    wg = sl(A, xx) + sl(B, xx);
                }
                sig = strand ? rev_comp4(wg) : wg;
            } else {
                sig = "GTAG";
            }
            t.gtag = sig;
            const int64_t canon = sig == "GTAG" ? 20 : 0;
            const int64_t sp = (h->o.strandpref && t.strand == (prim_rev ? "-" : "+")) ? 100 : 0;
            int64_t num = canon - ov + sp - best_score;
            int64_t d = num >= 0 ? num / 10 : -((-num + 9) / 10);           // Python floor division
            t.dist = h->o.maxdist == 0 ? 0 : d;
            t.dist_bool = h->o.maxdist == 0;
            t.n_hits = best.n_hits;
            ev.ties.push_back(t);
        }
    }
    return ev;
}


// ---- record_hits (:1276-1439) and its writers ---------------------------------------------
const int64_t kNone = INT64_MIN;               // an alignment end that is None

struct UCoord {                                // (chrom, pos, aend, strand) of an unspliced / broken alignment
    std::string chrom;
    int64_t pos, aend;
    std::string strand;
    bool operator<(const UCoord &b) const {
        return std::tie(chrom, pos, aend, strand) < std::tie(b.chrom, b.pos, b.aend, b.strand);
    }
    bool operator==(const UCoord &b) const {
        return chrom == b.chrom && pos == b.pos && aend == b.aend && strand == b.strand;
    }
};

std::string none_or(int64_t v) { return v == kNone ? std::string("None") : i2s(v); }

std::string repr_coord(const std::string &c, int64_t s, int64_t e, const std::string &st) {   // str(tuple)
    return "(" + py_repr(c) + ", " + none_or(s) + ", " + none_or(e) + ", " + py_repr(st) + ")";
}

int64_t need_int(int64_t v) {                  // an int operand of '%d' or '-' (None fails as in Python)
    if (v == kNone) throw Fatal{FC2_E_FORMAT, "TypeError: %d format: a number is required, not NoneType"};
    return v;
}

// parse_truth (:1148-1200)
void parse_truth(const std::string &align_str, bool stranded, std::set<Coord> &lin, std::set<Coord> &circ,
                 std::set<Coord> &unspl) {
    auto split = [](const std::string &s, char c) {
        std::vector<std::string> v;
        size_t p = 0;
        for (;;) {
            const size_t t = s.find(c, p);
            v.push_back(s.substr(p, t == std::string::npos ? std::string::npos : t - p));
            if (t == std::string::npos) break;
            p = t + 1;
        }
        return v;
    };
    auto to_int = [](const std::string &s) {
        char *e = nullptr;
        const long long v = strtoll(s.c_str(), &e, 10);
        if (s.empty() || *e) throw Fatal{FC2_E_FORMAT, "ValueError: invalid literal for int() with base 10: " + py_repr(s)};
        return (int64_t)v;
    };
    for (const std::string &mate_str : split(align_str, '|')) {
        bool spliced = false, has_chrom = false;
        std::string chrom, strand;
        int64_t start = 0, end = 0;
        bool has_start = false;
        for (const std::string &code : split(mate_str, ';')) {
            const std::vector<std::string> parts = split(code, ':');
            const std::string &op = parts[0];
            auto part = [&](size_t k) -> const std::string & {
                if (k >= parts.size()) throw Fatal{FC2_E_FORMAT, "IndexError: list index out of range"};
                return parts[k];
            };
            auto need_start = [&]() {
                if (!has_start) throw Fatal{FC2_E_FORMAT, "TypeError: unsupported operand type(s) for +: 'int' and 'NoneType'"};
            };
            if (op == "O") {
                chrom = part(1); start = to_int(part(2)); strand = part(3);
                has_chrom = true; has_start = true;
                end = start;
            } else if (op == "M") {
                need_start();
                end += to_int(part(1));
            } else if (op == "LS" || op == "CS") {
                const int64_t a = to_int(part(1)), b = to_int(part(2));
                need_start();
                const Coord c(chrom, a + start, b + start, strand);
                (op == "LS" ? lin : circ).insert(c);
                spliced = true;
                end = op == "LS" ? b + start : a + start;
            }
        }
        if (!spliced && has_chrom && !chrom.empty()) unspl.insert(Coord(chrom, start, end, stranded ? strand : "*"));
    }
}

std::string test_row(fc2_caller *h, const Frag &fr, const std::set<Coord> &lin_coords,
                     const std::set<Coord> &circ_coords, const std::vector<UCoord> &unspliced,
                     const std::vector<UCoord> &broken) {                     // :1202-1273
    const std::string &name = fr.name;
    const size_t p = name.rfind("___");
    if (name.find("___") == std::string::npos) return name + "\tN/A\tN/A\tN/A\tN/A\n";
    std::set<Coord> lin_ref, circ_ref, un_ref;
    parse_truth(name.substr(p + 3), h->o.stranded, lin_ref, circ_ref, un_ref);
    std::set<Coord> un_got;
    for (const UCoord &u : unspliced) un_got.insert(Coord(u.chrom, u.pos, u.aend, u.strand));
    std::string row = name;
    struct K { const char *kind, *ok; const std::set<Coord> *ref, *got; };
    const K ks[3] = {{"LINEAR_JUNCTIONS", "LIN_OK", &lin_ref, &lin_coords},
                     {"CIRCULAR_JUNCTIONS", "CIRC_OK", &circ_ref, &circ_coords},
                     {"UNSPLICED", "UNSPLICED_OK", &un_ref, &un_got}};
    for (const K &k : ks) {
        std::vector<std::string> fl;
        std::vector<std::string> miss, spur;
        for (const Coord &c : *k.ref)
            if (!k.got->count(c)) miss.push_back(repr_coord(std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c)));
        for (const Coord &c : *k.got)
            if (!k.ref->count(c)) spur.push_back(repr_coord(std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c)));
        if (!miss.empty()) fl.push_back(std::string("MISSED_") + k.kind + ":" + join(miss, ","));
        if (!spur.empty()) fl.push_back(std::string("SPURIOUS_") + k.kind + ":" + join(spur, ","));
        std::sort(fl.begin(), fl.end());
        row += '\t';
        row += !fl.empty() ? join(fl, ";") : (!k.ref->empty() ? std::string(k.ok) : std::string("N/A"));
    }
    row += '\t';
    if (!broken.empty()) {
        std::set<UCoord> bs(broken.begin(), broken.end());
        std::vector<std::string> v;
        for (const UCoord &b : bs) v.push_back(repr_coord(b.chrom, b.pos, b.aend, b.strand));
        row += "BROKEN_SEGMENTS:" + join(v, ";");
    } else {
        row += "N/A";
    }
    return row + "\n";
}

std::string multi_row(fc2_caller *h, const Frag &fr, const Hit &circ, const std::set<Coord> &lin_cons,
                      const std::set<Coord> &lin_incons, const std::set<UCoord> &un_cons,
                      const std::set<UCoord> &un_incons) {                    // :733-763
    (void)h;
    const int64_t score = (int64_t)lin_cons.size() - 10 * (int64_t)lin_incons.size() + (int64_t)un_cons.size() -
                          10 * (int64_t)un_incons.size();
    std::vector<std::string> cols = {std::get<0>(circ.coord), i2s(std::get<1>(circ.coord)),
                                     i2s(std::get<2>(circ.coord)), "ME:" + circ.name, i2s(score),
                                     std::get<3>(circ.coord), fr.name};
    std::vector<std::string> v;
    for (const Coord &c : lin_cons) v.push_back(i2s(std::get<1>(c)) + "-" + i2s(std::get<2>(c)));
    cols.push_back(v.empty() ? "NO_LIN_CONS" : join(v, ","));
    v.clear();
    for (const Coord &c : lin_incons)
        v.push_back("[" + std::get<0>(c) + ":" + i2s(std::get<1>(c)) + "-" + i2s(std::get<2>(c)) + "]");
    cols.push_back(v.empty() ? "NO_LIN_INCONS" : join(v, ","));
    v.clear();
    for (const UCoord &c : un_cons) v.push_back(i2s(need_int(c.pos)) + "-" + i2s(need_int(c.aend)));
    cols.push_back(v.empty() ? "NO_UNSPLICED_CONS" : join(v, ","));
    v.clear();
    for (const UCoord &c : un_incons) v.push_back("[" + c.chrom + ":" + i2s(need_int(c.pos)) + "-" + i2s(need_int(c.aend)) + "]");
    cols.push_back(v.empty() ? "NO_UNSPLICED_INCONS" : join(v, ","));
    return join(cols, "\t") + "\n";
}

// the evaluation results of the pending chunk
struct Results {
    const fc2_result *res;
    const uint64_t *tiemask;
    uint32_t tw;
    uint64_t stride;
};

const std::vector<Splice> &find_breakpoints(fc2_caller *h, int si, const Results &R,
                                            std::unordered_map<int, Eval> &cache) {
    auto it = cache.find(si);
    if (it == cache.end()) it = cache.emplace(si, decode(h, si, R.res[h->spans[si].eval], R.tiemask, R.tw, R.stride)).first;
    if (it->second.err) throw Fatal{it->second.err, it->second.msg};
    return it->second.ties;
}

using HitRef = std::pair<int, size_t>;          // (storage, index)

void record_hits(fc2_caller *h, Frag &fr, const Results &R, std::set<HitRef> &junctions,
                 std::set<std::string> &warns) {
    const auto &o = h->o;
    std::unordered_map<int, Eval> cache;
    std::set<Coord> circ_coords;
    HitRef circ{-1, 0};
    for (int si : fr.circ) {
        const Span &span = h->spans[si];
        if (!(span.uniq >= o.min_uniq_qual)) { incN(h, "circ_junc_not_unique"); continue; }
        const std::vector<Splice> &splices = find_breakpoints(h, si, R, cache);
        if (splices.empty()) {
            incN(h, "circ_no_bp");
            warns.insert("WARN_UNRESOLVED_EXTRA_BACKSPLICE");
            continue;
        }
        incN(h, "circ_spliced");
        const size_t n = o.allhits ? splices.size() : 1;
        for (size_t k = 0; k < n; ++k) {
            const size_t idx = storage_add(h, 0, splices[k], &fr.prim[span.mate]);
            circ = HitRef(0, idx);
            circ_coords.insert(h->st[0].hits[idx].coord);
            junctions.insert(circ);
        }
    }
    if (circ_coords.size() > 1) {
        for (const Coord &c : circ_coords) {
            warns.insert("WARN_MULTI_BACKSPLICE");
            const size_t idx = h->st[0].index.at(coord_key(h, c));
            add_flag(h->st[0].hits[idx], "WARN_MULTI_BACKSPLICE", fr.name);
            junctions.insert(HitRef(0, idx));
        }
        return;
    }
    if (circ_coords.empty() && o.nolinear) return;
    int64_t circ_start = 0, circ_end = 0;
    int circ_span = -1;
    if (!circ_coords.empty()) {
        const Coord &cc = h->st[0].hits[circ.second].coord;
        circ_start = std::get<1>(cc);
        circ_end = std::get<2>(cc);
        circ_span = fr.circ[0];
        if (fr.circ.size() > 1) warns.insert("SUPPORT_CLOSURE");
    }
    std::set<Coord> lin_cons, lin_incons, lin_coords;
    for (int si : fr.lin) {
        const Span &span = h->spans[si];
        if (!(span.uniq >= o.min_uniq_qual)) { incN(h, "lin_junc_not_unique"); continue; }
        const std::vector<Splice> &splices = find_breakpoints(h, si, R, cache);
        if (splices.empty()) {
            incN(h, "lin_no_bp");
            warns.insert("WARN_UNRESOLVED_LINSPLICE");
            continue;
        }
        incN(h, "lin_spliced");
        const size_t n = o.allhits ? splices.size() : 1;
        for (size_t k = 0; k < n; ++k) {
            const Splice &sp = splices[k];
            const size_t idx = storage_add(h, 1, sp, &fr.prim[span.mate]);
            junctions.insert(HitRef(1, idx));
            lin_coords.insert(h->st[1].hits[idx].coord);
            if (!circ_coords.empty()) {
                if (sp.start <= circ_start || sp.end >= circ_end) {
                    warns.insert("WARN_OUTSIDE_SPLICE_JUNCTION");
                    lin_incons.insert(sp.coord());
                } else {
                    lin_cons.insert(sp.coord());
                    warns.insert("SUPPORT_INSIDE_SPLICE_JUNCTION");
                }
            }
        }
    }
    if (o.test) {
        auto coords = [&](const Align &a) {
            const std::string s = o.stranded ? (a.rev ? "-" : "+") : "*";
            return UCoord{chrom_of(h, a.tid), a.pos, a.aend < 0 ? kNone : a.aend, s};
        };
        std::vector<UCoord> un, br;
        for (const Align &a : fr.unspliced) un.push_back(coords(a));
        for (const Align &a : fr.broken) br.push_back(coords(a));
        h->out[2] += test_row(h, fr, lin_coords, circ_coords, un, br);
    }
    if (!circ_coords.empty()) {
        std::set<UCoord> un_cons, un_incons;
        const int32_t circ_tid = fr.prim[h->spans[circ_span].mate].tid;
        for (const Align &a : fr.unspliced) {
            const UCoord c{chrom_of(h, a.tid), a.pos, a.aend < 0 ? kNone : a.aend, "*"};
            if (circ_tid != a.tid) {
                warns.insert("WARN_OTHER_CHROM_MATE");
                un_incons.insert(c);
            } else if (a.pos + o.asize <= circ_start || need_int(c.aend) - o.asize >= circ_end) {
                warns.insert("WARN_OUTSIDE_MATE");
                un_incons.insert(c);
            } else {
                warns.insert("SUPPORT_INSIDE_MATE");
                un_cons.insert(c);
            }
        }
        if (!fr.broken.empty()) warns.insert("BROKEN_SEGMENTS");
        if ((!un_cons.empty() || !un_incons.empty() || !lin_cons.empty() || !lin_incons.empty()) && o.multi_events &&
            o.write_multi)
            h->out[1] += multi_row(h, fr, h->st[0].hits[circ.second], lin_cons, lin_incons, un_cons, un_incons);
        for (const std::string &w : warns) add_flag(h->st[0].hits[circ.second], w, fr.name);
    }
}

void write_read(fc2_caller *h, const Align &m, const std::set<HitRef> &junctions,
                const std::set<std::string> &flags) {                          // :1442-1447
    if (!h->o.write_reads) return;
    std::vector<std::string> names;
    for (const HitRef &j : junctions) names.push_back(h->st[j.first].hits[j.second].name);
    std::sort(names.begin(), names.end());
    const std::string name = m.qname + " " + join(names, ",") + " " +
                             join(std::vector<std::string>(flags.begin(), flags.end()), ",");
    std::string &o = h->out[0];
    o += '@'; o += name; o += '\n';
    o += m.has_seq ? m.seq : std::string("None"); o += "\n+";
    o += name; o += '\n';
    o += m.has_qual ? m.qual : std::string("None"); o += '\n';
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
extern "C" int fc2_caller_open(const char *path, int is_bam, const fc2_caller_opts *opts, fc2_caller **out) {
    if (!path || !opts || !out) return fc2::fail(FC2_E_PARAM, "fc2_caller_open: null argument");
    *out = nullptr;
    fc2_ingest *ing = nullptr;
    int rc = fc2_ingest_open(path, is_bam, &ing);
    if (rc) return rc;
    fc2_caller *h = new fc2_caller();
    h->ing = ing;
    h->o = *opts;
    h->name = opts->name ? opts->name : "unknown";
    h->known_circ = opts->known_circ ? opts->known_circ : "";
    h->known_lin = opts->known_lin ? opts->known_lin : "";
    h->o.name = h->o.known_circ = h->o.known_lin = nullptr;
    if (h->o.chunksize == 0) h->o.chunksize = 100000;
    h->ip.asize = opts->asize;
    h->ip.nolinear = opts->nolinear;
    h->ip.noop = opts->noop;
    h->st[0].prefix = "circ";
    h->st[1].prefix = "lin";
    *out = h;
    return FC2_OK;
}

extern "C" int fc2_caller_set_genome(fc2_caller *h, const int32_t *tid_to_chrom, int32_t n_tid, const fc2_fasta *fasta,
                                     uint64_t *n_known_circ, uint64_t *n_known_lin) {
    if (!h || (n_tid > 0 && !tid_to_chrom)) return fc2::fail(FC2_E_PARAM, "fc2_caller_set_genome: bad arguments");
    h->tid2chrom.assign(tid_to_chrom, tid_to_chrom + (n_tid > 0 ? n_tid : 0));
    h->fasta = fasta;
    try {
        const uint64_t kc = load_known(h, 0, h->known_circ);
        const uint64_t kl = load_known(h, 1, h->known_lin);
        if (n_known_circ) *n_known_circ = kc;
        if (n_known_lin) *n_known_lin = kl;
    } catch (const Fatal &f) {
        return fc2::fail(f.code, f.msg);
    }
    return FC2_OK;
}

extern "C" fc2_ingest *fc2_caller_ingest(fc2_caller *h) { return h ? h->ing : nullptr; }

extern "C" void fc2_caller_close(fc2_caller *h) {
    if (!h) return;
    fc2_ingest_close(h->ing);
    delete h;
}

extern "C" int fc2_caller_next(fc2_caller *h, fc2_caller_batch *b, int *eof) {
    if (!h || !b) return fc2::fail(FC2_E_PARAM, "fc2_caller_next: null argument");
    {
        std::lock_guard<std::mutex> lk(h->qmu);
        if (h->queued.size() >= FC2_CALLER_MAX_QUEUED)
            return fc2::fail(FC2_E_PARAM, "fc2_caller_next: too many chunks not submitted");
    }
    h->bf_frags.clear();
    h->bf_spans.clear();
    h->bf_arena.clear();
    h->bf_off.clear();
    h->bf_pairs.clear();
    Fatal err{0, ""};
    const fc2::ing::FragSink sink = [&](const Mate *m1, const Mate *m2, bool) -> int {
        try {
            return on_fragment(h, m1, m2);
        } catch (const Fatal &f) {
            err = f;
            return f.code ? f.code : FC2_E_FORMAT;
        }
    };
    while (!h->eof && h->bf_frags.size() < h->o.chunksize) {
        int e = 0;
        const int rc = fc2::ing::pull(h->ing, &h->ip, h->o.chunksize, sink, &e);
        if (rc) return err.code ? fc2::fail(err.code, err.msg) : rc;
        h->eof = e != 0;
    }
    // the spans record_hits will evaluate, in fragment order (Caller._flush)
    for (const Frag &fr : h->bf_frags) {
        for (int pass = 0; pass < 2; ++pass) {
            for (int si : pass ? fr.lin : fr.circ) {
                Span &s = h->bf_spans[si];
                if (!(s.uniq >= h->o.min_uniq_qual)) continue;
                fc2_pair pr{};
                pr.a_pos = (int32_t)s.a_pos;
                pr.b_aend = (int32_t)s.b_aend;
                const int32_t c = (s.tid >= 0 && s.tid < (int32_t)h->tid2chrom.size()) ? h->tid2chrom[s.tid] : -1;
                pr.chrom = c < 0 ? 0u : (uint32_t)c;
                pr.read_len = (uint16_t)std::min<uint32_t>(s.read_len, 65535u);
                if (s.b_aend < 0)               // align_B.aend is None: packing the pair fails (int(None))
                    return fc2::fail(FC2_E_FORMAT, "TypeError: int() argument must be a string, a bytes-like object "
                                                   "or a number, not 'NoneType'");
                pr.flags = (uint8_t)((s.circ ? FC2_PAIR_BACKSPLICE : 0) |
                                     (fr.prim[s.mate].rev ? FC2_PAIR_PRIMARY_REV : 0) | (c < 0 ? FC2_PAIR_SKIP : 0));
                s.eval = (int64_t)h->bf_pairs.size();
                h->bf_pairs.push_back(pr);
                h->bf_off.push_back(s.read_off);
            }
        }
    }
    for (const Span &s : h->bf_spans)
        if (s.eval >= 0 && s.read_len > FC2_MAX_READ_LEN)
            return fc2::fail(FC2_E_RANGE, "read_part longer than " + std::to_string(FC2_MAX_READ_LEN) +
                                              " bases (fc2_result.best_x is 16-bit)");
    h->n_pairs += h->bf_pairs.size();
    h->bf_arena.append(16, '\0');                 // readers of the batch may load whole words past the end
    fc2_caller::Chunk c;
    c.frags.swap(h->bf_frags);
    c.spans.swap(h->bf_spans);
    c.arena.swap(h->bf_arena);
    c.b_off.swap(h->bf_off);
    c.b_pairs.swap(h->bf_pairs);
    std::lock_guard<std::mutex> lk(h->qmu);
    h->queued.push_back(std::move(c));           // moved vectors keep their buffers: *b stays valid
    const fc2_caller::Chunk &q = h->queued.back();
    b->n = q.b_pairs.size();
    b->reads = (const uint8_t *)q.arena.data();
    b->read_off = q.b_off.data();
    b->pairs = q.b_pairs.data();
    if (eof) *eof = h->eof ? 1 : 0;
    return FC2_OK;
}

extern "C" int fc2_caller_queued(fc2_caller *h) {
    if (!h) return 0;
    std::lock_guard<std::mutex> lk(h->qmu);
    return (int)h->queued.size();
}

extern "C" int fc2_caller_submit(fc2_caller *h, const fc2_result *results, const uint64_t *tiemask, uint32_t tw,
                                 uint64_t stride) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_caller_submit: null argument");
    {
        std::lock_guard<std::mutex> lk(h->qmu);
        if (h->queued.empty())
            return fc2::fail(FC2_E_PARAM, "fc2_caller_submit: no chunk handed out by fc2_caller_next");
        fc2_caller::Chunk &c = h->queued.front();
        h->frags.swap(c.frags);
        h->spans.swap(c.spans);
        h->arena.swap(c.arena);
        h->b_off.swap(c.b_off);
        h->b_pairs.swap(c.b_pairs);
        h->queued.pop_front();
    }
    if (!h->b_pairs.empty() && !results) return fc2::fail(FC2_E_PARAM, "fc2_caller_submit: results missing");
    if (h->o.allhits && !h->b_pairs.empty() && (!tiemask || tw < 2 || stride < h->b_pairs.size()))
        return fc2::fail(FC2_E_PARAM, "fc2_caller_submit: --all-hits needs the tie mask");
    const Results R{results, tiemask, tw, stride};
    try {
        for (Frag &fr : h->frags) {
            std::set<HitRef> junctions;
            std::set<std::string> warns;
            record_hits(h, fr, R, junctions, warns);
            if (!junctions.empty()) {
                if (fr.has[0]) write_read(h, fr.prim[0], junctions, warns);
                if (fr.has[1]) write_read(h, fr.prim[1], junctions, warns);
            }
        }
    } catch (const Fatal &f) {
        h->frags.clear();
        return fc2::fail(f.code, f.msg);
    }
    h->frags.clear();
    return FC2_OK;
}

extern "C" int fc2_caller_take(fc2_caller *h, int stream, const char **text, uint64_t *len) {
    if (!h || stream < 0 || stream > 2 || !text || !len) return fc2::fail(FC2_E_PARAM, "fc2_caller_take: bad arguments");
    h->rows_text.swap(h->out[stream]);
    h->out[stream].clear();
    *text = h->rows_text.c_str();
    *len = h->rows_text.size();
    return FC2_OK;
}

extern "C" int fc2_caller_rows(fc2_caller *h, int kind, const char **text, uint64_t *len) {
    if (!h || kind < 0 || kind > 1 || !text || !len) return fc2::fail(FC2_E_PARAM, "fc2_caller_rows: bad arguments");
    h->rows_text.clear();
    storage_rows(h, kind, h->rows_text);
    *text = h->rows_text.c_str();
    *len = h->rows_text.size();
    return FC2_OK;
}

extern "C" int fc2_caller_counter(fc2_caller *h, int i, const char **name, double *value) {
    if (!h || !name || !value) return fc2::fail(FC2_E_PARAM, "fc2_caller_counter: null argument");
    if (i == 0) {
        // the caller's own counters plus those the ingest kept for fragments it never handed
        // over (Caller.run_native adds the non-zero ones)
        std::map<std::string, double> m;
        for (const auto &kv : h->N) m[kv.first] += kv.second;
        for (const auto &kv : h->N_in) m[kv.first] += kv.second;
        fc2_ingest_counts c{};
        fc2_ingest_counts_get(h->ing, &c);
        const std::pair<const char *, uint64_t> ing[4] = {{"total_mates", c.total_mates},
                                                           {"unmapped_reads", c.unmapped_reads},
                                                           {"unspliced_mates", c.unspliced_mates},
                                                           {"seg_too_short_skip", c.seg_too_short_skip}};
        for (const auto &kv : ing)
            if (kv.second) m[kv.first] += (double)kv.second;
        h->counters_snapshot.assign(m.begin(), m.end());
    }
    if (i < 0 || (size_t)i >= h->counters_snapshot.size()) return FC2_E_RANGE;
    *name = h->counters_snapshot[(size_t)i].first.c_str();
    *value = h->counters_snapshot[(size_t)i].second;
    return FC2_OK;
}

extern "C" int fc2_caller_stats(fc2_caller *h, uint64_t *n_reads, uint64_t *n_pairs) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_caller_stats: null argument");
    fc2_ingest_counts c{};
    fc2_ingest_counts_get(h->ing, &c);
    if (n_reads) *n_reads = c.n_reads;
    if (n_pairs) *n_pairs = h->n_pairs;
    return FC2_OK;
}
