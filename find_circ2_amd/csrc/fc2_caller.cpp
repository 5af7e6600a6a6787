// fc2_caller.cpp -- native find_circ read loop around the breakpoint search
// (include/fc2_caller.h).  Same logic and output as find_circ2_amd/caller.py,
// which cites find_circ.py line by line; the comments here point at the
// reference where the semantics are subtle.
#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <errno.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <sys/resource.h>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <malloc.h>
#include <sys/mman.h>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <string_view>
#include <utility>
#include <vector>

#include "../../include/fc2_caller.h"
#include "fc2_common.h"
#include "fc2_cpuacct.h"
#include "fc2_gzpieces.h"
#include "fc2_ingest_impl.h"

using fc2::ing::MateRef;
using fc2::ing::PyNum;
using fc2::ing::Rec;
using fc2::ing::RecFields;

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

// ---- Python 2 arithmetic on AS / XS tag values (find_circ.py:809-819, :556-566, :593) -------------
const char *py_type(PyNum::Kind k) {
    switch (k) {
        case PyNum::INT: return "int";
        case PyNum::FLOAT: return "float";
        case PyNum::STR: return "str";
        default: return "array.array";
    }
}

// a - b as Python computes it: int - int an int, a float operand a float; false where Python raises
// TypeError (a str or array operand)
bool py_sub(const PyNum &a, const PyNum &b, PyNum &out) {
    if (!a.number() || !b.number()) return false;
    out = (a.k == PyNum::INT && b.k == PyNum::INT) ? PyNum::of_int(a.i - b.i) : PyNum::of_float(a.value() - b.value());
    return true;
}

Fatal sub_error(const char *op, PyNum::Kind a, PyNum::Kind b) {
    return Fatal{FC2_E_FORMAT, std::string("TypeError: unsupported operand type(s) for ") + op + ": '" + py_type(a) +
                                   "' and '" + py_type(b) + "'"};
}

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

struct CompTable {                             // comp() as a byte table
    char t[256];
    CompTable() { for (int c = 0; c < 256; ++c) t[c] = comp((char)c); }
};
const CompTable kComp;

// every byte of u is one of 'A' 'C' 'G' 'T' (exact zero-byte tests, eight bytes at once)
inline bool acgt8(uint64_t u) {
    auto zero = [](uint64_t y) { return ~(((y & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | y | 0x7F7F7F7F7F7F7F7Full); };
    const uint64_t m = zero(u ^ 0x4141414141414141ull) | zero(u ^ 0x4343434343434343ull) |
                       zero(u ^ 0x4747474747474747ull) | zero(u ^ 0x5454545454545454ull);
    return m == 0x8080808080808080ull;
}

// complement() walks the sequence forward (find_circ.py:54-55): a KeyError names the first byte
// outside the table.  Eight upper-case ACGT bytes at a time; any other byte goes through the table.
void check_comp(const std::string &s) {
    const unsigned char *in = (const unsigned char *)s.data();
    const size_t n = s.size();
    size_t k = 0;
    for (; k + 8 <= n; k += 8) {
        uint64_t u;
        memcpy(&u, in + k, 8);
        if (acgt8(u)) continue;
        for (size_t j = k; j < k + 8; ++j)
            if (!kComp.t[in[j]]) throw Fatal{FC2_E_KEY, std::string("KeyError: ") + py_repr(std::string(1, (char)in[j]))};
    }
    for (; k < n; ++k)
        if (!kComp.t[in[k]]) throw Fatal{FC2_E_KEY, std::string("KeyError: ") + py_repr(std::string(1, (char)in[k]))};
}

void rev_comp_into(const std::string &s, std::string &r) {
    check_comp(s);
    const size_t n = s.size();
    r.resize(n);
    const unsigned char *in = (const unsigned char *)s.data();
    char *out = &r[0];
    for (size_t k = 0; k < n; ++k) out[k] = kComp.t[in[n - 1 - k]];
}

std::string rev_comp(const std::string &s) {
    std::string r;
    rev_comp_into(s, r);
    return r;
}

// ---- data ----------------------------------------------------------------------
struct APos {                                  // where an alignment sits (unspliced / broken segments)
    int32_t tid = -1;
    int64_t pos = -1, aend = -1;               // aend -1: None
    bool rev = false;
};

struct Align : APos {                          // a primary: what record_hits and the writers read of it
    std::string qname, seq, qual;
    bool has_seq = false, has_qual = false;
};

APos apos_of(const RecFields &r) {
    APos a;
    a.tid = r.tid;
    a.pos = r.pos;
    a.aend = r.aend;
    a.rev = (r.flag & 0x10) != 0;
    return a;
}

// A chunk's read_part bytes: grows without initialising, as each fragment writes its own region
class ByteBuf {
  public:
    char *data() { return p_.get(); }
    const char *data() const { return p_.get(); }
    size_t size() const { return n_; }
    void clear() { n_ = 0; }
    void resize(size_t n) {
        if (n > cap_) {
            const size_t c = std::max(n, 2 * cap_);
            std::unique_ptr<char[]> q(new char[c]);
            if (n_) memcpy(q.get(), p_.get(), n_);
            p_.swap(q);
            cap_ = c;
        }
        n_ = n;
    }
    void swap(ByteBuf &o) noexcept {
        p_.swap(o.p_);
        std::swap(n_, o.n_);
        std::swap(cap_, o.cap_);
    }
  private:
    std::unique_ptr<char[]> p_;
    size_t n_ = 0, cap_ = 0;
};

// the primary's strings are swapped in, not copied: the record gets the recycled Align's buffers
// back (the ingest reads nothing of a handed-over fragment's records, FragSink)
void take_align(Align &a, Rec &r) {
    r.decode();                                 // SEQ / QUAL left in the parse block (fc2::ing::Rec)
    static_cast<APos &>(a) = apos_of(r);
    a.qname.swap(r.qname);
    a.seq.swap(r.seq);
    a.qual.swap(r.qual);
    a.has_seq = r.has_seq;
    a.has_qual = r.has_qual;
}

struct Span {                                  // JunctionSpan (:821-852)
    int mate;                                  // 0 = mate1, 1 = mate2 of the fragment
    int32_t tid;                               // chromosome (reference id of the segments)
    bool circ;                                 // is_backsplice: B.pos - A.aend < 0
    int64_t a_pos, b_aend;
    double weight;
    // JunctionSpan.uniq = min(uniq_A, uniq_B) (:829-831): its value when a number; a str / array
    // (uniq_num false) orders above every number in Python 2, so `uniq >= min_uniq_qual` holds
    double uniq;
    bool uniq_num;
    // Hit.add's anchor qualities (after the backsplice swap), numbers; q_bad: one of Hit.add's
    // subtractions raises TypeError (a str / array last AS or XS), the first with operands q_bad_l, q_bad_r
    bool q_bad;
    PyNum::Kind q_bad_l, q_bad_r;
    PyNum qA, qB;
    bool a_rev;                                // A.is_reverse after the swap
    uint64_t read_off;
    uint32_t read_len;
    int64_t eval = -1;                         // index in the evaluation batch (kLongEval | index: in its long list)
};

constexpr int64_t kLongEval = int64_t(1) << 62;

// `span.uniq >= options.min_uniq_qual` (:1299, :1351) with Python 2's ordering (nan compares false)
inline bool uniq_ok(const Span &s, int64_t min_uniq_qual) { return !s.uniq_num || s.uniq >= (double)min_uniq_qual; }

struct Frag {
    // what on_fragment writes, first and together (the chunk's Frags are written in order, and a
    // Frag is ~600 bytes: the fewer cache lines the consumer touches per fragment the better)
    bool has[2] = {false, false};
    bool dropped = false;                      // no pair record_hits would look at (on_fragment)
    // recorded in place (a fragment grouped on a parse thread, its batch pinned until the chunk is
    // processed): the mates' records are read where they are, name and primaries taken by
    // process_frag on the workers instead of by on_fragment
    bool in_batch = false;
    uint64_t span0 = 0, span_max = 0;          // its span slots [span0, span0 + span_max) in the chunk
    uint64_t arena0 = 0;                       // its read_part bytes from here (at most one read per pair)
    // the mates' records as process_mate reads them (next side): fields at the chunk's recf[r0,
    // r0 + nrec), the proper segments' indices at prop[p0, p0 + np)
    struct MateFields {
        uint32_t r0 = 0, nrec = 0, p0 = 0, np = 0;
    } mf[2];
    MateRef ref[2];
    std::string name;
    Align prim[2];
    std::vector<int> circ, lin;                // indices into the chunk's spans
    std::vector<APos> unspliced, broken;
};

// a mate's records as process_mate reads them: recorded fields, or records in their parse batch
struct RecsView {
    const RecFields *fields = nullptr;
    const Rec *recs = nullptr;
    const int32_t *idx = nullptr;
    const RecFields &operator[](size_t k) const {
        return fields ? fields[k] : static_cast<const RecFields &>(recs[idx[k]]);
    }
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

// Memory for the large per-run tables, cache-line aligned.  (Marking it for transparent huge pages
// cut the recording side's TLB misses but stalled the other thread's allocations behind the
// compaction it triggered: slower overall on the GPU box, so not done -- FC2_AB_TABLE_THP builds
// the form again for a same-box A/B.)
#ifdef FC2_AB_TABLE_THP
constexpr size_t kHugeTable = size_t(2) << 20;
inline size_t table_bytes(size_t bytes) { return (bytes + kHugeTable - 1) & ~(kHugeTable - 1); }
void *table_alloc(size_t bytes) {
    const size_t len = table_bytes(bytes);
    void *m = mmap(nullptr, len + kHugeTable, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) throw std::bad_alloc();
    const uintptr_t a = ((uintptr_t)m + kHugeTable - 1) & ~(uintptr_t)(kHugeTable - 1);
    if (a > (uintptr_t)m) munmap(m, a - (uintptr_t)m);
    const uintptr_t end = (uintptr_t)m + len + kHugeTable;
    if (end > a + len) munmap((void *)(a + len), end - (a + len));
    (void)madvise((void *)a, len, MADV_HUGEPAGE);
    return (void *)a;
}
void table_free(void *p, size_t bytes) {
    if (p) munmap(p, table_bytes(bytes));
}
constexpr size_t kArenaBlock = kHugeTable;
#else
void *table_alloc(size_t bytes) {
    void *p = aligned_alloc(64, (bytes + 63) / 64 * 64);
    if (!p) throw std::bad_alloc();
    return p;
}
void table_free(void *p, size_t) { free(p); }
constexpr size_t kArenaBlock = size_t(1) << 20;
#endif

// Open-addressing CKey -> index table (linear probing, power-of-two capacity, load <= 1/2): one flat
// array of 32-byte slots (two per cache line) instead of a node per junction
class CIndex {
  public:
    CIndex() = default;
    CIndex(const CIndex &) = delete;
    CIndex &operator=(const CIndex &) = delete;
    ~CIndex() { table_free(slots_, cap_ * sizeof(Slot)); }
    // the index of k, inserting v for a new key; second = inserted
    std::pair<size_t, bool> try_emplace(const CKey &k, size_t v) {
        if (2 * (n_ + 1) > cap_) grow();
        for (size_t i = CKeyHash()(k) & (cap_ - 1);; i = (i + 1) & (cap_ - 1)) {
            Slot &s = slots_[i];
            if (!s.v1) { s.k = k; s.v1 = (uint32_t)(v + 1); ++n_; return {v, true}; }
            if (s.k == k) return {(size_t)s.v1 - 1, false};
        }
    }
    void prefetch(const CKey &k) const {        // the slot a lookup of k starts at
        if (cap_) __builtin_prefetch(&slots_[CKeyHash()(k) & (cap_ - 1)]);
    }
    size_t at(const CKey &k) const {
        if (cap_)
            for (size_t i = CKeyHash()(k) & (cap_ - 1);; i = (i + 1) & (cap_ - 1)) {
                const Slot &s = slots_[i];
                if (!s.v1) break;
                if (s.k == k) return (size_t)s.v1 - 1;
            }
        throw std::out_of_range("CIndex::at");
    }
  private:
    struct Slot {
        CKey k;
        uint32_t v1;                            // index + 1; 0 = empty
        uint32_t pad;
    };
    static_assert(sizeof(Slot) == 32, "two slots per cache line");
    Slot *slots_ = nullptr;
    size_t cap_ = 0, n_ = 0;
    void grow() {
        Slot *old = slots_;
        const size_t old_cap = cap_;
        cap_ = old_cap ? 2 * old_cap : 1024;
        slots_ = (Slot *)table_alloc(cap_ * sizeof(Slot));
        memset((void *)slots_, 0, cap_ * sizeof(Slot));
        n_ = 0;
        for (size_t j = 0; j < old_cap; ++j)
            if (old[j].v1) try_emplace(old[j].k, (size_t)old[j].v1 - 1);
        table_free(old, old_cap * sizeof(Slot));
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

// Append-only byte store for the strings the junction tables keep (read names, canonical reads,
// flagged fragment names): one allocation per MiB instead of one per string; the bytes stay where
// they are until the caller is closed, as the tables themselves do.
class Arena {
  public:
    Arena() = default;
    Arena(const Arena &) = delete;
    Arena &operator=(const Arena &) = delete;
    ~Arena() {
        for (const auto &b : blocks_) table_free(b.first, b.second);
    }
    std::string_view put(const char *p, size_t n) {
        if (blocks_.empty() || used_ + n > cap_) {
            cap_ = std::max<size_t>(n, kArenaBlock);
            blocks_.emplace_back((char *)table_alloc(cap_), cap_);
            used_ = 0;
        }
        char *d = blocks_.back().first + used_;
        if (n) memcpy(d, p, n);
        used_ += n;
        return std::string_view(d, n);
    }
    std::string_view put(std::string_view v) { return put(v.data(), v.size()); }
  private:
    std::vector<std::pair<char *, size_t>> blocks_;
    size_t used_ = 0, cap_ = 0;
};

// A set of strings of which only the size is read (Hit.readnames / Hit.uniq): the first member
// inline, a short vector up to 16, a hash set past that; members live in the Arena.
struct StrSet {
    // up to 16 members in `first` + `more`, past that an open-addressing table; every member is kept
    // with its hash, so a lookup compares the strings themselves (in the Arena: a cache miss each) only
    // where the hashes agree.  The table is linear-probed and at most 3/4 full: no allocation per
    // member -- a junction that many reads support (a real library: tens to thousands of reads per
    // junction) grows its table log2(n) times instead of allocating a node per read
    struct Slot {
        uint64_t h;                            // 0: empty (hashes are forced odd)
        std::string_view s;
    };
    Slot first{0, {}};
    size_t n = 0;
    std::vector<Slot> more;
    std::unique_ptr<Slot[]> tab;
    uint32_t cap = 0;                          // slots in tab, a power of two (0: no table yet)
    static uint64_t hash(std::string_view s) { return (uint64_t)std::hash<std::string_view>()(s) | 1u; }
    bool find(std::string_view s, uint64_t h, size_t &at) const {
        for (size_t i = (size_t)(h >> 7) & (cap - 1);; i = (i + 1) & (cap - 1)) {
            if (!tab[i].h) { at = i; return false; }
            if (tab[i].h == h && tab[i].s == s) { at = i; return true; }
        }
    }
    void place(const Slot &x) {
        size_t at;
        find(x.s, x.h, at);
        tab[at] = x;
    }
    void grow(uint32_t to) {
        std::unique_ptr<Slot[]> old(std::move(tab));
        const uint32_t oc = cap;
        tab.reset(new Slot[to]());
        cap = to;
        for (uint32_t k = 0; k < oc; ++k)
            if (old[k].h) place(old[k]);
    }
    bool contains(std::string_view s, uint64_t h) const {
        if (cap) {
            size_t at;
            return find(s, h, at);
        }
        if (n && first.h == h && first.s == s) return true;
        for (const Slot &x : more)
            if (x.h == h && x.s == s) return true;
        return false;
    }
    bool contains(std::string_view s) const { return contains(s, hash(s)); }
    // true if s was new
    bool insert(std::string_view s, Arena &a) {
        const uint64_t h = hash(s);
        if (cap) {
            size_t at;
            if (find(s, h, at)) return false;
            if (4 * (n + 1) > 3 * (size_t)cap) {
                grow(2 * cap);
                find(s, h, at);
            }
            tab[at] = Slot{h, a.put(s)};
            ++n;
            return true;
        }
        if (contains(s, h)) return false;
        const Slot v{h, a.put(s)};
        if (!n) first = v;
        else more.push_back(v);
        if (++n > 16) {                         // to the table: 17 members in 64 slots
            grow(64);
            place(first);
            for (const Slot &x : more) place(x);
            more.clear();
            more.shrink_to_fit();
        }
        return true;
    }
    size_t size() const { return n; }
};

// Hit.uniq (:579-580, :590): the set of (read, rc(read)) of every spliced read; only
// len(uniq) / 2 is read.  Stored as the set C of canonical forms min(read, rc(read)) plus the number
// of palindromic members (read == rc(read)), so len(uniq) = 2|C| - palindromes exactly, with one
// string per distinct read instead of two.
struct CanonSet {
    StrSet canon;
    int64_t palindromes = 0;
    // read must hold table bytes only (check_comp); rc(read) is built only when it is the smaller
    void insert(const std::string &read, Arena &a);
    int64_t size() const { return 2 * (int64_t)canon.size() - palindromes; }
};

// The flags record_hits attaches to a circ junction (find_circ.py:1319-1439), in sorted order:
// sets of them print sorted (Python sorts / iterates these sets' sorted keys), so a bit mask
// walked from bit 0 up gives the same order.
enum Warn : uint32_t {
    W_BROKEN_SEGMENTS, W_SUPPORT_CLOSURE, W_SUPPORT_INSIDE_MATE, W_SUPPORT_INSIDE_SPLICE_JUNCTION,
    W_WARN_MULTI_BACKSPLICE, W_WARN_OTHER_CHROM_MATE, W_WARN_OUTSIDE_MATE, W_WARN_OUTSIDE_SPLICE_JUNCTION,
    W_WARN_UNRESOLVED_EXTRA_BACKSPLICE, W_WARN_UNRESOLVED_LINSPLICE, kNumWarn
};
const char *const kWarnName[kNumWarn] = {
    "BROKEN_SEGMENTS", "SUPPORT_CLOSURE", "SUPPORT_INSIDE_MATE", "SUPPORT_INSIDE_SPLICE_JUNCTION",
    "WARN_MULTI_BACKSPLICE", "WARN_OTHER_CHROM_MATE", "WARN_OUTSIDE_MATE", "WARN_OUTSIDE_SPLICE_JUNCTION",
    "WARN_UNRESOLVED_EXTRA_BACKSPLICE", "WARN_UNRESOLVED_LINSPLICE"};
constexpr uint32_t kWarnNotWarn = (1u << W_BROKEN_SEGMENTS) | (1u << W_SUPPORT_CLOSURE) |
                                  (1u << W_SUPPORT_INSIDE_MATE) | (1u << W_SUPPORT_INSIDE_SPLICE_JUNCTION);

// Hit.read_flags: fragment name -> its set of flags (a mask); the first fragment inline
struct FlagReads {
    std::string_view first;
    uint32_t first_mask = 0;
    size_t n = 0;
    std::unique_ptr<std::unordered_map<std::string_view, uint32_t>> more;
    void add(const std::string &frag, uint32_t bit, Arena &a) {
        if (n && first == frag) { first_mask |= bit; return; }
        if (n && more) {
            auto it = more->find(std::string_view(frag));
            if (it != more->end()) { it->second |= bit; return; }
        }
        const std::string_view v = a.put(frag);
        if (!n) { first = v; first_mask = bit; }
        else {
            if (!more) more.reset(new std::unordered_map<std::string_view, uint32_t>());
            more->emplace(v, bit);
        }
        ++n;
    }
    template <class F> void each(F f) const {
        if (n) f(first_mask);
        if (more)
            for (const auto &kv : *more) f(kv.second);
    }
};

struct Hit {                                   // Hit (:486-654)
    int64_t novel = 0;                         // > 0: named <name>_<prefix>_<novel:06d> (:684-686)
    std::string known_name;                    // novel == 0: the name a known-sites file gave
    CKey key;                                  // the coordinate (chrom, start, end, strand) as ids
    int64_t n_reads = 0;
    StrSet readnames;
    CanonSet uniq;
    bool has_mq = false;
    PyNum mq_a, mq_b;                          // sorted(mapquals_A / _B, reverse=True)[0] (:593): the first maximum
    double n_weighted = 0.;
    int64_t n_spanned = 0;
    double n_uniq_bridges = 0.;
    PyMin edits, overlaps, n_hits;
    std::string signal = "NNNN";
    bool added = false;                        // Hit.add ran: strandmatch 'N/A' (else 'NA', :504, :532)
    uint32_t flag_n[kNumWarn] = {};            // Hit.flags: count per flag (present iff > 0)
    FlagReads read_flags;
    bool has_tissue = false;
    double tissue = 0.;
};

// Hits in insertion (= dict) order, in blocks that never move (references stay valid);
// a Hit is constructed when it is added
class HitVec {
  public:
    HitVec() = default;
    HitVec(const HitVec &) = delete;
    HitVec &operator=(const HitVec &) = delete;
    ~HitVec() {
        for (size_t k = 0; k < n_; ++k) (*this)[k].~Hit();
        for (Hit *b : blocks_) table_free(b, kBlock * sizeof(Hit));
    }
    size_t size() const { return n_; }
    Hit &operator[](size_t k) { return blocks_[k >> kShift][k & (kBlock - 1)]; }
    const Hit &operator[](size_t k) const { return blocks_[k >> kShift][k & (kBlock - 1)]; }
    Hit &emplace_back() {
        if ((n_ >> kShift) == blocks_.size()) blocks_.push_back((Hit *)table_alloc(kBlock * sizeof(Hit)));
        Hit *h = &(*this)[n_];
        new (h) Hit();
        ++n_;
        return *h;
    }
  private:
    static constexpr size_t kShift = 12, kBlock = size_t(1) << kShift;
    std::vector<Hit *> blocks_;
    size_t n_ = 0;
};

// ---- the recording side, parallel (fc2_caller_submit) --------------------------------------
// record_hits (:1276-1439) touches three kinds of state: the fragment's own (its spans' results,
// the coordinates, flags and rows it derives from them), the junction tables (Hit.add of every
// splice, :526-582, and the flags), and the names, given by first appearance (:684-686).  A chunk
// is therefore recorded in phases: (A) the fragments, cut into contiguous ranges, on all workers:
// everything record_hits decides from the fragment alone, including every exception it can raise,
// with each table update emitted as an event for the shard that owns the junction's coordinate;
// (B) the shards on all workers, each applying its events in input order -- so every float sum
// of a junction (:544, :563, :579) and every min / last-value field sees its updates in the
// sequential order; (C) one thread names the chunk's new junctions by merging the shards' first
// appearances; (D) the ranges again: the read names and multi_events rows, which need the names,
// written per range and joined in input order.
constexpr int kShards = 16;

struct JRef {                                  // a junction: its shard and its index there
    uint32_t shard = 0, idx = 0;
};

struct Shard {
    HitVec hits[2];                            // 0 circ, 1 lin; never relocated
    CIndex index[2];                           // coordinate -> index in hits
    Arena strings;                             // the hits' read names, canonical reads, fragment names
    std::vector<std::pair<uint64_t, uint32_t>> fresh[2];   // this chunk's new junctions: (seq, idx)
};

inline int shard_of(const CKey &k) { return (int)(CKeyHash()(k) >> 60) & (kShards - 1); }

struct SEv {                                   // one table update of a shard (phase A -> B)
    uint64_t seq;                              // fragment index << 32 | the fragment's add ordinal
    CKey key;
    uint32_t frag;                             // fragment index in the chunk
    uint32_t slot;                             // the range's slot: written (add) / read (flag)
    int32_t span;                              // Splice.junc_span (a span of the chunk)
    int32_t dist, ov, n_hits;
    uint8_t kind;                              // 0 circ, 1 lin
    uint8_t op;                                // 0 Hit.add (+ the read), 1 add_flag
    uint8_t warn;                              // op 1: the flag
    uint8_t dist_bool;                         // -d 0: dist is simple_match's bool
    uint8_t mate, gtag_len;
    char gtag[6];
};

struct FOut {                                  // a fragment with junctions (phase A -> D)
    uint32_t frag;
    uint32_t warns;
    uint32_t j0, nj;                           // its distinct junctions: RangeOut::jk[j0, j0 + nj)
    int64_t m0 = -1;                           // multi_events row: parts at RangeOut::mtext[m0, ...)
    uint32_t m1 = 0, m2 = 0;                   // ... lengths of the text before / after the name
    uint32_t circ_slot = 0;
};

struct RangeOut {                              // one range of a chunk's fragments
    std::vector<SEv> ev[kShards];
    std::vector<JRef> slots;                   // one per add event, resolved in phase B
    std::vector<FOut> fouts;
    std::vector<std::pair<uint8_t, uint32_t>> jk;   // (kind, slot) of FOut junctions
    std::string mtext, test, out0, out1;
    std::vector<std::pair<const char *, double>> N;
    int64_t err_frag = -1;                     // the first fragment that raised (phase A), or -1
    int err_code = 0;
    std::string err_msg;
    void clear() {
        for (auto &v : ev) v.clear();
        slots.clear();
        fouts.clear();
        jk.clear();
        mtext.clear();
        test.clear();
        out0.clear();
        out1.clear();
        N.clear();
        err_frag = -1;
        err_code = 0;
        err_msg.clear();
    }
};

// Fork-join workers: run(n, f) calls f(0) .. f(n-1) on the workers and the calling thread and
// returns when all have returned.  Tasks are claimed from a counter tagged with the run's
// generation, so a worker still leaving the previous run can never take a task of this one.
class WorkPool {
  public:
    explicit WorkPool(int n_workers) {
        for (int k = 0; k < n_workers; ++k) th_.emplace_back([this] { loop(); });
    }
    ~WorkPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return (int)th_.size() + 1; }
    // as run, with an exception of a task (bad_alloc, a Fatal) handed to the caller after all
    // tasks returned: the first one, by task index
    void run_checked(int n, const std::function<void(int)> &f) {
        std::vector<std::exception_ptr> ex((size_t)std::max(n, 0));
        run(n, [&](int k) {
            try {
                f(k);
            } catch (...) {
                ex[(size_t)k] = std::current_exception();
            }
        });
        for (auto &e : ex)
            if (e) std::rethrow_exception(e);
    }
    void run(int n, const std::function<void(int)> &f) {
        if (n <= 0) return;
        if (n == 1 || th_.empty()) {
            for (int k = 0; k < n; ++k) f(k);
            return;
        }
        uint64_t g;
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &f;
            n_ = n;
            done_ = 0;
            g = ++gen_;
            next_.store(g << 32);
        }
        cv_.notify_all();
        work(g, &f, n);
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return done_ == n; });
    }
  private:
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)> *job_ = nullptr;
    int n_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
    std::atomic<uint64_t> next_{0};
    void work(uint64_t g, const std::function<void(int)> *job, int n) {
        for (;;) {
            uint64_t v = next_.load();
            do {
                if ((v >> 32) != g || (int)(v & 0xFFFFFFFFu) >= n) return;
            } while (!next_.compare_exchange_weak(v, v + 1));
            (*job)((int)(v & 0xFFFFFFFFu));
            std::lock_guard<std::mutex> lk(m_);
            if (++done_ == n) done_cv_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)> *job;
            int n;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
                n = n_;
            }
            work(seen, job, n);
        }
    }
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
    // an error of the input or of process_mate met while forming a chunk: the fragments before it
    // are handed out first (the reference records each fragment before reading the next), the
    // error comes with the following fc2_caller_next
    int next_err = FC2_OK;
    std::string next_err_msg;
    // Two sides that may run on two threads at once: fc2_caller_next forms chunks (ingest,
    // process_mate, the pairs) into the bf_* fields, fc2_caller_submit records the oldest queued chunk
    // (record_hits, tables, writers) from the plain fields.  They share only the queue (mutex) and
    // read-only state (options, genome map, reference names); each side has its own counters.
    std::vector<Frag> bf_frags;                 // the chunk being formed (next): its first bf_nfrags
    size_t bf_nfrags = 0;                       // entries (the rest are recycled objects)
    std::vector<Span> bf_spans;
    ByteBuf bf_arena;                           // read_part bytes
    uint64_t bf_nspans = 0, bf_narena = 0;      // span slots / arena bytes reserved so far
    std::vector<RecFields> bf_recf;             // the chunk's mates' records (Frag::MateFields)
    std::vector<int32_t> bf_prop;
    // runs of fragments a parse thread grouped, recorded whole (the bulk sink): fragments
    // [f0, f0 + r.n) of the chunk, their spans and read parts from span0 / arena0 on
    struct Seg {
        fc2::ing::RegionRef r;
        size_t f0;
        uint64_t span0, arena0;
    };
    std::vector<Seg> bf_segs;
    std::unique_ptr<WorkPool> next_pool;        // the next side's workers (process_mate)
    std::vector<std::vector<std::pair<const char *, double>>> next_N;   // their counters per range
    std::vector<std::pair<int64_t, Fatal>> next_err_at;                 // their first error per range
    std::vector<uint64_t> bf_off;
    std::vector<fc2_pair> bf_pairs;
    std::vector<fc2_long_pair> bf_long;         // pairs with read parts over FC2_MAX_READ_LEN
    std::vector<int64_t> bf_starts, bf_ends;    // process_mate scratch
    std::vector<size_t> bf_order;
    std::vector<Frag> frags;                    // the chunk being recorded (submit): first nfrags
    size_t nfrags = 0;
    std::vector<Span> spans;
    ByteBuf arena;
    std::vector<uint64_t> b_off;
    std::vector<fc2_pair> b_pairs;
    std::vector<fc2_long_pair> b_long;
    // the oldest queued chunk's long-pair results (fc2_caller_submit_long): results, tie words and
    // each pair's first tie word (fc2_long_geometry)
    std::vector<fc2_long_result> l_res;
    std::vector<uint64_t> l_ties, l_tie_off;
    bool l_staged = false;
    // chunks handed out by fc2_caller_next and not yet submitted, oldest first: the caller may
    // read ahead (form chunk k+1 while chunk k is on the GPU or being recorded)
    struct Chunk {
        std::vector<Frag> frags;
        size_t nfrags = 0;
        std::vector<Span> spans;
        ByteBuf arena;
        std::vector<uint64_t> b_off;
        std::vector<fc2_pair> b_pairs;
        std::vector<fc2_long_pair> b_long;
    };
    std::deque<Chunk> queued;
    // recorded chunks handed back to the next side: their fragments' strings and vectors keep their
    // capacity, so forming a chunk allocates nothing in steady state, and nothing allocated on one
    // thread is freed on the other
    std::vector<Chunk> spare;
    bool read_side_released = false;            // release_read_side ran (after the last chunk): the
    fc2_ingest_counts ing_final{};              // input is closed then, its final counts kept here
    uint64_t inflate_final[2] = {0, 0};         // (and its GPU / CPU inflate counts)
    std::thread release_thr;                    // ... on this thread (joined by fc2_caller_close)
    std::mutex qmu;                             // guards queued and spare
    // fc2_caller_stats' values, published by fc2_caller_next on the thread that advances the input
    // (a recording thread may ask for them while the reader runs)
    std::atomic<uint64_t> st_reads{0}, st_pairs{0};
    // aggregation: SpliceSiteStorage (:657-730) of circ (0) and linear (1) junctions, its dict cut
    // into kShards shards by the coordinate's hash (Shard); the dict order -- known sites, then
    // junctions by first appearance, which also gives the names (:684-686) -- is kept in order[]
    Shard sh[kShards];
    std::vector<JRef> order[2];                 // every junction in insertion (= dict) order
    int64_t novel[2] = {0, 0};                  // junctions named so far (:684-686)
    std::string prefix[2] = {"circ", "lin"};
    // the recording side's workers and per-range scratch (fc2_caller_submit)
    std::unique_ptr<WorkPool> pool;
    std::vector<RangeOut> ranges;
    size_t min_range_frags = 2048;              // fragments per range at least (FC2_CALLER_MIN_RANGE)
    std::unordered_map<std::string, uint32_t> ids;    // interned chromosome / strand strings (submit side)
    std::vector<std::string> id_names;                // ... and back
    std::vector<int64_t> tid_cid;                     // reference id -> interned chromosome (submit side)
    std::vector<std::pair<const char *, double>> N;   // the reference's counters, keyed by literal
                                                      // (merged by name into sorted keys on output)
    std::vector<std::pair<const char *, double>> N_in; // the same for the counters the next side bumps
    std::string out[3];                         // reads, multi, test text since the last take
    fc2::GzPieces reads_gz;                     // fc2_caller_set_reads_gz: out[0] goes here
    std::string taken[3];                       // fc2_caller_take's buffers (valid until the next take)
    std::string rows_text;
    std::vector<std::pair<std::string, double>> counters_snapshot;
    uint64_t n_pairs = 0;
    uint64_t n_chunks = 0;                      // chunks formed (next side)
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
    h->id_names.push_back(v);
    return id;
}

uint32_t strand_id(fc2_caller *h, const std::string &strand) {
    if (strand.size() == 1 && (strand[0] == '+' || strand[0] == '-')) return strand[0] == '-' ? 1u : 0u;
    return 2u + intern(h, strand);
}

// the same key straight from a Splice (Splice.coord, :801-806), without building the tuple
CKey coord_key(fc2_caller *h, const Splice &sp) {
    const uint32_t c = sp.cid >= 0 ? (uint32_t)sp.cid : intern(h, sp.chrom);
    return sp.start < sp.end ? CKey{sp.start, sp.end, c, strand_id(h, sp.strand)}
                             : CKey{sp.end, sp.start, c, strand_id(h, sp.strand)};
}

// a junction's coordinate strings back from its key
const std::string &key_chrom(const fc2_caller *h, const CKey &k) { return h->id_names[k.chrom]; }
const std::string &key_strand(const fc2_caller *h, const CKey &k) {
    static const std::string plus("+"), minus("-");
    return k.strand == 0 ? plus : k.strand == 1 ? minus : h->id_names[k.strand - 2];
}
Coord key_coord(const fc2_caller *h, const CKey &k) { return Coord(key_chrom(h, k), k.start, k.end, key_strand(h, k)); }

// ---- Hit / SpliceSiteStorage ----------------------------------------------------------
void hit_add(fc2_caller *h, Hit &t, const Splice &sp) {
    t.signal = sp.gtag;
    t.added = true;
    if (h->o.stranded)   // Splice has no strandmatch attribute (:532-533)
        throw Fatal{FC2_E_FORMAT, "AttributeError: 'Splice' object has no attribute 'strandmatch'"};
    t.edits.add(sp.dist, sp.dist_bool);
    t.overlaps.add(sp.ov, false);
    t.n_hits.add(sp.n_hits, false);
    // only known sites come here (Splice(None, ...), :676): no junc_span, nothing more to add (:542)
}

// Hit.add's anchor-quality part (:558-566): qA / qB are numbers (check_add raised otherwise)
void hit_quals(Hit &t, const Span &s) {
    if (s.qA.value() != 0 && s.qB.value() != 0) t.n_uniq_bridges += s.weight;   // `if qA and qB` (nan is true)
    if (!t.has_mq) { t.has_mq = true; t.mq_a = s.qA; t.mq_b = s.qB; return; }
    if (s.qA.value() > t.mq_a.value()) t.mq_a = s.qA;      // the first of equal maxima stays (stable sort)
    if (s.qB.value() > t.mq_b.value()) t.mq_b = s.qB;
}

void CanonSet::insert(const std::string &read, Arena &a) {
    const size_t n = read.size();
    const unsigned char *in = (const unsigned char *)read.data();
    // read against rc(read) byte by byte (unsigned, as std::string compares) up to the first
    // difference, which nearly always comes at once: rc is built only when it is the smaller
    size_t k = 0;
    auto rc_at = [&](size_t j) { return (unsigned char)kComp.t[in[n - 1 - j]]; };
    while (k < n && in[k] == rc_at(k)) ++k;
    const int cmp = k == n ? 0 : (in[k] < rc_at(k) ? -1 : 1);
    if (cmp <= 0) {
        if (canon.insert(read, a) && cmp == 0) palindromes += 1;
        return;
    }
    static thread_local std::string rc;
    rc.resize(n);
    char *o = &rc[0];
    for (size_t j = 0; j < n; ++j) o[j] = kComp.t[in[n - 1 - j]];
    canon.insert(rc, a);
}

// Hit.add of a splice from the chunk (:547-582) as phase B applies it: the checks that raise
// (stranded, :532-533; a non-integer anchor quality, :558-566; rev_comp of the read, :573-582)
// already passed in phase A (check_add)
void hit_apply(const fc2_caller *h, Hit &t, const SEv &e) {
    t.signal.assign(e.gtag, e.gtag_len);
    t.added = true;
    t.edits.add(e.dist, e.dist_bool != 0);
    t.overlaps.add(e.ov, false);
    t.n_hits.add(e.n_hits, false);
    const Span &s = h->spans[(size_t)e.span];
    t.n_spanned += 1;
    t.n_weighted += s.weight;
    hit_quals(t, s);
}

// the span-dependent part of Hit.add that needs the fragment's primary (its read passed
// check_comp in phase A's store before the event was made: rev_comp(read), :573, :582)
void hit_add_read(Arena &a, Hit &t, const Span &s, const Align &prim) {
    t.readnames.insert(prim.qname, a);
    const std::string &read = prim.seq;
    t.n_reads += 1;
    t.has_tissue = true;
    t.tissue += s.weight;
    t.uniq.insert(read, a);
}

// the junction's name (find_circ.py:684-686), appended to out
void hit_name(const fc2_caller *h, int kind, const Hit &t, std::string &out) {
    if (!t.novel) { out += t.known_name; return; }
    out += h->name;                             // name + "_%s_%06d" % (prefix, novel)
    out += '_';
    out += h->prefix[kind];
    out += '_';
    char d[24];
    int n = 0;
    for (uint64_t v = (uint64_t)t.novel; v; v /= 10) d[n++] = (char)('0' + v % 10);
    while (n < 6) d[n++] = '0';
    while (n) out += d[--n];
}

void add_flag(Arena &a, Hit &t, uint32_t w, const std::string &frag) {
    t.flag_n[w] += 1;
    t.read_flags.add(frag, 1u << w, a);
}

const Hit &hit_at(const fc2_caller *h, int kind, const JRef &j) { return h->sh[j.shard].hits[kind][j.idx]; }

// categories (:601-654) as literals, into cats[]; returns how many
int categories(const fc2_caller *h, const Hit &t, const char *cats[8]) {
    const auto &o = h->o;
    int n = 0;
    if (t.signal != "GTAG") cats[n++] = "NON_CANONICAL";
    if (t.mq_a.value() == 0 || t.mq_b.value() == 0) cats[n++] = "WARN_NON_UNIQUE_ANCHOR";
    if (t.n_uniq_bridges == 0) cats[n++] = "WARN_NO_UNIQ_BRIDGES";
    if (t.n_hits.v > 1) cats[n++] = "WARN_AMBIGUOUS_BP";
    const int64_t mov = t.overlaps.v, med = t.edits.v;
    if (mov == 0 && med == 0) {
    } else if (mov < 2 && med < 2) {
        cats[n++] = "WARN_EXT_1MM";
    } else if (mov >= 2 || med >= 2) {
        cats[n++] = "WARN_EXT_2MM+";
    }
    const int64_t start = t.key.start, end = t.key.end;
    if (end - start < o.short_threshold) cats[n++] = "SHORT";
    else if (end - start > o.huge_threshold) cats[n++] = "HUGE";
    int64_t unbroken = 0, unwarned = 0;
    double total = 0.;
    t.read_flags.each([&](uint32_t mask) {
        total += 1.;
        if (!(mask & (1u << W_BROKEN_SEGMENTS))) unbroken += 1;
        unwarned += __builtin_popcount(mask & kWarnNotWarn);
    });
    if (total) {
        if (!unbroken) cats[n++] = "WARN_ALWAYS_BROKEN";
        if (!unwarned) cats[n++] = "WARN_ALWAYS_WARN";
    }
    return n;
}

std::string join(const std::vector<std::string> &v, const char *sep) {
    std::string r;
    for (size_t k = 0; k < v.size(); ++k) {
        if (k) r += sep;
        r += v[k];
    }
    return r;
}

void app_int(std::string &out, int64_t v) {   // str(int)
    char d[24];
    int n = 0;
    uint64_t u = v < 0 ? 0 - (uint64_t)v : (uint64_t)v;
    do { d[n++] = (char)('0' + u % 10); u /= 10; } while (u);
    if (v < 0) out += '-';
    while (n) out += d[--n];
}

void app_py2_float(std::string &out, double v) {   // py2_float, integral values without snprintf
    if (v == v && v > -1e12 && v < 1e12 && v == (double)(int64_t)v && !(v == 0 && signbit(v))) {
        app_int(out, (int64_t)v);                  // '%.12g' of an integer below 1e12 is its digits
        out += ".0";
        return;
    }
    out += py2_float(v);
}

void app_pynum(std::string &out, const PyNum &v) {  // str() of an anchor quality: int or float
    if (v.k == PyNum::FLOAT) app_py2_float(out, v.f);
    else app_int(out, v.i);
}

void app_pymin(std::string &out, const PyMin &m) {
    if (m.is_bool) out += m.v ? "True" : "False";
    else app_int(out, m.v);
}

// store_list (:690-730) for the junctions [b, e) of the dict order: their rows appended to outs, the
// counters of the ones skipped into N (reads the tables only: ranges run on the workers at once)
void storage_rows(const fc2_caller *h, int kind, size_t b, size_t e, std::string &outs,
                  std::vector<std::pair<const char *, double>> &N) {
    const auto &o = h->o;
    for (size_t k = b; k < e; ++k) {             // dict order
        const Hit &t = hit_at(h, kind, h->order[kind][k]);
        if (!t.n_reads) continue;
        const double qa = t.mq_a.value(), qb = t.mq_b.value(), mq = (double)o.min_uniq_qual;
        if (o.halfunique) {
            if (qa < mq && qb < mq) { incN_into(N, "anchor_not_uniq", 1.); continue; }
        } else if (qa < mq || qb < mq) {
            incN_into(N, "anchor_not_uniq", 1.);
            continue;
        }
        if (t.n_uniq_bridges == 0 && !o.report_nobridges) { incN_into(N, "no_uniq_bridges", 1.); continue; }
        // the 22 columns of find_circ.py:712-730, appended in place
        const char tab = '\t';
        outs += key_chrom(h, t.key); outs += tab;
        app_int(outs, t.key.start); outs += tab;
        app_int(outs, t.key.end); outs += tab;
        hit_name(h, kind, t, outs); outs += tab;
        app_int(outs, (int64_t)t.readnames.size()); outs += tab;
        outs += key_strand(h, t.key); outs += tab;
        app_py2_float(outs, t.n_weighted); outs += tab;
        app_int(outs, t.n_spanned); outs += tab;
        app_int(outs, t.uniq.size() / 2); outs += tab;
        app_py2_float(outs, t.n_uniq_bridges); outs += tab;
        app_pynum(outs, t.mq_a); outs += tab;
        app_pynum(outs, t.mq_b); outs += tab;
        if (t.has_tissue) outs += h->name;
        outs += tab;
        if (t.has_tissue) app_py2_float(outs, t.tissue);
        outs += tab;
        app_pymin(outs, t.edits); outs += tab;
        app_pymin(outs, t.overlaps); outs += tab;
        app_pymin(outs, t.n_hits); outs += tab;
        outs += t.signal; outs += tab;
        outs += t.added ? "N/A" : "NA"; outs += tab;
        const char *cats[8];
        const int nc = categories(h, t, cats);
        std::sort(cats, cats + nc, [](const char *x, const char *y) { return strcmp(x, y) < 0; });
        for (int c = 0; c < nc; ++c) {
            if (c) outs += ',';
            outs += cats[c];
        }
        outs += tab;
        bool any_flag = false;
        for (uint32_t w = 0; w < kNumWarn; ++w) any_flag |= t.flag_n[w] > 0;
        if (any_flag) {
            bool first = true;
            for (uint32_t w = 0; w < kNumWarn; ++w)
                if (t.flag_n[w]) { if (!first) outs += ','; outs += kWarnName[w]; first = false; }
            outs += tab;
            first = true;
            for (uint32_t w = 0; w < kNumWarn; ++w)
                if (t.flag_n[w]) { if (!first) outs += ','; app_int(outs, t.flag_n[w]); first = false; }
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
        const int si = shard_of(key);
        Shard &S = h->sh[si];
        const auto ins = S.index[kind].try_emplace(key, S.hits[kind].size());
        // a repeated coordinate keeps its first dict position, with the later line's Hit
        Hit &t = ins.second ? S.hits[kind].emplace_back() : S.hits[kind][ins.first];
        if (ins.second) h->order[kind].push_back(JRef{(uint32_t)si, (uint32_t)ins.first});
        t = Hit();
        t.known_name = fl[3];
        t.key = key;
        hit_add(h, t, sp);
        ++n;
    }
    fclose(f);
    return n;
}

// ---- fragments ----------------------------------------------------------------------
std::string chrom_of(const fc2_caller *h, int32_t tid) {         // fast_chrom_lookup (:471-477)
    const char *nm = fc2_ingest_ref_name(h->ing, tid);
    if (tid < 0 || !nm) throw Fatal{FC2_E_FORMAT, "ValueError: reference id " + i2s(tid) + " out of range"};
    return nm;
}

PyNum uniqness(const RecFields &a) {                                    // :809-819
    if (!a.has_as) throw Fatal{FC2_E_KEY, "KeyError: \"tag 'AS' not present\""};
    if (!a.has_xs) return a.as;                                         // a str / array AS stays as it is
    PyNum u;
    if (!py_sub(a.as, a.xs, u)) throw sub_error("-=", a.as.k, a.xs.k);  // u -= get_tag('XS')
    return u;
}

// Hit.add's anchor quality (find_circ.py:556-559): dict(tags) keeps the LAST AS / XS of a record,
// and get('XS', 0) defaults to the int 0.  Only Hit.add reads it, so a non-number matters only for a
// span that reaches a Hit (check_add raises there); false, with the operands' kinds, when the
// subtraction raises
bool dict_quality(const RecFields &a, PyNum &q, PyNum::Kind &l, PyNum::Kind &r) {
    const PyNum xs = a.has_xs ? a.xs_last : PyNum::of_int(0);
    l = a.as_last.k;
    r = xs.k;
    return py_sub(a.as_last, xs, q);
}

const char *kNoneLen = "TypeError: object of type 'NoneType' has no len()";

// process_mate (:1492-1527) with adjacent_segment_pairs (:1058-1140), on the mate's recorded
// fields (Frag::MateFields) and its primary's sequence (fr.prim[mi], taken by on_fragment): spans
// into the fragment's slots of `spans` from *sk on, read parts into `arena` from *ap on
void process_mate(const fc2_caller *h, const RecsView &recs, size_t nrec, const int32_t *proper, size_t n, int mi,
                  Frag &fr, Span *spans, uint64_t &sk, char *arena, uint64_t &ap,
                  std::vector<std::pair<const char *, double>> &N) {
    const RecFields &prim = recs[0];
    if (n < 2) {
        incN_into(N, "unspliced_mates", 1.);
        fr.unspliced.push_back(apos_of(prim));
        return;
    }
    if (!prim.has_seq) throw Fatal{FC2_E_FORMAT, kNoneLen};      // L = len(mate.full_seq)
    const std::string &seq = fr.prim[mi].seq;
    const int64_t L = (int64_t)seq.size();
    const double weight = 1. / ((double)n - 1.);
    int64_t st_small[16], en_small[16];
    size_t ord_small[16];
    std::vector<int64_t> st_big, en_big;
    std::vector<size_t> ord_big;
    int64_t *starts = st_small, *ends = en_small;
    size_t *order = ord_small;
    if (n > 16) {
        st_big.resize(n); en_big.resize(n); ord_big.resize(n);
        starts = st_big.data(); ends = en_big.data(); order = ord_big.data();
    }
    for (size_t k = 0; k < n; ++k) {
        const RecFields &s = recs[proper[k]];
        if (s.qlen < 0) throw Fatal{FC2_E_FORMAT, kNoneLen};     // len(s.query)
        starts[k] = s.astart;
        ends[k] = s.astart + s.qlen;
        order[k] = k;
    }
    for (size_t i = 1; i < n; ++i) {           // stable insertion sort by query start (n is small)
        const size_t v = order[i];
        size_t j = i;
        while (j > 0 && starts[order[j - 1]] > starts[v]) { order[j] = order[j - 1]; --j; }
        order[j] = v;
    }
    int64_t min_s = L, max_e = 0;
    for (size_t k = 0; k + 1 < n; ++k) {
        const size_t a = order[k], b = order[k + 1];
        if (ends[a] - starts[a] < h->o.asize || ends[b] - starts[b] < h->o.asize) {
            incN_into(N, "seg_too_short_skip", 1.);
            continue;
        }
        const RecFields &A = recs[proper[a]], &B = recs[proper[b]];
        const int64_t q_start = std::min(starts[a], starts[b]), q_end = std::max(ends[a], ends[b]);
        (void)chrom_of(h, A.tid);
        Span s;
        s.mate = mi;
        s.tid = A.tid;
        const PyNum ua = uniqness(A), ub = uniqness(B);
        if (A.aend < 0) throw Fatal{FC2_E_FORMAT, "TypeError: unsupported operand type(s) for -: 'int' and 'NoneType'"};
        s.circ = B.pos - A.aend < 0;
        s.a_pos = A.pos;
        s.b_aend = B.aend;
        s.weight = weight;
        // min(uniq_A, uniq_B) in Python 2: numbers by value (ub only if strictly smaller), a number
        // before a str / array; two non-numbers give a non-number
        if (ua.number() && ub.number()) s.uniq = ub.value() < ua.value() ? ub.value() : ua.value();
        else s.uniq = ua.number() ? ua.value() : ub.value();
        s.uniq_num = ua.number() || ub.number();
        PyNum qa, qb;
        PyNum::Kind la, ra, lb, rb;
        const bool qa_ok = dict_quality(A, qa, la, ra), qb_ok = dict_quality(B, qb, lb, rb);
        // after Hit.add's swap (backsplice: A, B = B, A) qA comes first: its failure is the one raised
        const bool first_ok = s.circ ? qb_ok : qa_ok, second_ok = s.circ ? qa_ok : qb_ok;
        s.q_bad = !(first_ok && second_ok);
        s.q_bad_l = !first_ok ? (s.circ ? lb : la) : (s.circ ? la : lb);
        s.q_bad_r = !first_ok ? (s.circ ? rb : ra) : (s.circ ? ra : rb);
        s.qA = s.circ ? qb : qa;
        s.qB = s.circ ? qa : qb;
        s.a_rev = s.circ ? (B.flag & 0x10) != 0 : (A.flag & 0x10) != 0;
        // read_part = primary.seq[q_start:q_end] (Python slice)
        const int64_t lo = std::max<int64_t>(0, std::min(q_start, L)), hi = std::max(lo, std::min(q_end, L));
        s.read_off = ap;
        s.read_len = (uint32_t)(hi - lo);
        if (hi > lo) memcpy(arena + ap, seq.data() + lo, (size_t)(hi - lo));
        ap += (uint64_t)(hi - lo);
        spans[sk] = s;
        (s.circ ? fr.circ : fr.lin).push_back((int)sk);
        ++sk;
        min_s = std::min(min_s, q_start);
        max_e = std::max(max_e, q_end);
    }
    if (max_e < L - h->o.asize || min_s > h->o.asize) {
        const bool prev = (prim.flag & 0x10) != 0;
        for (size_t k = 1; k < nrec; ++k)
            if (recs[k].tid != prim.tid) fr.broken.push_back(apos_of(recs[k]));
        for (size_t k = 1; k < nrec; ++k)
            if (recs[k].tid == prim.tid && ((recs[k].flag & 0x10) != 0) != prev) fr.broken.push_back(apos_of(recs[k]));
    }
}

// on_fragment's processing of one recorded fragment (both mates, process_mate) and the reference's
// filter on the result (Caller._flush): no circ span, or no span at all with --no-linear
void process_frag(const fc2_caller *h, Frag &fr, const std::vector<RecFields> &recf, const std::vector<int32_t> &prop,
                  Span *spans, char *arena, std::vector<std::pair<const char *, double>> &N) {
    fr.circ.clear();
    fr.lin.clear();
    fr.unspliced.clear();
    fr.broken.clear();
    for (uint64_t k = 0; k < fr.span_max; ++k) spans[fr.span0 + k].eval = -1;   // unused slots
    if (fr.in_batch) {                          // what on_fragment takes of a fragment it recorded in place
        fr.name.assign(fr.ref[1].rec(0).qname);
        for (int k = 0; k < 2; ++k)
            if (fr.has[k]) take_align(fr.prim[k], fr.ref[k].rec(0));
    }
    uint64_t sk = fr.span0, ap = fr.arena0;
    for (int k = 0; k < 2; ++k) {
        if (!fr.has[k]) continue;
        if (fr.in_batch) {
            const MateRef &m = fr.ref[k];
            RecsView v;
            v.recs = m.base;
            v.idx = m.idx;
            process_mate(h, v, m.n, m.proper, m.np, k, fr, spans, sk, arena, ap, N);
        } else {
            const Frag::MateFields &mf = fr.mf[k];
            RecsView v;
            v.fields = recf.data() + mf.r0;
            process_mate(h, v, mf.nrec, prop.data() + mf.p0, mf.np, k, fr, spans, sk, arena, ap, N);
        }
    }
    fr.dropped = (fr.circ.empty() && h->o.nolinear) || (fr.circ.empty() && fr.lin.empty());
}

// The sink of the ingest's pull loop: the fragment's records are recorded (their fields, the
// primaries' strings) into the chunk's next slot, with room for the spans and read parts it can
// have.  With `defer` the chunk's fragments are processed afterwards on the next side's workers
// (fc2_caller_next); otherwise (-B writes records while reading, and the reference stops at a
// failing fragment) here, raising where process_mate raises.
int on_fragment(fc2_caller *h, MateRef *m1, MateRef *m2, bool defer) {
    // the next slot of the chunk; a recycled Frag is reset field by field (capacity kept)
    if (h->bf_nfrags == h->bf_frags.size()) h->bf_frags.emplace_back();
    Frag &fr = h->bf_frags[h->bf_nfrags];
    fr.in_batch = defer && m2->stable && (!m1 || m1->stable);
    if (!fr.in_batch) fr.name.assign(m2->rec(0).qname);   // Fragment(mate2.primary.qname, ...)
    fr.dropped = false;
    MateRef *ms[2] = {m1, m2};
    fr.span0 = h->bf_nspans;
    fr.arena0 = h->bf_narena;
    uint64_t smax = 0, amax = 0;
    const size_t recf0 = h->bf_recf.size(), prop0 = h->bf_prop.size();
    for (int k = 0; k < 2; ++k) {
        fr.has[k] = ms[k] != nullptr;
        Frag::MateFields &mf = fr.mf[k];
        mf = Frag::MateFields();
        if (!ms[k]) continue;
        const MateRef &m = *ms[k];
        if (m.np >= 2) {
            smax += m.np - 1;
            amax += (uint64_t)(m.np - 1) * m.seq_len;
        }
        if (fr.in_batch) {                      // read in place by process_frag
            fr.ref[k] = m;
            continue;
        }
        mf.r0 = (uint32_t)h->bf_recf.size();
        mf.nrec = m.n;
        for (uint32_t j = 0; j < m.n; ++j) h->bf_recf.push_back(static_cast<const RecFields &>(m.rec(j)));
        mf.p0 = (uint32_t)h->bf_prop.size();
        mf.np = m.np;
        h->bf_prop.insert(h->bf_prop.end(), m.proper, m.proper + m.np);
        take_align(fr.prim[k], m.rec(0));
    }
    fr.span_max = smax;
    h->bf_nspans += smax;
    h->bf_narena += amax;
    ++h->bf_nfrags;
    if (defer) return FC2_OK;
    if (h->bf_spans.size() < h->bf_nspans) h->bf_spans.resize(h->bf_nspans);
    if (h->bf_arena.size() < h->bf_narena) h->bf_arena.resize(h->bf_narena);
    process_frag(h, fr, h->bf_recf, h->bf_prop, h->bf_spans.data(), h->bf_arena.data(), h->N_in);
    if (fr.dropped) {                           // not pending: its spans are never evaluated
        --h->bf_nfrags;                         // the slot is reused by the next fragment
        h->bf_nspans = fr.span0;
        h->bf_narena = fr.arena0;
        h->bf_recf.resize(recf0);
        h->bf_prop.resize(prop0);
    }
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

// the interned chromosome of every span the chunk evaluates, before the workers read tid_cid
// (a reference id outside the header stays unresolved: decode raises chrom_of's error for it)
void resolve_chroms(fc2_caller *h) {
    for (const Span &s : h->spans) {
        if (s.eval < 0 || (s.tid >= 0 && (size_t)s.tid < h->tid_cid.size() && h->tid_cid[(size_t)s.tid] >= 0)) continue;
        const char *nm = s.tid >= 0 ? fc2_ingest_ref_name(h->ing, s.tid) : nullptr;
        if (!nm) continue;
        if ((size_t)s.tid >= h->tid_cid.size()) h->tid_cid.resize((size_t)s.tid + 1, -1);
        h->tid_cid[(size_t)s.tid] = intern(h, nm);
    }
}

// the evaluation results of the pending chunk: the batch's (fc2_caller_submit) and its long pairs'
// (fc2_caller_submit_long)
struct Results {
    const fc2_result *res;
    const uint64_t *tiemask;
    uint32_t tw;
    uint64_t stride;
    const fc2_long_result *lres;
    const uint64_t *lties, *ltie_off;
};

// fills ev (a reused scratch object: its vectors keep their capacity)
void decode(const fc2_caller *h, int si, const Results &R, Eval &ev) {
    ev.err = 0;
    ev.msg.clear();
    ev.ties.clear();
    const Span &s = h->spans[si];
    // the pair and its result, from the batch or the long list (the same fields, wider)
    struct {
        int64_t a_pos, b_aend, L;
        uint32_t chrom;
        uint8_t flags;
    } pr;
    struct {
        int64_t best_x, dist, ov;
        uint64_t n_ties;
        uint16_t info;
    } r;
    const bool is_long = (s.eval & kLongEval) != 0;
    const uint64_t ei = (uint64_t)(s.eval & ~kLongEval);
    if (is_long) {
        const fc2_long_pair &p = h->b_long[ei];
        const fc2_long_result &q = R.lres[ei];
        pr = {p.a_pos, p.b_aend, (int64_t)p.read_len, p.chrom, p.flags};
        r = {q.best_x, q.dist, q.ov, q.n_ties, q.info};
    } else {
        const fc2_pair &p = h->b_pairs[ei];
        const fc2_result &q = R.res[ei];
        pr = {p.a_pos, p.b_aend, (int64_t)p.read_len, p.chrom, p.flags};
        r = {q.best_x, q.dist, q.ov, q.n_ties, q.info};
    }
    // tie bit (strand, x): the batch's tie rows, or the pair's own tie words
    const uint64_t lhalf = is_long ? (R.ltie_off[ei + 1] - R.ltie_off[ei]) / 2 : 0;
    auto tie_bit = [&](int strand, int64_t xx) -> bool {
        const uint64_t k = (uint64_t)(xx >> 6), b = (uint64_t)(xx & 63);
        if (is_long) return (R.lties[R.ltie_off[ei] + (strand ? lhalf : 0) + k] >> b) & 1ull;
        const uint64_t row = strand ? R.tw / 2 + k : k;
        return (R.tiemask[row * R.stride + ei] >> b) & 1ull;
    };
    if (s.tid < 0 || (size_t)s.tid >= h->tid_cid.size() || h->tid_cid[(size_t)s.tid] < 0) {
        (void)chrom_of(h, s.tid);                          // raises for an id outside the header
        throw Fatal{FC2_E_PARAM, "native caller: chromosome of span not resolved"};   // (resolve_chroms)
    }
    const int64_t cid = h->tid_cid[(size_t)s.tid];
    const std::string &chrom = h->id_names[(size_t)cid];    // (nothing below interns a new name)
    if (pr.flags & FC2_PAIR_SKIP) {
        const int32_t c = s.tid < (int32_t)h->tid2chrom.size() ? h->tid2chrom[(size_t)s.tid] : -1;
        if (c < 0) {                            // chromosome missing from the genome (get_data, :193; A's window)
            ev.err = FC2_E_KEY;
            ev.msg = "KeyError: " + py_repr(chrom);
        } else {                                // align_B.aend None: B's window, `B.aend - eff_a` (:902)
            ev.err = FC2_E_FORMAT;
            ev.msg = "TypeError: unsupported operand type(s) for -: 'NoneType' and 'int'";
        }
        return;
    }
    if (r.info & FC2_RES_ERR_KEY) {
        ev.err = FC2_E_KEY;
        ev.msg = "KeyError: splice signal with a byte outside ACGTN (find_circ.py:927)";
        return;
    }
    if (r.info & FC2_RES_ERR_WIN) {
        ev.err = FC2_E_FORMAT;
        // numpy 1.x (Python 2): unequal-length `!=` gives the scalar True, whose .sum() fails (:861-863)
        ev.msg = "AttributeError: 'bool' object has no attribute 'sum'";
        return;
    }
    if (r.best_x < 0) return;
    const int64_t e = h->o.asize - h->o.margin;
    const int64_t L = pr.L, l = L - 2 * e, x = r.best_x;
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
        return;
    }
    // all ties in (x asc, '+' before '-') order from the tie mask (hotpath._expand_ties)
    bool have_win = false;
    std::string winA, winB;
    for (int64_t xx = 0; xx <= l; ++xx) {
        for (int strand = 0; strand < 2; ++strand) {
            if (!tie_bit(strand, xx)) continue;
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
                    if (!have_win) {                // the windows once per pair (:900-902)
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
                        winA = window(a0, a0 + l + 2);
                        winB = window(b1 - l - 2, b1);
                        have_win = true;
                    }
                    auto sl = [](const std::string &w, int64_t p) {   // w[p:p+2]
                        if (p >= (int64_t)w.size()) return std::string();
                        return w.substr((size_t)p, 2);
                    };
                    wg = sl(winA, xx) + sl(winB, xx);
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

std::string test_row(const fc2_caller *h, const Frag &fr, const std::set<Coord> &lin_coords,
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

// the multi_events row (:733-763) as the text before and after the circ junction's name, which
// phase D fills in; raises (need_int) exactly where the row itself would
void multi_row_parts(const fc2_caller *h, const Frag &fr, const CKey &circ, const std::set<Coord> &lin_cons,
                     const std::set<Coord> &lin_incons, const std::set<UCoord> &un_cons,
                     const std::set<UCoord> &un_incons, std::string &p1, std::string &p2) {
    const int64_t score = (int64_t)lin_cons.size() - 10 * (int64_t)lin_incons.size() + (int64_t)un_cons.size() -
                          10 * (int64_t)un_incons.size();
    p1 = key_chrom(h, circ) + "\t" + i2s(circ.start) + "\t" + i2s(circ.end) + "\tME:";
    std::vector<std::string> cols = {i2s(score), key_strand(h, circ), fr.name};
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
    p2 = "\t" + join(cols, "\t") + "\n";
}


// record_hits' per-fragment scratch (find_circ.py:1276-1439): reused objects, so recording a
// fragment allocates nothing beyond what the junction tables keep
struct KeySlot {                                // a junction of the fragment: kind, coordinate, slot
    int kind;
    CKey key;
    uint32_t slot;
};

struct FragScratch {
    std::vector<int> ev_si;                     // find_breakpoints' results of this fragment, by span
    std::vector<Eval> evs;
    size_t n_ev = 0;
    std::vector<KeySlot> circ, lin, junc;       // distinct circ / linear junctions; every junction
    uint32_t warns = 0;                         // Warn bits
    std::vector<std::string> names;             // write_read: the junction names, sorted
    std::string tail;                           // ... and the name part both mates share
    std::string p1, p2;                         // multi_events row parts
    bool comp_ok[2] = {false, false};           // the mate's read passed check_comp in this fragment
    void reset() { n_ev = 0; circ.clear(); lin.clear(); junc.clear(); warns = 0; comp_ok[0] = comp_ok[1] = false; }
};

const std::vector<Splice> &find_breakpoints(const fc2_caller *h, int si, const Results &R, FragScratch &F) {
    size_t k = 0;
    while (k < F.n_ev && F.ev_si[k] != si) ++k;
    if (k == F.n_ev) {                          // first evaluation of this span in the fragment
        if (F.n_ev == F.evs.size()) { F.evs.emplace_back(); F.ev_si.push_back(0); }
        F.ev_si[k] = si;
        decode(h, si, R, F.evs[k]);
        ++F.n_ev;
    }
    const Eval &ev = F.evs[k];
    if (ev.err) throw Fatal{ev.err, ev.msg};
    return ev.ties;
}

// the key of a Splice from decode (cid resolved, strand '+' / '-'): coord_key without interning
CKey splice_key(const Splice &sp) {
    const uint32_t c = (uint32_t)sp.cid, st = sp.strand == "-" ? 1u : 0u;
    return sp.start < sp.end ? CKey{sp.start, sp.end, c, st} : CKey{sp.end, sp.start, c, st};
}

// add a junction to a fragment's list unless its coordinate is there (one junction per coordinate)
void add_unique(std::vector<KeySlot> &v, const KeySlot &x) {
    for (const KeySlot &y : v)
        if (y.kind == x.kind && y.key == x.key) return;
    v.push_back(x);
}

// phase A, one fragment: record_hits (:1276-1439) up to the table updates, which become events;
// raises Fatal exactly where record_hits would, with the same message
void phase_a_frag(const fc2_caller *h, uint32_t fi, const Frag &fr, const Results &R, FragScratch &F,
                  RangeOut &ro) {
    const auto &o = h->o;
    F.reset();
    uint32_t ord = 0;
    auto count = [&](const char *k) { incN_into(ro.N, k, 1.); };
    // Hit.add of one splice (storage_add, :526-582): the raising checks now, the update as an event
    auto store = [&](int kind, const Splice &sp, const Span &span) -> KeySlot {
        if (o.stranded)   // Splice has no strandmatch attribute (:532-533)
            throw Fatal{FC2_E_FORMAT, "AttributeError: 'Splice' object has no attribute 'strandmatch'"};
        if (span.q_bad)   // qA / qB = AS - XS of a str / array tag (:558-559)
            throw sub_error("-", span.q_bad_l, span.q_bad_r);
        if (!F.comp_ok[span.mate]) {            // rev_comp(read) raises here (:573, :582); once per mate
            check_comp(fr.prim[span.mate].seq);
            F.comp_ok[span.mate] = true;
        }
        SEv e;
        e.key = splice_key(sp);
        // input order of the table updates: the fragment's index in the chunk, then its add ordinal
        // (32 bits each: --all-hits ties of long reads can number far beyond 2^20 in one fragment)
        if (ord == UINT32_MAX) throw Fatal{FC2_E_RANGE, "native caller: more than 2^32 - 1 junction updates in one fragment"};
        e.seq = ((uint64_t)fi << 32) | ord++;
        e.frag = fi;
        e.slot = (uint32_t)ro.slots.size();
        ro.slots.emplace_back();
        e.span = sp.span;
        e.dist = (int32_t)sp.dist;
        e.ov = (int32_t)sp.ov;
        e.n_hits = (int32_t)sp.n_hits;
        e.kind = (uint8_t)kind;
        e.op = 0;
        e.warn = 0;
        e.dist_bool = sp.dist_bool;
        e.mate = (uint8_t)span.mate;
        e.gtag_len = (uint8_t)std::min<size_t>(sp.gtag.size(), sizeof e.gtag);
        memcpy(e.gtag, sp.gtag.data(), e.gtag_len);
        ro.ev[shard_of(e.key)].push_back(e);
        return KeySlot{kind, e.key, e.slot};
    };
    auto flag = [&](const KeySlot &j, uint32_t w) {
        SEv e{};
        e.key = j.key;
        e.frag = fi;
        e.slot = j.slot;
        e.kind = 0;
        e.op = 1;
        e.warn = (uint8_t)w;
        ro.ev[shard_of(j.key)].push_back(e);
    };
    auto finish = [&]() {                       // what write_read / the multi row need later
        if (F.junc.empty()) return;
        FOut fo;
        fo.frag = fi;
        fo.warns = F.warns;
        fo.j0 = (uint32_t)ro.jk.size();
        fo.nj = (uint32_t)F.junc.size();
        for (const KeySlot &j : F.junc) ro.jk.emplace_back((uint8_t)j.kind, j.slot);
        ro.fouts.push_back(fo);
    };
    KeySlot circ{0, CKey{}, 0};
    for (int si : fr.circ) {
        const Span &span = h->spans[si];
        if (!uniq_ok(span, o.min_uniq_qual)) { count("circ_junc_not_unique"); continue; }
        const std::vector<Splice> &splices = find_breakpoints(h, si, R, F);
        if (splices.empty()) {
            count("circ_no_bp");
            F.warns |= 1u << W_WARN_UNRESOLVED_EXTRA_BACKSPLICE;
            continue;
        }
        count("circ_spliced");
        const size_t n = o.allhits ? splices.size() : 1;
        for (size_t k = 0; k < n; ++k) {
            circ = store(0, splices[k], span);
            add_unique(F.circ, circ);           // circ_coords: one coordinate per junction
            add_unique(F.junc, circ);
        }
    }
    if (F.circ.size() > 1) {
        for (const KeySlot &j : F.circ) {
            F.warns |= 1u << W_WARN_MULTI_BACKSPLICE;
            flag(j, W_WARN_MULTI_BACKSPLICE);
        }
        finish();
        return;
    }
    if (F.circ.empty() && o.nolinear) { finish(); return; }
    int64_t circ_start = 0, circ_end = 0;
    int circ_span = -1;
    if (!F.circ.empty()) {
        circ = F.circ[0];
        circ_start = circ.key.start;
        circ_end = circ.key.end;
        circ_span = fr.circ[0];
        if (fr.circ.size() > 1) F.warns |= 1u << W_SUPPORT_CLOSURE;
    }
    std::set<Coord> lin_cons, lin_incons;
    for (int si : fr.lin) {
        const Span &span = h->spans[si];
        if (!uniq_ok(span, o.min_uniq_qual)) { count("lin_junc_not_unique"); continue; }
        const std::vector<Splice> &splices = find_breakpoints(h, si, R, F);
        if (splices.empty()) {
            count("lin_no_bp");
            F.warns |= 1u << W_WARN_UNRESOLVED_LINSPLICE;
            continue;
        }
        count("lin_spliced");
        const size_t n = o.allhits ? splices.size() : 1;
        for (size_t k = 0; k < n; ++k) {
            const Splice &sp = splices[k];
            const KeySlot j = store(1, sp, span);
            add_unique(F.junc, j);
            if (o.test) add_unique(F.lin, j);
            if (!F.circ.empty()) {
                if (sp.start <= circ_start || sp.end >= circ_end) {
                    F.warns |= 1u << W_WARN_OUTSIDE_SPLICE_JUNCTION;
                    lin_incons.insert(sp.coord());
                } else {
                    lin_cons.insert(sp.coord());
                    F.warns |= 1u << W_SUPPORT_INSIDE_SPLICE_JUNCTION;
                }
            }
        }
    }
    if (o.test) {
        auto coords = [&](const APos &a) {
            const std::string st = o.stranded ? (a.rev ? "-" : "+") : "*";
            return UCoord{chrom_of(h, a.tid), a.pos, a.aend < 0 ? kNone : a.aend, st};
        };
        std::vector<UCoord> un, br;
        for (const APos &a : fr.unspliced) un.push_back(coords(a));
        for (const APos &a : fr.broken) br.push_back(coords(a));
        std::set<Coord> lin_coords, circ_coords;
        for (const KeySlot &j : F.lin) lin_coords.insert(key_coord(h, j.key));
        for (const KeySlot &j : F.circ) circ_coords.insert(key_coord(h, j.key));
        ro.test += test_row(h, fr, lin_coords, circ_coords, un, br);
    }
    if (!F.circ.empty()) {
        std::set<UCoord> un_cons, un_incons;
        const int32_t circ_tid = fr.prim[h->spans[circ_span].mate].tid;
        for (const APos &a : fr.unspliced) {
            const UCoord c{chrom_of(h, a.tid), a.pos, a.aend < 0 ? kNone : a.aend, "*"};
            if (circ_tid != a.tid) {
                F.warns |= 1u << W_WARN_OTHER_CHROM_MATE;
                un_incons.insert(c);
            } else if (a.pos + o.asize <= circ_start || need_int(c.aend) - o.asize >= circ_end) {
                F.warns |= 1u << W_WARN_OUTSIDE_MATE;
                un_incons.insert(c);
            } else {
                F.warns |= 1u << W_SUPPORT_INSIDE_MATE;
                un_cons.insert(c);
            }
        }
        if (!fr.broken.empty()) F.warns |= 1u << W_BROKEN_SEGMENTS;
        const bool multi = (!un_cons.empty() || !un_incons.empty() || !lin_cons.empty() || !lin_incons.empty()) &&
                           o.multi_events && o.write_multi;
        if (multi) multi_row_parts(h, fr, circ.key, lin_cons, lin_incons, un_cons, un_incons, F.p1, F.p2);
        for (uint32_t w = 0; w < kNumWarn; ++w)
            if (F.warns & (1u << w)) flag(circ, w);
        finish();
        if (multi) {
            FOut &fo = ro.fouts.back();
            fo.m0 = (int64_t)ro.mtext.size();
            fo.m1 = (uint32_t)F.p1.size();
            fo.m2 = (uint32_t)F.p2.size();
            fo.circ_slot = circ.slot;
            ro.mtext += F.p1;
            ro.mtext += F.p2;
        }
        return;
    }
    finish();
}

// phase A over a range of fragments: stops at the first fragment that raises
void phase_a(const fc2_caller *h, size_t f0, size_t f1, const Results &R, RangeOut &ro) {
    static thread_local FragScratch F;
    ro.clear();
    for (size_t f = f0; f < f1; ++f) {
        try {
            phase_a_frag(h, (uint32_t)f, h->frags[f], R, F, ro);
        } catch (const Fatal &e) {              // (a test row written before the error stays, :1361)
            ro.err_frag = (int64_t)f;
            ro.err_code = e.code;
            ro.err_msg = e.msg;
            return;
        }
    }
}

// phase B, one shard: its events of every range in input order, up to the failing fragment fe
void phase_b(fc2_caller *h, int s, size_t n_ranges, uint64_t fe) {
    Shard &S = h->sh[s];
    S.fresh[0].clear();
    S.fresh[1].clear();
    constexpr size_t kAhead = 8;
    for (size_t r = 0; r < n_ranges; ++r) {
        RangeOut &ro = h->ranges[r];
        const std::vector<SEv> &v = ro.ev[s];
        for (size_t k = 0; k < v.size(); ++k) {
            const SEv &e = v[k];
            if (e.frag >= fe) break;
            if (k + kAhead < v.size()) S.index[v[k + kAhead].kind].prefetch(v[k + kAhead].key);
            if (e.op == 0) {
                HitVec &hv = S.hits[e.kind];
                const auto ins = S.index[e.kind].try_emplace(e.key, hv.size());
                if (ins.second) {
                    Hit &t = hv.emplace_back();
                    t.key = e.key;
                    S.fresh[e.kind].emplace_back(e.seq, (uint32_t)ins.first);
                }
                Hit &t = hv[ins.first];
                hit_apply(h, t, e);
                const Span &span = h->spans[(size_t)e.span];
                hit_add_read(S.strings, t, span, h->frags[e.frag].prim[e.mate]);
                ro.slots[e.slot] = JRef{(uint32_t)s, (uint32_t)ins.first};
            } else {
                const JRef j = ro.slots[e.slot];
                add_flag(S.strings, S.hits[0][j.idx], e.warn, h->frags[e.frag].name);
            }
        }
    }
}

// phase C: the chunk's new junctions named in order of first appearance (:684-686)
void phase_c(fc2_caller *h) {
    for (int kind = 0; kind < 2; ++kind) {
        size_t pos[kShards] = {};
        for (;;) {                              // merge of the shards' lists (each in seq order)
            int best = -1;
            uint64_t bseq = 0;
            for (int s = 0; s < kShards; ++s) {
                const auto &fl = h->sh[s].fresh[kind];
                if (pos[s] < fl.size() && (best < 0 || fl[pos[s]].first < bseq)) { best = s; bseq = fl[pos[s]].first; }
            }
            if (best < 0) break;
            const uint32_t idx = h->sh[best].fresh[kind][pos[best]++].second;
            h->sh[best].hits[kind][idx].novel = ++h->novel[kind];
            h->order[kind].push_back(JRef{(uint32_t)best, idx});
        }
    }
}

// phase D over a range: read names (write_read, :1442-1447) and multi_events rows, which need the
// junction names, for the fragments before fe
void phase_d(const fc2_caller *h, RangeOut &ro, uint64_t fe) {
    static thread_local FragScratch F;
    for (const FOut &fo : ro.fouts) {
        if (fo.frag >= fe) break;
        const Frag &fr = h->frags[fo.frag];
        if (fo.m0 >= 0) {
            ro.out1.append(ro.mtext, (size_t)fo.m0, fo.m1);
            hit_name(h, 0, hit_at(h, 0, ro.slots[fo.circ_slot]), ro.out1);
            ro.out1.append(ro.mtext, (size_t)fo.m0 + fo.m1, fo.m2);
        }
        if (!h->o.write_reads) continue;
        // ' <sorted junction names> <sorted flags>': the part of the read names both mates share
        const size_t nj = fo.nj;
        if (F.names.size() < nj) F.names.resize(nj);
        for (size_t k = 0; k < nj; ++k) {
            const auto &j = ro.jk[fo.j0 + k];
            F.names[k].clear();
            hit_name(h, j.first, hit_at(h, j.first, ro.slots[j.second]), F.names[k]);
        }
        if (nj > 1) std::sort(F.names.begin(), F.names.begin() + (std::ptrdiff_t)nj);
        std::string &t = F.tail;
        t.assign(1, ' ');
        for (size_t k = 0; k < nj; ++k) {
            if (k) t += ',';
            t += F.names[k];
        }
        t += ' ';
        bool first = true;
        for (uint32_t w = 0; w < kNumWarn; ++w)
            if (fo.warns & (1u << w)) { if (!first) t += ','; t += kWarnName[w]; first = false; }
        for (int m = 0; m < 2; ++m) {
            if (!fr.has[m]) continue;
            // '@<qname> <sorted junction names> <sorted flags>' , seq, '+' + the same name, qual
            const Align &a = fr.prim[m];
            std::string &o = ro.out0;
            o += '@';
            const size_t n0 = o.size();
            o += a.qname;
            o += t;
            const size_t n1 = o.size();
            o += '\n';
            if (a.has_seq) o += a.seq;
            else o += "None";
            o += "\n+";
            o.append(o, n0, n1 - n0);
            o += '\n';
            if (a.has_qual) o += a.qual;
            else o += "None";
            o += '\n';
        }
    }
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
    if (const char *env = getenv("FC2_CALLER_MIN_RANGE"))   // fragments per phase-A range at least (tests)
        if (atoi(env) > 0) h->min_range_frags = (size_t)atoi(env);
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

extern "C" int fc2_caller_inflate_counts(const fc2_caller *h, uint64_t *gpu_blocks, uint64_t *cpu_blocks) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_caller_inflate_counts: null argument");
    if (!h->read_side_released) return fc2_ingest_inflate_counts(h->ing, gpu_blocks, cpu_blocks);
    if (gpu_blocks) *gpu_blocks = h->inflate_final[0];
    if (cpu_blocks) *cpu_blocks = h->inflate_final[1];
    return FC2_OK;
}

// the input's counts: live, or as they were when the input was released (release_read_side)
static void ingest_counts(const fc2_caller *h, fc2_ingest_counts *c) {
    if (h->read_side_released) *c = h->ing_final;
    else fc2_ingest_counts_get(h->ing, c);
}

extern "C" void fc2_caller_close(fc2_caller *h) {
    if (!h) return;
    if (h->release_thr.joinable()) h->release_thr.join();   // the read side's release (fc2_caller_rows)
    fc2_ingest_close(h->ing);                   // (joins the parse-ahead threads)
    delete h;
    if (fc2::cpu::enabled()) {                  // CPU seconds per stage over the run (fc2_cpuacct.h)
        static const char *const kName[fc2::cpu::kStages] = {"inflate", "split", "parse+group", "consumer",
                                                              "next pool", "submit pool", "submit serial", "gzip"};
        std::atomic<int64_t> *t = fc2::cpu::totals();
        fprintf(stderr, "cpu s:");
        for (int k = 0; k < fc2::cpu::kStages; ++k) fprintf(stderr, " %s %.3f", kName[k], (double)t[k].exchange(0) * 1e-9);
        fprintf(stderr, "\n");
    }
}

// a fragment of a bulk-recorded run (fc2_caller::Seg): what on_fragment writes for one recorded in
// place, from its GFrag
static void fill_from_seg(const fc2_caller::Seg &sg, size_t f, Frag &fr) {
    const size_t i = f - sg.f0;
    const fc2::ing::GFrag &g = sg.r.g[i];
    const uint64_t sb = i ? sg.r.g[i - 1].span_cum : sg.r.span_before;
    const uint64_t ab = i ? sg.r.g[i - 1].arena_cum : sg.r.arena_before;
    fr.in_batch = true;
    fr.dropped = false;
    fr.span0 = sg.span0 + (sb - sg.r.span_before);
    fr.arena0 = sg.arena0 + (ab - sg.r.arena_before);
    fr.span_max = g.span_cum - sb;
    for (int k = 0; k < 2; ++k) {
        fr.has[k] = k == 1 || g.n[0] != 0;
        fr.mf[k] = Frag::MateFields();
        if (!fr.has[k]) continue;
        MateRef &m = fr.ref[k];
        m.base = sg.r.recs;
        m.idx = sg.r.gidx + g.r0[k];
        m.n = (uint32_t)g.n[k];
        m.proper = sg.r.gidx + g.p0[k];
        m.np = (uint32_t)g.np[k];
        m.seq_len = g.seq_len[k];
        m.stable = true;
    }
}

// the next side's workers (FC2_NEXT_THREADS, default min(8, cores)): process_mate over fragment
// ranges, the chunk's pairs
static void ensure_next_pool(fc2_caller *h) {
    if (h->next_pool) return;
    const char *env = getenv("FC2_NEXT_THREADS");
    const int nt = env && atoi(env) > 0 ? atoi(env) : (int)std::min(8u, std::max(1u, std::thread::hardware_concurrency()));
    h->next_pool.reset(new WorkPool(std::max(1, std::min(nt, 64)) - 1));
}

extern "C" int fc2_caller_next(fc2_caller *h, fc2_caller_batch *b, int *eof) {
    if (!h || !b) return fc2::fail(FC2_E_PARAM, "fc2_caller_next: null argument");
    struct PublishStats {                          // on every way out of this call
        fc2_caller *h;
        ~PublishStats() {
            fc2_ingest_counts c{};
            ingest_counts(h, &c);
            h->st_reads.store(c.n_reads, std::memory_order_relaxed);
            h->st_pairs.store(h->n_pairs, std::memory_order_relaxed);
        }
    } publish{h};
    {
        std::lock_guard<std::mutex> lk(h->qmu);
        if (h->queued.size() >= FC2_CALLER_MAX_QUEUED)
            return fc2::fail(FC2_E_PARAM, "fc2_caller_next: too many chunks not submitted");
    }
    if (h->read_side_released) {                   // the input was read to its end and closed
        memset((void *)b, 0, sizeof(*b));
        if (eof) *eof = 1;
        return FC2_OK;
    }
    {
        std::lock_guard<std::mutex> lk(h->qmu);
        if (!h->spare.empty()) {                   // a recorded chunk's buffers (see fc2_caller::spare)
            fc2_caller::Chunk &c = h->spare.back();
            h->bf_frags.swap(c.frags);
            h->bf_spans.swap(c.spans);
            h->bf_arena.swap(c.arena);
            h->bf_off.swap(c.b_off);
            h->bf_pairs.swap(c.b_pairs);
            h->bf_long.swap(c.b_long);
            h->spare.pop_back();
        }
    }
    if (h->next_err) {
        const int code = h->next_err;
        h->next_err = FC2_OK;
        return fc2::fail(code, h->next_err_msg);
    }
    h->bf_nfrags = 0;
    h->bf_nspans = h->bf_narena = 0;
    h->bf_segs.clear();
    h->bf_recf.clear();
    h->bf_prop.clear();
    h->bf_off.clear();
    h->bf_pairs.clear();
    h->bf_long.clear();
    // the chunk's fragments are processed after they are all read, on the next side's workers --
    // unless -B writes records while reading (the reference's writer stops at a failing fragment)
    const bool defer = !fc2::ing::writes_records(h->ing);
    // fragments grouped on the parse threads are recorded in place: their batches stay pinned until
    // this chunk's fragments are processed below
    fc2::ing::set_pin(h->ing, defer);
    Fatal err{0, ""};
    // a run of fragments grouped on a parse thread: recorded whole, each fragment's slot filled by
    // the workers below (fill_from_seg); its spans and read parts take their room here
    const fc2::ing::BulkSink bulk = [&](const fc2::ing::RegionRef &r) -> int {
        h->bf_segs.push_back(fc2_caller::Seg{r, h->bf_nfrags, h->bf_nspans, h->bf_narena});
        const size_t need = h->bf_nfrags + r.n;
        if (h->bf_frags.size() < need) h->bf_frags.resize(need);
        h->bf_nfrags = need;
        h->bf_nspans += r.g[r.n - 1].span_cum - r.span_before;
        h->bf_narena += r.g[r.n - 1].arena_cum - r.arena_before;
        return FC2_OK;
    };
    const fc2::ing::FragSink sink = [&](MateRef *m1, MateRef *m2, bool) -> int {
        try {
            return on_fragment(h, m1, m2, defer);
        } catch (const Fatal &f) {
            err = f;
            return f.code ? f.code : FC2_E_FORMAT;
        }
    };
    // the first chunks ramp up (1/16, 1/8, 1/4, 1/2 of chunksize): the recording side starts early
    // instead of waiting for a whole first chunk; chunk boundaries change nothing in the outputs
    const uint64_t limit = std::max<uint64_t>(1, (uint64_t)h->o.chunksize >> (h->n_chunks < 4 ? 4 - h->n_chunks : 0));
    ++h->n_chunks;
    if (h->bf_frags.size() < limit + 1) h->bf_frags.reserve(limit + 1);   // no Frag moved while the chunk forms
    int in_code = FC2_OK;                      // an error of the input (or, without defer, of a fragment)
    std::string in_msg;
    static const bool timing = getenv("FC2_CALLER_TIMING") != nullptr;   // phase times on stderr
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t0 = now();
    fc2::cpu::Scope acct(fc2::cpu::CONSUME);      // this thread's share of the call (the pools count apart)
    while (!h->eof && h->bf_nfrags < limit && !fc2::ing::pin_full(h->ing)) {
        int e = 0;
        const int rc = fc2::ing::pull(h->ing, &h->ip, limit - h->bf_nfrags, sink, &e,   // at most `limit` per chunk
                                      defer ? &bulk : nullptr);
        if (rc) {
            in_code = err.code ? err.code : rc;
            in_msg = err.code ? err.msg : std::string(fc2_last_error());
            break;
        }
        h->eof = e != 0;
    }
    const auto t1 = now();
    if (defer) {
        // process_mate of every fragment on the workers, in ranges; the first fragment that raises
        // ends the chunk there (an input error after it is never reached)
        h->bf_spans.resize(h->bf_nspans);
        h->bf_arena.resize(h->bf_narena);
        ensure_next_pool(h);
        const size_t nf = h->bf_nfrags;
        const size_t T = std::max<size_t>(1, std::min<size_t>((size_t)h->next_pool->size(),
                                                              nf / std::max<size_t>(1, h->min_range_frags)));
        if (h->next_N.size() < T) h->next_N.resize(T);
        h->next_err_at.assign(T, std::pair<int64_t, Fatal>(-1, Fatal{0, ""}));
        Span *spans = h->bf_spans.data();
        char *arena = h->bf_arena.data();
        h->next_pool->run_checked((int)T, [&](int r) {
            fc2::cpu::Scope acct(fc2::cpu::NEXT_POOL);
            auto &N = h->next_N[(size_t)r];
            N.clear();
            const size_t fa = nf * (size_t)r / T;
            // the first run (bulk-recorded) not ending before fa
            size_t si = (size_t)(std::upper_bound(h->bf_segs.begin(), h->bf_segs.end(), fa,
                                                  [](size_t f, const fc2_caller::Seg &sg) { return f < sg.f0; }) -
                                 h->bf_segs.begin());
            if (si) --si;
            for (size_t f = fa, f1 = nf * (size_t)(r + 1) / T; f < f1; ++f) {
                while (si < h->bf_segs.size() && h->bf_segs[si].f0 + h->bf_segs[si].r.n <= f) ++si;
                if (si < h->bf_segs.size() && h->bf_segs[si].f0 <= f) fill_from_seg(h->bf_segs[si], f, h->bf_frags[f]);
                try {
                    process_frag(h, h->bf_frags[f], h->bf_recf, h->bf_prop, spans, arena, N);
                } catch (const Fatal &x) {
                    h->next_err_at[(size_t)r] = {(int64_t)f, x};
                    return;
                }
            }
        });
        size_t fe = nf;
        for (size_t r = 0; r < T; ++r) {
            for (const auto &kv : h->next_N[r]) incN_in(h, kv.first, kv.second);
            if (h->next_err_at[r].first >= 0) {
                fe = (size_t)h->next_err_at[r].first;
                in_code = h->next_err_at[r].second.code ? h->next_err_at[r].second.code : FC2_E_FORMAT;
                in_msg = h->next_err_at[r].second.msg;
                break;
            }
        }
        if (fe < nf) h->bf_spans.resize(h->bf_frags[fe].span0);   // no span of a fragment not processed
        // drop the fragments with no span record_hits looks at (rare: the ingest hands out only
        // fragments with pairs), keeping the order
        size_t k = 0;
        for (size_t f = 0; f < fe; ++f) {
            if (h->bf_frags[f].dropped) continue;
            if (k != f) std::swap(h->bf_frags[k], h->bf_frags[f]);
            ++k;
        }
        h->bf_nfrags = k;
        fc2::ing::release(h->ing);             // every kept fragment has taken what it needs
    }
    const auto t2 = now();
    if (in_code) {
        if (!h->bf_nfrags) return fc2::fail(in_code, in_msg);
        h->next_err = in_code;                     // hand out the fragments before it first
        h->next_err_msg = in_msg;
    }
    // the spans record_hits will evaluate, in fragment order (Caller._flush): counted per fragment
    // range, then written at each range's offset, on the next side's workers
    {
        ensure_next_pool(h);
        const size_t nf = h->bf_nfrags;
        const size_t T = std::max<size_t>(1, std::min<size_t>((size_t)h->next_pool->size(),
                                                              nf / std::max<size_t>(1, h->min_range_frags)));
        // (pairs with read parts over FC2_MAX_READ_LEN go to the long list: counted apart)
        std::vector<uint64_t> cnt(T + 1, 0), cnt_long(T + 1, 0);
        const int64_t min_uq = h->o.min_uniq_qual;
        auto eligible = [&](const Span &sp) { return uniq_ok(sp, min_uq); };
        h->next_pool->run((int)T, [&](int r) {
            fc2::cpu::Scope acct(fc2::cpu::NEXT_POOL);
            uint64_t n = 0, nl = 0;
            for (size_t f = nf * (size_t)r / T, f1 = nf * (size_t)(r + 1) / T; f < f1; ++f) {
                const Frag &fr = h->bf_frags[f];
                for (int pass = 0; pass < 2; ++pass)
                    for (int si : pass ? fr.lin : fr.circ) {
                        const Span &sp = h->bf_spans[si];
                        if (!eligible(sp)) continue;
                        if (sp.read_len > FC2_MAX_READ_LEN) ++nl; else ++n;
                    }
            }
            cnt[(size_t)r + 1] = n;
            cnt_long[(size_t)r + 1] = nl;
        });
        for (size_t r = 0; r < T; ++r) {
            cnt[r + 1] += cnt[r];
            cnt_long[r + 1] += cnt_long[r];
        }
        h->bf_pairs.resize(cnt[T]);
        h->bf_off.resize(cnt[T]);
        h->bf_long.resize(cnt_long[T]);
        h->next_pool->run((int)T, [&](int r) {
            fc2::cpu::Scope acct(fc2::cpu::NEXT_POOL);
            uint64_t k = cnt[(size_t)r], kl = cnt_long[(size_t)r];
            for (size_t f = nf * (size_t)r / T, f1 = nf * (size_t)(r + 1) / T; f < f1; ++f) {
                const Frag &fr = h->bf_frags[f];
                for (int pass = 0; pass < 2; ++pass) {
                    for (int si : pass ? fr.lin : fr.circ) {
                        Span &sp = h->bf_spans[si];
                        if (!eligible(sp)) continue;
                        // align_B.aend None: not scanned; find_breakpoints raises when it reaches B's
                        // window (decode)
                        const bool none_aend = sp.b_aend < 0;
                        const int32_t c = (sp.tid >= 0 && sp.tid < (int32_t)h->tid2chrom.size()) ? h->tid2chrom[sp.tid] : -1;
                        const uint8_t flags = (uint8_t)((sp.circ ? FC2_PAIR_BACKSPLICE : 0) |
                                                        (fr.prim[sp.mate].rev ? FC2_PAIR_PRIMARY_REV : 0) |
                                                        (c < 0 || none_aend ? FC2_PAIR_SKIP : 0));
                        if (sp.read_len > FC2_MAX_READ_LEN) {
                            fc2_long_pair lp{};
                            lp.read_off = sp.read_off;
                            lp.read_len = sp.read_len;
                            lp.chrom = c < 0 ? 0u : (uint32_t)c;
                            lp.a_pos = (int32_t)sp.a_pos;
                            lp.b_aend = none_aend ? 0 : (int32_t)sp.b_aend;
                            lp.flags = flags;
                            sp.eval = kLongEval | (int64_t)kl;
                            h->bf_long[kl++] = lp;
                            continue;
                        }
                        fc2_pair pr{};
                        pr.a_pos = (int32_t)sp.a_pos;
                        pr.b_aend = none_aend ? 0 : (int32_t)sp.b_aend;
                        pr.chrom = c < 0 ? 0u : (uint32_t)c;
                        pr.read_len = (uint16_t)sp.read_len;
                        pr.flags = flags;
                        sp.eval = (int64_t)k;
                        h->bf_pairs[k] = pr;
                        h->bf_off[k] = sp.read_off;
                        ++k;
                    }
                }
            }
        });
    }
    if (h->bf_spans.size() > h->bf_nspans) h->bf_spans.resize(h->bf_nspans);
    h->n_pairs += h->bf_pairs.size() + h->bf_long.size();
    if (timing) {
        uint64_t grouped = 0;
        const double wait = fc2::ing::take_wait_ms(h->ing, &grouped);
        double iw, sb, pi;
        fc2::ing::take_stage_ms(h->ing, &iw, &sb, &pi);
        fprintf(stderr, "next nf=%zu read=%.2f (waiting for parsers %.2f, grouped there %llu) process=%.2f pairs=%.2f ms"
                " | upstream: inflate wait %.2f, splitter blocked %.2f, parsers idle %.2f ms\n",
                h->bf_nfrags, ms(t0, t1), wait, (unsigned long long)grouped, ms(t1, t2), ms(t2, now()), iw, sb, pi);
    }
    h->bf_arena.resize(h->bf_narena + 16);       // readers of the batch may load whole words past the end
    memset(h->bf_arena.data() + h->bf_narena, 0, 16);
    fc2_caller::Chunk c;
    c.frags.swap(h->bf_frags);
    c.nfrags = h->bf_nfrags;
    h->bf_nfrags = 0;
    c.spans.swap(h->bf_spans);
    c.arena.swap(h->bf_arena);
    c.b_off.swap(h->bf_off);
    c.b_pairs.swap(h->bf_pairs);
    c.b_long.swap(h->bf_long);
    std::lock_guard<std::mutex> lk(h->qmu);
    h->queued.push_back(std::move(c));           // moved vectors keep their buffers: *b stays valid
    const fc2_caller::Chunk &q = h->queued.back();
    b->n = q.b_pairs.size();
    b->reads = (const uint8_t *)q.arena.data();
    b->read_off = q.b_off.data();
    b->pairs = q.b_pairs.data();
    b->n_long = q.b_long.size();
    b->long_pairs = q.b_long.data();
    if (eof) *eof = h->eof && !h->next_err ? 1 : 0;   // an error still to report: not the end yet
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
        if (!c.b_long.empty() && !h->l_staged)   // (the chunk stays queued: they may still be staged)
            return fc2::fail(FC2_E_PARAM, "fc2_caller_submit: the chunk's long pairs have no results "
                                          "(fc2_caller_submit_long)");
        h->frags.swap(c.frags);
        h->nfrags = c.nfrags;
        h->spans.swap(c.spans);
        h->arena.swap(c.arena);
        h->b_off.swap(c.b_off);
        h->b_pairs.swap(c.b_pairs);
        h->b_long.swap(c.b_long);
        h->queued.pop_front();
        h->l_staged = false;                     // (l_res / l_ties stay for this chunk's record_hits)
    }
    if (!h->b_pairs.empty() && !results) return fc2::fail(FC2_E_PARAM, "fc2_caller_submit: results missing");
    if (h->o.allhits && !h->b_pairs.empty() && (!tiemask || tw < 2 || stride < h->b_pairs.size()))
        return fc2::fail(FC2_E_PARAM, "fc2_caller_submit: --all-hits needs the tie mask");
    const Results R{results, tiemask, tw, stride, h->l_res.data(), h->l_ties.data(), h->l_tie_off.data()};
    int rc = FC2_OK;
    try {
        resolve_chroms(h);
        if (!h->pool) {
            const char *env = getenv("FC2_CALLER_THREADS");
            int nt = env && atoi(env) > 0 ? atoi(env) : (int)std::min(12u, std::max(1u, std::thread::hardware_concurrency()));
            nt = std::max(1, std::min(nt, 64));
            h->pool.reset(new WorkPool(nt - 1));
        }
        // (A) ranges of fragments -> events per shard, text that needs no names
        const size_t nf = h->nfrags;
        const size_t T = std::max<size_t>(1, std::min<size_t>((size_t)h->pool->size(), nf / std::max<size_t>(1, h->min_range_frags)));
        if (h->ranges.size() < T) h->ranges.resize(T);
        static const bool timing = getenv("FC2_CALLER_TIMING") != nullptr;
        auto now = [] { return std::chrono::steady_clock::now(); };
        const auto t0 = now();
        struct rusage ru0;
        getrusage(RUSAGE_SELF, &ru0);
        h->pool->run_checked((int)T, [&](int r) {
            fc2::cpu::Scope acct(fc2::cpu::SUBMIT_POOL);
            phase_a(h, nf * (size_t)r / T, nf * (size_t)(r + 1) / T, R, h->ranges[(size_t)r]);
        });
        uint64_t fe = nf;                       // the first fragment that raised (or none)
        size_t n_r = T;                         // the ranges that count: up to the one that raised
        for (size_t r = 0; r < T; ++r)
            if (h->ranges[r].err_frag >= 0) { fe = (uint64_t)h->ranges[r].err_frag; n_r = r + 1; break; }
        // (B) the shards apply their events in input order; (C) names; (D) read names, multi rows
        const auto t1 = now();
        h->pool->run_checked(kShards, [&](int sidx) {
            fc2::cpu::Scope acct(fc2::cpu::SUBMIT_POOL);
            phase_b(h, sidx, n_r, fe);
        });
        const auto t2 = now();
        {
            fc2::cpu::Scope acct(fc2::cpu::SUBMIT_SERIAL);
            phase_c(h);
        }
        const auto t3 = now();
        h->pool->run_checked((int)n_r, [&](int r) {
            fc2::cpu::Scope acct(fc2::cpu::SUBMIT_POOL);
            phase_d(h, h->ranges[(size_t)r], fe);
        });
        const auto t4 = now();
        if (timing) {
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            struct rusage ru1;
            getrusage(RUSAGE_SELF, &ru1);
            fprintf(stderr, "submit nf=%zu T=%zu A=%.2f B=%.2f C=%.2f D=%.2f ms minflt=%ld user=%.1f sys=%.1f ms\n", nf, T,
                    ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4), ru1.ru_minflt - ru0.ru_minflt,
                    (ru1.ru_utime.tv_sec - ru0.ru_utime.tv_sec) * 1e3 + (ru1.ru_utime.tv_usec - ru0.ru_utime.tv_usec) / 1e3,
                    (ru1.ru_stime.tv_sec - ru0.ru_stime.tv_sec) * 1e3 + (ru1.ru_stime.tv_usec - ru0.ru_stime.tv_usec) / 1e3);
        }
        for (size_t r = 0; r < n_r; ++r) {
            RangeOut &ro = h->ranges[r];
            for (const auto &kv : ro.N) incN(h, kv.first, kv.second);
            if (h->reads_gz.is_open()) {
                h->reads_gz.append_owned(ro.out0);   // each range's text is one gzip member, not copied
            } else {
                h->out[0] += ro.out0;
            }
            h->out[1] += ro.out1;
            h->out[2] += ro.test;
        }
        if (fe < nf) {
            const RangeOut &ro = h->ranges[n_r - 1];
            rc = fc2::fail(ro.err_code, ro.err_msg);
        }
    } catch (const Fatal &f) {
        rc = fc2::fail(f.code, f.msg);
    }
    if (h->reads_gz.is_open() && !h->out[0].empty()) h->reads_gz.append(h->out[0]);
    // hand the chunk's buffers back to the next side (fc2_caller::spare)
    fc2_caller::Chunk c;
    c.frags.swap(h->frags);
    c.spans.swap(h->spans);
    c.arena.swap(h->arena);
    c.b_off.swap(h->b_off);
    c.b_pairs.swap(h->b_pairs);
    c.b_long.swap(h->b_long);
    h->nfrags = 0;
    std::lock_guard<std::mutex> lk(h->qmu);
    if (h->spare.size() < 4) h->spare.push_back(std::move(c));
    return rc;
}

extern "C" int fc2_caller_submit_long(fc2_caller *h, const fc2_long_result *results, uint64_t n_long,
                                      const uint64_t *ties, uint64_t n_tie_words) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_caller_submit_long: null argument");
    std::lock_guard<std::mutex> lk(h->qmu);
    if (h->queued.empty()) return fc2::fail(FC2_E_PARAM, "fc2_caller_submit_long: no chunk handed out by fc2_caller_next");
    const std::vector<fc2_long_pair> &lp = h->queued.front().b_long;
    if (n_long != lp.size())
        return fc2::fail(FC2_E_PARAM, "fc2_caller_submit_long: " + std::to_string(n_long) + " results for " +
                                          std::to_string(lp.size()) + " long pairs");
    if (n_long && !results) return fc2::fail(FC2_E_PARAM, "fc2_caller_submit_long: results missing");
    fc2_params p{};
    p.asize = h->o.asize;
    p.margin = h->o.margin;
    p.maxdist = h->o.maxdist;
    p.noncanonical = h->o.noncanonical;
    p.allhits = h->o.allhits;
    h->l_tie_off.resize(n_long + 1);
    if (int rc = fc2_long_geometry(&p, n_long, lp.data(), nullptr, h->l_tie_off.data())) return rc;
    if (h->o.allhits) {
        if (n_tie_words != h->l_tie_off[n_long] || (n_tie_words && !ties))
            return fc2::fail(FC2_E_PARAM, "fc2_caller_submit_long: --all-hits needs " +
                                              std::to_string(h->l_tie_off[n_long]) + " tie words");
        h->l_ties.assign(ties, ties + n_tie_words);
    } else {
        h->l_ties.clear();
    }
    h->l_res.assign(results, results + n_long);
    h->l_staged = true;
    return FC2_OK;
}

extern "C" int fc2_caller_submit_compact(fc2_caller *h, const void *words, int width, uint64_t n_words,
                                         const fc2_result_escape *esc, uint64_t n_esc, const uint64_t *tiemask,
                                         uint32_t tw, uint64_t stride) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_caller_submit_compact: null argument");
    size_t n = 0;
    {
        std::lock_guard<std::mutex> lk(h->qmu);
        if (h->queued.empty())
            return fc2::fail(FC2_E_PARAM, "fc2_caller_submit_compact: no chunk handed out by fc2_caller_next");
        n = h->queued.front().b_pairs.size();
    }
    if (n_words != n)
        return fc2::fail(FC2_E_PARAM, "fc2_caller_submit_compact: " + std::to_string(n_words) +
                                          " words for a batch of " + std::to_string(n) + " pairs");
    // the chunk's 8-byte results back from the transfer form, into per-thread scratch (a chunk's
    // worth: what record_hits reads next, still in cache)
    static thread_local std::vector<fc2_result> scratch;
    scratch.resize(std::max<size_t>(n, 1));
    if (n) {
        fc2_params p{};
        p.asize = h->o.asize;
        p.margin = h->o.margin;
        p.maxdist = h->o.maxdist;
        p.noncanonical = h->o.noncanonical;
        if (int rc = fc2_result_expand(&p, words, width, n, esc, n_esc, scratch.data(), 1)) return rc;
    }
    return fc2_caller_submit(h, n ? scratch.data() : nullptr, tiemask, tw, stride);
}

extern "C" int fc2_caller_take(fc2_caller *h, int stream, const char **text, uint64_t *len) {
    if (!h || stream < 0 || stream > 2 || !text || !len) return fc2::fail(FC2_E_PARAM, "fc2_caller_take: bad arguments");
    // each stream has its own hand-out buffer, so both keep their capacity (no regrowth per chunk)
    std::string &t = h->taken[stream];
    t.swap(h->out[stream]);
    h->out[stream].clear();
    *text = t.c_str();
    *len = t.size();
    return FC2_OK;
}

extern "C" int fc2_caller_set_reads_gz(fc2_caller *h, const char *path, int level, int threads, uint64_t piece) {
    if (!h || !path || level < 0 || level > 9) return fc2::fail(FC2_E_PARAM, "fc2_caller_set_reads_gz: bad arguments");
    if (h->reads_gz.is_open() || h->n_pairs) return fc2::fail(FC2_E_PARAM, "fc2_caller_set_reads_gz: call once, before reading");
    std::string err;
    if (!h->reads_gz.open(path, level, threads, piece ? (size_t)piece : size_t(4) << 20, err))
        return fc2::fail(FC2_E_IO, err);
    return FC2_OK;
}

extern "C" int fc2_caller_close_reads(fc2_caller *h) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_caller_close_reads: null argument");
    if (h->reads_gz.is_open() && !h->out[0].empty()) h->reads_gz.append(h->out[0]);
    std::string err;
    if (!h->reads_gz.close(err)) return fc2::fail(FC2_E_IO, err);
    return FC2_OK;
}

// Once the input is read and every chunk recorded, the read side -- the recycled chunks, the
// fragments, spans and read parts of both sides, and the input itself with its parse blocks -- is
// only memory: it is destroyed on a thread of their own while the rows are formatted, and the freed
// heap is handed back (malloc_trim), so neither the rows nor the process's exit pay for its pages.
static void release_read_side(fc2_caller *h) {
#ifdef FC2_AB_NO_RELEASE                        // A/B build only (scripts/prof/ab_cli.py): keep it all
    return;
#endif
    if (h->read_side_released || !h->eof || h->next_err) return;
    {
        std::lock_guard<std::mutex> g(h->qmu);
        if (!h->queued.empty()) return;
    }
    fc2_ingest_counts_get(h->ing, &h->ing_final);
    fc2_ingest_inflate_counts(h->ing, &h->inflate_final[0], &h->inflate_final[1]);
    h->read_side_released = true;
    struct Bag {
        std::vector<fc2_caller::Chunk> spare;
        std::vector<Frag> f[2];
        std::vector<Span> s[2];
        ByteBuf a[2];
        std::vector<RecFields> recf;
        std::vector<fc2_caller::Seg> segs;
    };
    std::unique_ptr<Bag> b(new Bag);
    b->spare.swap(h->spare);
    b->f[0].swap(h->bf_frags), b->f[1].swap(h->frags);
    b->s[0].swap(h->bf_spans), b->s[1].swap(h->spans);
    b->a[0].swap(h->bf_arena), b->a[1].swap(h->arena);
    b->recf.swap(h->bf_recf);
    b->segs.swap(h->bf_segs);
    h->bf_nfrags = h->nfrags = 0;
    // the input too: its parse blocks and records (~0.75 GB at 2M reads) -- fc2_caller_ingest returns
    // NULL from here on, fc2_caller_next reports the end, the counters come from ing_final
    fc2_ingest *ing = h->ing;
    h->ing = nullptr;
    try {
        h->release_thr = std::thread([bag = std::move(b), ing]() mutable {
            fc2_ingest_close(ing);
            bag.reset();
            malloc_trim(0);
        });
    } catch (const std::system_error &) {       // no thread: here, then
        fc2_ingest_close(ing);
    }
}

extern "C" int fc2_caller_rows(fc2_caller *h, int kind, const char **text, uint64_t *len) {
    if (!h || kind < 0 || kind > 1 || !text || !len) return fc2::fail(FC2_E_PARAM, "fc2_caller_rows: bad arguments");
    release_read_side(h);
    h->rows_text.clear();
    // the rows of ranges of the dict order formatted on the workers, joined in order
    const size_t nj = h->order[kind].size();
    const size_t T = std::max<size_t>(1, std::min<size_t>(h->pool ? (size_t)h->pool->size() : 1, nj / 4096));
    std::vector<std::string> parts(T);
    std::vector<std::vector<std::pair<const char *, double>>> Ns(T);
    auto range = [&](int r) { storage_rows(h, kind, nj * (size_t)r / T, nj * (size_t)(r + 1) / T, parts[(size_t)r], Ns[(size_t)r]); };
    try {
        if (T > 1) h->pool->run_checked((int)T, range);
        else range(0);
    } catch (const std::bad_alloc &) {
        return fc2::fail(FC2_E_PARAM, "fc2_caller_rows: out of memory");
    }
    size_t total = 0;
    for (const std::string &p : parts) total += p.size();
    h->rows_text.reserve(total);
    for (size_t r = 0; r < T; ++r) {
        h->rows_text += parts[r];
        for (const auto &kv : Ns[r]) incN(h, kv.first, kv.second);
    }
    *text = h->rows_text.c_str();
    *len = h->rows_text.size();
    return FC2_OK;
}

// fc2_caller_rows written straight to a file descriptor: the dict order cut into ranges the workers
// format while a writer thread writes each finished range in order and frees it -- no joined copy of
// the table (over 1 GB when every read has a junction of its own), no copy into Python
extern "C" int fc2_caller_write_rows(fc2_caller *h, int kind, int fd, uint64_t *len) {
    if (!h || kind < 0 || kind > 1 || fd < 0) return fc2::fail(FC2_E_PARAM, "fc2_caller_write_rows: bad arguments");
    release_read_side(h);
    const size_t nj = h->order[kind].size();
    const size_t W = h->pool ? (size_t)h->pool->size() : 1;
    const size_t R = std::max<size_t>(1, std::min<size_t>(4 * W, nj / 4096));
    std::vector<std::string> parts(R);
    std::vector<std::vector<std::pair<const char *, double>>> Ns(R);
    std::vector<char> ready(R, 0);
    std::mutex mu;
    std::condition_variable cv;
    bool abandon = false;
    int werr = 0;
    uint64_t written = 0;
    auto writer = [&]() {
        for (size_t r = 0; r < R; ++r) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return ready[r] || abandon; });
                if (!ready[r]) return;
            }
            const char *p = parts[r].data();
            size_t left = parts[r].size();
            while (left && !werr) {
                const ssize_t w = ::write(fd, p, left);
                if (w < 0) {
                    if (errno == EINTR) continue;
                    werr = errno;
                    break;
                }
                p += w, left -= (size_t)w, written += (uint64_t)w;
            }
            std::string().swap(parts[r]);
        }
    };
    auto range = [&](int r) {
        storage_rows(h, kind, nj * (size_t)r / R, nj * (size_t)(r + 1) / R, parts[(size_t)r], Ns[(size_t)r]);
        std::lock_guard<std::mutex> g(mu);
        ready[(size_t)r] = 1;
        cv.notify_all();
    };
    std::thread wt;
    try {
        wt = std::thread(writer);
    } catch (const std::system_error &) {          // no thread: format all, then write here
    }
    try {
        if (R > 1 && h->pool) h->pool->run_checked((int)R, range);
        else for (size_t r = 0; r < R; ++r) range((int)r);
    } catch (const std::bad_alloc &) {
        {
            std::lock_guard<std::mutex> g(mu);
            abandon = true;
            cv.notify_all();
        }
        if (wt.joinable()) wt.join();
        return fc2::fail(FC2_E_PARAM, "fc2_caller_write_rows: out of memory");
    }
    if (wt.joinable()) wt.join();
    else writer();
    for (size_t r = 0; r < R; ++r)
        for (const auto &kv : Ns[r]) incN(h, kv.first, kv.second);
    if (len) *len = written;
    if (werr) return fc2::fail(FC2_E_IO, std::string("IOError: [Errno ") + std::to_string(werr) + "] " + strerror(werr));
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
        ingest_counts(h, &c);
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
    if (n_reads) *n_reads = h->st_reads.load(std::memory_order_relaxed);
    if (n_pairs) *n_pairs = h->st_pairs.load(std::memory_order_relaxed);
    return FC2_OK;
}
