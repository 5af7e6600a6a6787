// Internal interface of the native ingest (fc2_ingest.cpp) for the native caller
// (fc2_caller.cpp): parsed records, mates, and a pull loop that hands fragments
// carrying anchor pairs to a sink instead of formatting them as SAM text.
#pragma once
#include <stdint.h>

#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "../../include/fc2_ingest.h"

namespace fc2 {
namespace ing {

// A tag value as pysam's get_tag returns it and Python 2 computes with it (find_circ.py:809-819,
// :556-566): an int for the integer types c C s S i I, a float for 'f' (the stored float32, widened
// to a double as pysam does; SAM text is rounded to float32 as htslib stores it), a str for A Z H,
// an array for B.  Only numbers take part in arithmetic; the caller raises Python's TypeError where
// the reference would subtract a non-number.
struct PyNum {
    enum Kind : uint8_t { INT = 0, FLOAT = 1, STR = 2, ARRAY = 3 };
    union {
        int64_t i;
        double f;
    };
    Kind k;
    PyNum() : i(0), k(INT) {}
    static PyNum of_int(int64_t v) { PyNum n; n.i = v; return n; }
    static PyNum of_float(double v) { PyNum n; n.f = v; n.k = FLOAT; return n; }
    static PyNum other(Kind kind) { PyNum n; n.k = kind; return n; }
    bool number() const { return k == INT || k == FLOAT; }
    double value() const { return k == FLOAT ? f : (double)i; }   // exact for |int| < 2^53 (tag ints are 32-bit)
};

// the plain fields of a record (swapped as one block, see swap(Rec &, Rec &))
struct RecFields {
    uint32_t flag = 0;
    int32_t tid = -1;
    int64_t pos = -1;
    int64_t aend = -1;     // -1: None (unmapped / no cigar)
    int32_t astart = 0;    // aligned_start_from_cigar (:1086-1097)
    int32_t qlen = -1;     // len(query); -1: query is None (SEQ '*')
    bool has_seq = false;  // SEQ / QUAL "*" -> false
    bool has_qual = false;
    // AS / XS tags as pysam's get_tag returns them (the first occurrence): present?, value
    bool has_as = false, has_xs = false;
    PyNum as, xs;
    // the LAST occurrence of each, as dict(read.tags) gives it (Hit.add, find_circ.py:556-557)
    PyNum as_last, xs_last;
};

// SEQ / QUAL a parse thread left where they are in the record's parse block (which stays until
// its batch is reused): most records never need them, only the primaries of handed fragments do
struct LazySeq {
    const char *seq = nullptr, *qual = nullptr;
    int32_t n_seq = -1;        // -1: Rec::seq / qual hold the decoded strings
    int32_t n_qual = 0;        // SAM text: QUAL's length (BAM: n_seq bytes, 0xFF for none)
    bool bam = false;          // 4-bit BAM bases and binary qualities; else SAM text
};

struct Rec : RecFields {
    std::string text;      // SAM line (no newline): for the Python hand-back and the -B writer
    std::string raw;       // BAM input with a -B writer: block_size + record bytes
    std::string qname;
    std::string seq, qual;  // SEQ / QUAL (see decode())
    uint32_t seq_n = 0;    // seq.size() once decoded ("*" counts 1, as the string does)
    LazySeq lz;
    bool unmapped() const { return flag & 0x4; }
    bool read1() const { return flag & 0x40; }
    bool reverse() const { return flag & 0x10; }
    // seq / qual from the parse block if a parse thread left them there; a record decodes before
    // it leaves its batch (RecList::take) or is read (the native caller's take_align)
    void decode() {
        if (lz.n_seq >= 0) decode_lazy();
    }
    void decode_lazy();
};

// member-wise: the strings swap their buffers, the plain fields swap as one block (cheaper than
// std::swap's three moves of every member)
inline void swap(Rec &a, Rec &b) noexcept {
    std::swap(static_cast<RecFields &>(a), static_cast<RecFields &>(b));
    a.text.swap(b.text);
    a.raw.swap(b.raw);
    a.qname.swap(b.qname);
    a.seq.swap(b.seq);
    a.qual.swap(b.qual);
    std::swap(a.seq_n, b.seq_n);
    std::swap(a.lz, b.lz);
}

// A mate's records.  Slots past size() stay constructed: take() swaps a parsed record into the next
// slot and hands the slot's previous contents (strings with their capacity) back to the caller, so
// a record is moved once on its way from the parser into a mate, and nothing is freed.
class RecList {
  public:
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    Rec &operator[](size_t k) { return v_[k]; }
    const Rec &operator[](size_t k) const { return v_[k]; }
    Rec *begin() { return v_.data(); }
    Rec *end() { return v_.data() + n_; }
    const Rec *begin() const { return v_.data(); }
    const Rec *end() const { return v_.data() + n_; }
    void clear() { n_ = 0; }
    void take(Rec &r) {
        if (n_ == v_.size()) v_.emplace_back();
        r.decode();                     // (its parse block may be reused while the mate is open)
        swap(v_[n_++], r);
    }
  private:
    std::vector<Rec> v_;
    size_t n_ = 0;
};

struct Mate {
    RecList recs;                // primary first, then every added segment (for hand-back)
    std::vector<int> proper;     // indices into recs
    bool valid = false;
};

// A mate as the sink sees it: its records, the primary first, and the indices of its proper
// segments among them.  The records sit in the ingest's Mate or -- for a fragment a parse thread
// grouped on its own (group_batch in fc2_ingest.cpp) -- in place in their parse batch, where `idx`
// lists their positions.
struct MateRef {
    Rec *base = nullptr;
    const int32_t *idx = nullptr;      // null: the records are base[0, n)
    uint32_t n = 0;
    const int32_t *proper = nullptr;   // indices into this mate's records
    uint32_t np = 0;
    uint32_t seq_len = 0;              // len(SEQ) of the primary (rec(0).seq.size())
    // the records (and idx, proper) stay where they are until release(): the sink may keep the
    // reference instead of copying what it needs (set_pin; fragments grouped on a parse thread)
    bool stable = false;
    Rec &rec(size_t k) const { return base[idx ? idx[k] : k]; }
};

// A handed fragment a parse thread grouped on its own (group_batch): its mates' records by position
// in the batch (gidx), the run.log counts and fragments closed up to it in the batch's region, and
// the cumulative span / read-part room its spans need (for the caller's chunk offsets)
struct GFrag {
    int32_t r0[2], n[2], p0[2], np[2];  // mate 0 = the other mate (n[0] == 0: none), 1 = current
    uint32_t seq_len[2];                // len(SEQ) of each mate's primary
    bool must;
    fc2_ingest_counts cum;              // counts of the region through this fragment
    uint64_t frags;                     // fragments closed in the region through this one
    uint64_t span_cum, arena_cum;       // sum over the batch's handed fragments through this one of
                                        // (np - 1) and (np - 1) * seq_len per mate with np >= 2
};

// Consecutive handed fragments of one batch, stable until release() (set_pin): the bulk sink
// records them without touching each fragment (the caller's workers read them later)
struct RegionRef {
    Rec *recs;
    const GFrag *g;                     // g[0, n)
    size_t n;
    const int32_t *gidx;
    uint64_t span_before, arena_before; // span_cum / arena_cum of the batch's handed fragment before g[0]
};
using BulkSink = std::function<int(const RegionRef &)>;

// Fragments that carry anchor pairs (or that the reference would fail on: must_see) are passed
// to the sink in input order; m1 = the other mate (may be null), m2 = the current mate.
// The sink may take the mates' strings (swap them out): the loop reads nothing of a fragment's
// records after handing it over.
using FragSink = std::function<int(MateRef *m1, MateRef *m2, bool must_see)>;

// The loop of fc2_ingest_next with a sink instead of SAM text; a non-zero return of the sink
// stops the loop and is returned.  With `bulk` and pinning on, the fragments a parse thread grouped
// go to `bulk` a run at a time, in input order with the sink's.
int pull(fc2_ingest *h, const fc2_ingest_params *p, uint64_t max_frags, const FragSink &sink, int *eof,
         const BulkSink *bulk = nullptr);

// true when the ingest writes records while reading (-B, fc2_ingest_set_bam_out): the reference
// stops writing at a failing fragment, so the caller must process each fragment as it comes
bool writes_records(const fc2_ingest *h);

// pinning: with `on`, parse batches whose fragments were handed over stay untouched (their records
// are not reused) until release(); the sink then gets stable MateRefs for them
void set_pin(fc2_ingest *h, bool on);
void release(fc2_ingest *h);
// as many batches pinned as allowed (FC2_PIN_MAX, default 64): pull returns, the chunk ends there
bool pin_full(const fc2_ingest *h);

// the consumer's time spent waiting for parse-ahead batches since the last call, and the handed
// fragments grouped on the parse threads meanwhile (FC2_CALLER_TIMING)
double take_wait_ms(fc2_ingest *h, uint64_t *grouped = nullptr);

// the stages upstream of the consumer since the last call (FC2_CALLER_TIMING): the reader's wait for
// inflated BGZF batches, the splitter's wait for a free block slot, the parse threads' idle time
void take_stage_ms(fc2_ingest *h, double *inflate_wait, double *split_block, double *parse_idle);

}  // namespace ing
}  // namespace fc2
