// fc2_ingest.cpp -- native SAM/BAM ingest: parse, group into fragments, form
// anchor pairs; hand back only the fragments that carry pairs (include/fc2_ingest.h).
//
// Grouping follows collected_bwa_mem_segments (find_circ.py:1450-1486): the
// first record always opens a mate; later unmapped records are counted and
// skipped; a record continues the current mate if it has the same qname and
// read1 flag, opens the other mate if the read1 flag differs, and otherwise
// closes the fragment.  Pairing follows MateSegments.add_segment /
// adjacent_segment_pairs / process_mate (:1039-1140, 1492-1527).
#include <ctype.h>
#include <emmintrin.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <chrono>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/fc2_ingest.h"
#include "fc2_bamout.h"
#include "fc2_common.h"
#include "fc2_cpuacct.h"
#include "fc2_deflate.h"
#include "fc2_inflate.h"
#include "fc2_ingest_impl.h"

using fc2::ing::Mate;
using fc2::ing::MateRef;
using fc2::ing::Rec;

namespace {

// CIGAR helpers ------------------------------------------------------------
struct CigarInfo {
    int64_t ref_span = 0;
    int32_t astart = 0, lead_s = 0, trail_s = 0;
    bool any = false;
};

CigarInfo cigar_info(const std::vector<std::pair<int, int>> &ops) {
    CigarInfo c;
    c.any = !ops.empty();
    bool stop = false;
    for (auto &o : ops) {
        if (o.first == 0 || o.first == 2 || o.first == 3 || o.first == 7 || o.first == 8) c.ref_span += o.second;
        if (!stop) {
            if (o.first == 4 || o.first == 5) c.astart += o.second;
            else if (o.first == 0) stop = true;
        }
    }
    for (auto &o : ops) {              // leading soft clips (hard clips skipped)
        if (o.first == 4) c.lead_s += o.second;
        else if (o.first != 5) break;
    }
    for (auto it = ops.rbegin(); it != ops.rend(); ++it) {
        if (it->first == 4) c.trail_s += it->second;
        else if (it->first != 5) break;
    }
    return c;
}

int cig_code(char c) {
    switch (c) {
        case 'M': return 0; case 'I': return 1; case 'D': return 2; case 'N': return 3; case 'S': return 4;
        case 'H': return 5; case 'P': return 6; case '=': return 7; case 'X': return 8; default: return -1;
    }
}

void finish_rec(Rec &r, const std::vector<std::pair<int, int>> &ops, int64_t seqlen) {
    CigarInfo c = cigar_info(ops);
    r.astart = c.astart;
    r.aend = (r.unmapped() || !c.any) ? -1 : r.pos + c.ref_span;
    // len(seq[lead_s : len(seq) - trail_s]) with Python slice semantics (pysam's query when the
    // clips exceed SEQ: an empty string, or a negative end counted from the back)
    if (r.has_seq) {
        const int64_t n = seqlen;
        int64_t b = c.lead_s, e = n - c.trail_s;
        if (e < 0) e += n;
        b = b > n ? n : b;
        e = e < 0 ? 0 : (e > n ? n : e);
        r.qlen = (int32_t)(e > b ? e - b : 0);
    } else {
        r.qlen = -1;
    }
}

}  // namespace

void fc2::ing::Rec::decode_lazy() {
    const int32_t n = lz.n_seq;
    if (lz.bam) {
        // two bases per byte through a 256-entry table of base pairs
        static const struct Pairs {
            char t[256][2];
            Pairs() {
                static const char *SEQ = "=ACMGRSVTWYHKDBN";
                for (int v = 0; v < 256; ++v) { t[v][0] = SEQ[v >> 4]; t[v][1] = SEQ[v & 0xF]; }
            }
        } kPairs;
        const uint8_t *p = (const uint8_t *)lz.seq, *q = (const uint8_t *)lz.qual;
        if (n == 0) {
            seq.assign(1, '*');
        } else {
            seq.resize((size_t)n);
            for (int k = 0; k + 1 < n; k += 2) memcpy(&seq[k], kPairs.t[p[k >> 1]], 2);
            if (n & 1) seq[n - 1] = kPairs.t[p[(n - 1) >> 1]][0];
        }
        if (n == 0 || q[0] == 0xFF) qual.assign(1, '*');
        else { qual.resize((size_t)n); for (int k = 0; k < n; ++k) qual[k] = (char)(q[k] + 33); }
    } else {
        seq.assign(lz.seq, (size_t)n);
        qual.assign(lz.qual, (size_t)lz.n_qual);
    }
    lz.n_seq = -1;
}

namespace {

// ---- parallel BGZF ----------------------------------------------------------------------
// BAM is a series of BGZF blocks (gzip members of <= 64 KiB with the compressed size in a
// "BC" extra field), so the blocks can be inflated independently.  A batch of blocks is
// read sequentially and inflated by a few threads while the previous batch is parsed.
bool read_full(int fd, uint8_t *dst, size_t n, size_t &got) {
    got = 0;
    while (got < n) {
        ssize_t k;
        do { k = read(fd, dst + got, n - got); } while (k < 0 && errno == EINTR);
        if (k < 0) return false;
        if (k == 0) break;
        got += (size_t)k;
    }
    return true;
}

// BGZF block size from an 18+-byte header, 0 if the header is not BGZF
size_t bgzf_block_size(const uint8_t *h, size_t avail) {
    if (avail < 18 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return 0;
    const size_t xlen = h[10] | (h[11] << 8);
    if (avail < 12 + xlen) return 0;
    for (size_t p = 12; p + 4 <= 12 + xlen;) {
        const size_t slen = h[p + 2] | (h[p + 3] << 8);
        if (h[p] == 'B' && h[p + 1] == 'C' && slen == 2 && p + 6 <= 12 + xlen) return (size_t)(h[p + 4] | (h[p + 5] << 8)) + 1;
        p += 4 + slen;
    }
    return 0;
}

// a byte vector whose growth leaves the new bytes uninitialised (inflate overwrites them)
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U> &) noexcept {}
    // a GPU-inflated batch's buffer comes from the pinned pool (fc2_inflate.h), so the inflated bytes
    // are downloaded straight into it; every other buffer, and any when the pool has none, from the heap
    static constexpr size_t kPinnedMin = size_t(8) << 20;
    T *allocate(size_t n) {
        if (n * sizeof(T) >= kPinnedMin)
            if (void *p = fc2::inf::pinned_take(n * sizeof(T))) return static_cast<T *>(p);
        return std::allocator<T>::allocate(n);
    }
    void deallocate(T *p, size_t n) {
        if (n * sizeof(T) >= kPinnedMin && fc2::inf::pinned_give(p)) return;
        std::allocator<T>::deallocate(p, n);
    }
    template <class U>
    void construct(U *p) noexcept {
        ::new (static_cast<void *>(p)) U;
    }
    template <class U, class... Args>
    void construct(U *p, Args &&...args) {
        ::new (static_cast<void *>(p)) U(std::forward<Args>(args)...);
    }
};
using CharBuf = std::vector<char, NoInitAlloc<char>>;

// kHead bytes of headroom in front of a batch's inflated bytes: the parse-ahead splitter moves the
// record cut by the previous batch's end there instead of copying the batch (bgzf_split_loop)
constexpr size_t kHead = size_t(1) << 16;

constexpr uint64_t kNoExit = ~uint64_t(0);

// The BAM records of one inflated batch as the inflating threads saw them (bgzf_split_loop jumps
// through these instead of reading every record's block_size from cold memory on its one thread):
// per BGZF block, the record starts a walk visits inside the block when it begins at the block's
// first plausible record (batch offsets, ascending), and where that walk leaves the block (kNoExit:
// it met a block_size below 32 or could not read one).  A start is only a guess until the split
// loop's own chain of records -- the reference's order of block sizes -- reaches it.
struct RecLists {
    size_t n = 0;                               // the batch's inflated bytes
    std::vector<size_t> ooff;                   // block k's bytes: [ooff[k], ooff[k + 1])
    std::vector<std::vector<uint32_t>> starts;
    std::vector<uint64_t> exit;
};

struct BgzfBatch {
    CharBuf out;                 // kHead bytes of headroom, then the inflated bytes
    size_t n = 0;                // inflated bytes
    bool eof = false;
    std::string err;
    std::shared_ptr<RecLists> recs;             // null: none (a batch of 4 GiB or more)
    const char *data() const { return out.data() + kHead; }
};

// a plausible BAM record at p (`avail` bytes readable from p): the fixed fields and read name as the
// SAM/BAM specification constrains them (a guess; see RecLists)
bool bam_plausible(const uint8_t *p, size_t avail) {
    if (avail < 36) return false;
    int32_t bs, ref, pos, lseq, nref, npos;
    uint16_t ncig;
    memcpy(&bs, p, 4), memcpy(&ref, p + 4, 4), memcpy(&pos, p + 8, 4), memcpy(&ncig, p + 16, 2);
    memcpy(&lseq, p + 20, 4), memcpy(&nref, p + 24, 4), memcpy(&npos, p + 28, 4);
    const uint32_t lname = p[12];
    if (bs < 32 || bs >= (1 << 28) || ref < -1 || pos < -1 || lname < 1 || lseq < 0 || nref < -1 || npos < -1)
        return false;
    if (32u + lname + 4ull * ncig + ((uint64_t)lseq + 1) / 2 + (uint64_t)lseq > (uint64_t)bs) return false;
    if (36 + (size_t)lname > avail) return true;
    if (p[36 + lname - 1] != 0) return false;
    for (uint32_t k = 0; k + 1 < lname; ++k)
        if (p[36 + k] < 0x21 || p[36 + k] > 0x7e) return false;
    return true;
}

// RecLists for the block [b0, b1) of data, reading nothing outside it (its neighbours may still be
// being inflated): the first offset where a plausible record is followed by another plausible one
// (or by the block's end), then block_size to block_size
void walk_block(const char *data, size_t b0, size_t b1, std::vector<uint32_t> &starts, uint64_t &exit) {
    starts.clear();
    exit = kNoExit;
    const uint8_t *d = (const uint8_t *)data;
    size_t o = b0;
    for (; o + 36 <= b1; ++o) {
        if (!bam_plausible(d + o, b1 - o)) continue;
        int32_t bs;
        memcpy(&bs, d + o, 4);
        const size_t nx = o + 4 + (size_t)bs;
        if (nx + 36 <= b1 && !bam_plausible(d + nx, b1 - nx)) continue;
        break;
    }
    if (o + 36 > b1) return;                    // inside one record, or too short to tell
    while (o + 4 <= b1) {
        int32_t bs;
        memcpy(&bs, d + o, 4);
        if (bs < 32) return;
        starts.push_back((uint32_t)o);
        o += 4 + (size_t)bs;
    }
    exit = o;
}

int bgzf_threads() {
    const char *e = getenv("FC2_INGEST_THREADS");
    int n = e ? atoi(e) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(n, 8));
}

// BGZF blocks inflated on a GPU (fc2_ingest_set_gpu_inflate; fc2_inflate.hip): the device's stream
// and buffers, made by the first batch that uses them (on the batch reader's thread, one batch at a
// time); a block the GPU refused or whose CRC-32 does not match is inflated on the CPU as before
struct GpuInflate {
    int device = -1;
    uint32_t max_blocks = 0;
    fc2::inf::Gpu *g = nullptr;
    std::future<std::pair<fc2::inf::Gpu *, std::string>> opening;   // gpu_open, started by the set call
    bool failed = false;                       // the device could not be had or failed: CPU from then on
    std::string err;
    std::atomic<uint64_t> gpu_blocks{0}, cpu_blocks{0};
    // FC2_CALLER_TIMING: the batch reader's time reading, submitting chunks, waiting for the device,
    // inflating refused blocks; batches whose buffer was pinned (downloaded into directly)
    int64_t read_ns = 0, add_ns = 0, wait_ns = 0, cpu_ns = 0;
    int batches = 0, pinned = 0;
    // fc2_ingest_set_gpu_inflate_from: nothing is made on the device until start_after bytes of the
    // input were read (inputs smaller than that never touch it); `blocks` is then the batch size the
    // next batches take (0: the ingest's own).  launched / read_bytes: the batch reader's alone (one
    // batch at a time)
    uint64_t start_after = 0, read_bytes = 0;
    bool launched = true;
    std::atomic<int> blocks{0};
    void launch(bool wait) {
        const int dev = device;
        const uint32_t mb = max_blocks;
        opening = std::async(wait ? std::launch::deferred : std::launch::async, [dev, mb]() {
            std::string e;
            fc2::inf::Gpu *g = fc2::inf::gpu_open(dev, mb, kHead + (size_t)mb * 65536, e);
            return std::make_pair(g, e);
        });
        launched = true;
        blocks = (int)max_blocks;
    }
    ~GpuInflate() {
        if (getenv("FC2_CALLER_TIMING") && batches)
            fprintf(stderr, "gpu inflate: %d batches (%d pinned), %llu blocks on the GPU, %llu on the CPU; reader s: "
                    "read %.3f submit %.3f wait %.3f cpu %.3f\n", batches, pinned, (unsigned long long)gpu_blocks.load(),
                    (unsigned long long)cpu_blocks.load(), (read_ns - add_ns) * 1e-9, add_ns * 1e-9, wait_ns * 1e-9,
                    cpu_ns * 1e-9);
        if (opening.valid()) g = opening.get().first;
        fc2::inf::gpu_close(g);
    }
};

static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

constexpr size_t kGpuChunk = 256;              // blocks per GPU chunk (16 MiB inflated)

// reads up to `max_blocks` blocks (the first `pre` bytes of the first header are in `pre`)
BgzfBatch bgzf_batch(int fd, std::vector<uint8_t> pre, int max_blocks, int n_threads, std::shared_ptr<GpuInflate> gi) {
    BgzfBatch B;
    std::vector<uint8_t> raw;
    std::vector<size_t> boff, bsz;
    raw.swap(pre);
    if (gi && !gi->launched && gi->read_bytes >= gi->start_after) gi->launch(false);
    // the GPU inflates the batch in chunks as they are read (fc2_inflate.h), into the batch buffer
    // itself -- a pinned one from the pool, made max_blocks * 64 KiB long up front
    bool gpu = gi && !gi->failed && max_blocks <= (int)gi->max_blocks;
    // the device's buffers and the pinned pool, made meanwhile: until they are ready (pinning the
    // buffers takes a few hundred ms) the batches are inflated on the CPU
    if (gpu && !gi->g && gi->opening.valid() &&
        gi->opening.wait_for(std::chrono::seconds(0)) == std::future_status::ready) {
        auto r = gi->opening.get();
        gi->g = r.first;
        if (!gi->g) gi->failed = true, gi->err = r.second;
    }
    gpu = gpu && gi->g;
    size_t submitted = 0;
    auto submit = [&](bool last) {             // blocks read so far, in chunks of kGpuChunk
        if (!gpu) return;
        if (boff.size() - submitted < kGpuChunk && !(last && boff.size() > submitted)) return;
        fc2::cpu::Scope acct(fc2::cpu::INFLATE);
        const int64_t a0 = now_ns();
        fc2::inf::gpu_add(gi->g, raw.data(), boff.data(), bsz.data(), submitted, boff.size());
        gi->add_ns += now_ns() - a0;
        submitted = boff.size();
    };
    const int64_t t0 = now_ns();
    if (gpu) {
        B.out.resize(kHead + (size_t)max_blocks * 65536);
        fc2::inf::gpu_begin(gi->g, B.out.data() + kHead);
        gi->batches += 1;
        gi->pinned += fc2::inf::pinned_owns(B.out.data());
    }
    size_t pos = 0;
    while ((int)boff.size() < max_blocks) {
        size_t got;
        if (raw.size() - pos < 18) {           // header
            const size_t have = raw.size() - pos;
            raw.resize(pos + 18);
            if (!read_full(fd, raw.data() + pos + have, 18 - have, got)) { B.err = "read error"; break; }
            if (have + got == 0) { raw.resize(pos); B.eof = true; break; }
            if (have + got < 18) { B.err = "truncated BGZF block header"; break; }
        }
        const size_t xlen = raw[pos + 10] | (raw[pos + 11] << 8);
        if (raw.size() - pos < 12 + xlen) {
            const size_t have = raw.size() - pos;
            raw.resize(pos + 12 + xlen);
            if (!read_full(fd, raw.data() + pos + have, 12 + xlen - have, got) || got < 12 + xlen - have) {
                B.err = "truncated BGZF block header";
                break;
            }
        }
        const size_t bs = bgzf_block_size(raw.data() + pos, raw.size() - pos);
        if (bs < 12 + xlen + 8) { B.err = "not a BGZF block"; break; }
        const size_t have = raw.size() - pos;
        raw.resize(pos + bs);
        if (!read_full(fd, raw.data() + pos + have, bs - have, got) || got < bs - have) {
            B.err = "truncated BGZF block";
            break;
        }
        boff.push_back(pos);
        bsz.push_back(bs);
        pos += bs;
        submit(false);
    }
    bool on_gpu = false;
    int64_t t2 = 0;
    if (gpu) {                                 // (after an error too: the device must be done with B.out)
        submit(true);
        const int64_t t1 = now_ns();
        gi->read_ns += t1 - t0;
        fc2::cpu::Scope acct(fc2::cpu::INFLATE);
        on_gpu = fc2::inf::gpu_finish(gi->g, gi->err);
        if (!on_gpu) gi->failed = true;        // (the CPU inflates every block of this batch and the next)
        t2 = now_ns();
        gi->wait_ns += t2 - t1;
    }
    if (gi) gi->read_bytes += pos;
    if (!B.err.empty()) return B;
    const size_t nb = boff.size();
    std::vector<size_t> ooff(nb + 1, 0);
    for (size_t i = 0; i < nb; ++i) {
        const uint8_t *t = raw.data() + boff[i] + bsz[i] - 4;
        ooff[i + 1] = ooff[i] + (size_t)(t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24));
    }
    B.n = ooff[nb];
    B.out.resize(kHead + B.n);
    // the blocks the CPU inflates: all of them, or those the GPU refused
    std::vector<uint8_t> on_cpu(nb, on_gpu ? 0 : 1);
    size_t n_cpu = on_gpu ? 0 : nb;
    if (on_gpu)
        for (size_t i = 0; i < nb; ++i)
            if (fc2::inf::gpu_status(gi->g, i) != 0) on_cpu[i] = 1, ++n_cpu;
    // every block's records listed by the thread that inflated it, while they are in its cache
    RecLists *R = nullptr;
    if (B.n < (uint64_t(1) << 32) && nb) {
        B.recs = std::make_shared<RecLists>();
        R = B.recs.get();
        R->n = B.n;
        R->ooff = ooff;
        R->starts.resize(nb);
        R->exit.assign(nb, kNoExit);
    }
    std::atomic<size_t> next{0};
    std::atomic<bool> bad{false};
    auto work = [&]() {
        fc2::cpu::Scope acct(fc2::cpu::INFLATE);
        fc2::dfl::Inflater inf;                 // libdeflate (zlib without it): fc2_deflate.h
        if (!inf.ok()) { bad = true; return; }
        for (size_t i; (i = next.fetch_add(1)) < nb && !bad;) {
            char *dst = B.out.data() + kHead + ooff[i];
            const size_t n = ooff[i + 1] - ooff[i];
            if (on_cpu[i]) {
                const uint8_t *blk = raw.data() + boff[i];
                const size_t xl = blk[10] | (blk[11] << 8);
                const uint8_t *t = blk + bsz[i] - 8;
                const uint32_t crc = t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24);
                if (!inf.exact(blk + 12 + xl, bsz[i] - 12 - xl - 8, dst, n) || fc2::dfl::crc32(dst, n) != crc) {
                    bad = true;
                    break;
                }
            }
            if (R) walk_block(B.out.data() + kHead, ooff[i], ooff[i + 1], R->starts[i], R->exit[i]);
        }
    };
    const int nt = (int)std::min<size_t>((size_t)n_threads, R ? nb : n_cpu);
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    if (nt > 0) work();
    for (auto &t : pool) t.join();
    if (bad) B.err = "corrupt BGZF block";
    if (gpu) {                                 // (the batches the GPU took: its blocks, and those it refused)
        gi->gpu_blocks += nb - n_cpu;
        gi->cpu_blocks += n_cpu;
        gi->cpu_ns += now_ns() - t2;
    }
    return B;
}

}  // namespace

struct fc2_ingest {
    int fd = -1;
    // what the bytes are, detected from the bytes themselves (never from the file name), as
    // htslib's hts_detect_format does for pysam.Samfile(path_or_'-', 'r'|'rb') (find_circ.py:461-469):
    // the byte source (plain, BGZF blocks, or any other gzip stream) and, below it, BAM or SAM text
    enum Src { SRC_RAW, SRC_BGZF, SRC_GZIP } src = SRC_RAW;
    bool bam = false;
    bool eof_in = false;
    // an input error met by the sequential reader (read(2) failure, corrupt gzip stream); reported
    // after the records before it, where the input ends
    int in_rc = 0;
    std::string in_err;
    // raw input buffer (SAM text or inflated BAM)
    std::vector<char> buf;
    size_t beg = 0, end = 0;
    // zlib
    z_stream zs{};
    bool z_init = false;
    std::vector<char> zin;
    bool z_done = false;
    bool z_mid = false;          // inside a gzip member (its end not yet seen)
    // BGZF (the BAM case): batches inflated in parallel, one batch ahead of the parser
    bool bgzf = false;
    int bgzf_nt = 1;
    int bgzf_blocks = 256;       // BGZF blocks per inflated batch (FC2_BGZF_BATCH: small in the tests)
    std::future<BgzfBatch> bgzf_next;
    std::shared_ptr<GpuInflate> gpu_inflate;     // fc2_ingest_set_gpu_inflate (null: the CPU inflates)
    std::atomic<int64_t> inflate_wait_ns{0};     // the reader's wait for inflated BGZF batches (timing)
    std::string z_err;
    // header
    std::string header;
    std::vector<std::string> refs;
    std::vector<int64_t> ref_len;
    std::unordered_map<std::string, int> tid_of;
    // -B/--bam: anchor alignments of every processed mate (find_circ.py:1134-1140)
    fc2::bam::Writer *bam_out = nullptr;
    bool bam_stopped = false;    // the reference raised inside process_mate: nothing after it is written
    std::string bam_err;
    // grouping state
    bool started = false;
    Mate current, other;
    bool have_other = false;
    uint64_t n_records = 0;
    std::string out;
    fc2_ingest_counts counts{};
    bool finished = false;
    bool need_text = true;       // false once a native caller pulls structured fragments
    bool pin = false;            // fc2::ing::set_pin (applies to the parse-ahead batches)
    // fc2_ingest_next: an error met after some fragments were formed is returned by the next call,
    // after those fragments (the reference records each fragment before it reads the next)
    int deferred_rc = FC2_OK;
    std::string deferred_msg;
    // parse scratch, reused across records (no per-record allocation in steady state)
    struct ParseScratch {
        std::vector<std::pair<int, int>> ops;
        std::string last_rn;     // RNAME -> tid cache (consecutive records share a chromosome)
        int last_tid = -1;
    } ps;
    std::vector<std::pair<int, int>> ops;
    Rec scratch;                 // the record being parsed (sequential path); mates swap theirs back
    // SAM records parsed ahead on threads of their own (native caller pulls, no -B writer): a
    // splitter thread owns the input from then on and cuts it into newline-aligned blocks, parser
    // threads turn blocks into record batches, the consumer takes the batches in input order
    struct SamAhead;
    std::unique_ptr<SamAhead> ahead;
    ~fc2_ingest();
};

// BGZF blocks the next batch takes: the GPU inflate's size once it started, else the ingest's
int batch_blocks(const fc2_ingest *h) {
    const GpuInflate *gi = h->gpu_inflate.get();
    const int b = gi ? gi->blocks.load() : 0;
    return b > 0 ? b : h->bgzf_blocks;
}

// The parse-ahead threads.  The splitter reads the input into blocks cut after the last newline
// (4 MiB each, numbered), parser threads turn each block into a batch of records, and the consumer
// (next_record) takes the batches in block order.  Records travel back with their buffers (the
// consumer swaps in a recycled record), so steady state allocates nothing.  A read or parse error
// ends the stream at that record, where the consumer reports it.
struct fc2_ingest::SamAhead {
    struct Batch {
        uint64_t seq = 0;
        std::string block;                      // the block's bytes (whole lines)
        // or, BGZF input (bgzf_split_loop): whole records in place in an inflated batch
        std::shared_ptr<const CharBuf> vbuf;
        size_t voff = 0, vlen = 0;
        std::vector<Rec> recs;
        size_t n = 0;
        int rc = FC2_OK;
        std::string err;
        int read_rc = FC2_OK;                   // read(2) failed after the block's lines: reported
        std::string read_err;                   // once they are parsed (records before an error first)
        bool eof = false;                       // the last block of the input
        // fragments the parse thread grouped on its own (group_batch): records [gs, gt) form whole
        // fragments (gs == gt: none); the handed ones are listed with the counts up to them
        using GFrag = fc2::ing::GFrag;
        uint32_t gs = 0, gt = 0;
        std::vector<GFrag> gfrags;
        std::vector<int32_t> gidx;              // record positions and proper indices of gfrags' mates
        fc2_ingest_counts gtotal{};             // counts of the whole region (records [gs, gt))
        uint64_t gtotal_frags = 0;
    };
    static constexpr size_t kBlock = size_t(4) << 20;
    size_t block = kBlock;                      // FC2_PARSE_BLOCK (bytes): small blocks in the tests
    static constexpr int kParsers = 3;          // default parser threads (FC2_PARSE_THREADS)
    static constexpr size_t kInflight = 24;     // blocks read but not yet consumed (FC2_PARSE_INFLIGHT)
    size_t max_inflight = kInflight;
    std::mutex m;
    std::condition_variable cv;
    std::deque<std::unique_ptr<Batch>> todo;    // read, not yet parsed (block order)
    std::map<uint64_t, std::unique_ptr<Batch>> done;   // parsed, by block number
    std::vector<std::unique_ptr<Batch>> spare;
    size_t inflight = 0;
    uint64_t next_consume = 0;
    double wait_ms = 0;                         // the consumer's time waiting for parsed batches
    // FC2_CALLER_TIMING: the splitter blocked on the consumer (all blocks in flight), the parsers
    // idle (no block to parse), summed over parser threads
    std::atomic<int64_t> split_block_ns{0}, parse_idle_ns{0};
    uint64_t split_steps = 0, split_jumps = 0;  // bgzf_split_loop: records read one at a time, list jumps
    std::unique_ptr<Batch> cur;                 // the consumer's batch
    size_t pos = 0;
    // grouping on the parse threads (pull only: the sink path); the consumer's place in a batch's
    // region: past its first record's close (in_region), the next handed fragment, counts applied
    fc2_ingest_params gp{};
    bool group = false;
    bool in_region = false;
    size_t gnext = 0;
    fc2_ingest_counts gapplied{};
    uint64_t gapplied_frags = 0;
    uint64_t grouped = 0;                       // handed fragments grouped on the parse threads
    bool pin = false;                           // set_pin: consumed batches wait in `pinned` for release()
    std::vector<std::unique_ptr<Batch>> pinned;
    size_t max_pinned = 64;                     // pull stops there (FC2_PIN_MAX): few handed fragments
                                                // must not pin the whole input
    bool stop = false;
    std::thread splitter;
    std::vector<std::thread> parsers;
    // the splitter waits for input in poll() on the input and this pipe, so closing the ingest
    // never waits for a slow or stalled writer upstream (an aligner feeding stdin)
    int wake[2] = {-1, -1};
    SamAhead() {
        if (pipe(wake) != 0) wake[0] = wake[1] = -1;
    }
    ~SamAhead() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        if (wake[1] >= 0) {
            const char c = 1;
            ssize_t k;
            do { k = write(wake[1], &c, 1); } while (k < 0 && errno == EINTR);
        }
        if (splitter.joinable()) splitter.join();
        for (std::thread &t : parsers) t.join();
        for (int fd : wake)
            if (fd >= 0) close(fd);
        if ((split_steps || split_jumps) && getenv("FC2_CALLER_TIMING"))   // (the splitter has joined)
            fprintf(stderr, "bgzf split: %llu records read one at a time, %llu jumps through the record lists\n",
                    (unsigned long long)split_steps, (unsigned long long)split_jumps);
    }
};

namespace {

// ---- input plumbing --------------------------------------------------------
bool fill_raw(fc2_ingest *h, std::vector<char> &dst, size_t want) {
    // append up to `want` bytes of raw file data to dst; false at EOF
    size_t old = dst.size();
    dst.resize(old + want);
    ssize_t k;
    do { k = read(h->fd, dst.data() + old, want); } while (k < 0 && errno == EINTR);
    if (k < 0) { h->in_rc = FC2_E_IO; h->in_err = std::string("read error: ") + strerror(errno); }
    if (k <= 0) { dst.resize(old); return false; }
    dst.resize(old + (size_t)k);
    return true;
}

// make at least n bytes available in buf[beg..end); false if the input ends first
bool ensure(fc2_ingest *h, size_t n) {
    while (h->end - h->beg < n) {
        if (h->beg > 0) {  // compact
            memmove(h->buf.data(), h->buf.data() + h->beg, h->end - h->beg);
            h->end -= h->beg;
            h->beg = 0;
        }
        if (h->buf.size() < h->end + (1 << 22)) h->buf.resize(h->end + (1 << 22));
        if (h->src == fc2_ingest::SRC_RAW) {
            if (h->eof_in) return false;
            ssize_t k;
            do { k = read(h->fd, h->buf.data() + h->end, h->buf.size() - h->end); } while (k < 0 && errno == EINTR);
            if (k < 0) { h->in_rc = FC2_E_IO; h->in_err = std::string("read error: ") + strerror(errno); }
            if (k <= 0) { h->eof_in = true; return false; }
            h->end += (size_t)k;
        } else if (h->src == fc2_ingest::SRC_BGZF) {
            if (h->z_done) return false;
            const auto w0 = std::chrono::steady_clock::now();
            BgzfBatch b = h->bgzf_next.get();   // (bgzf_split_loop reads batches without this copy)
            h->inflate_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
            if (!b.err.empty()) { h->z_err = b.err; h->z_done = true; return false; }
            if (b.eof) h->z_done = true;
            else h->bgzf_next = std::async(std::launch::async, bgzf_batch, h->fd, std::vector<uint8_t>(), batch_blocks(h),
                                           h->bgzf_nt, h->gpu_inflate);
            if (h->buf.size() < h->end + b.n) h->buf.resize(h->end + b.n);
            if (b.n) memcpy(h->buf.data() + h->end, b.data(), b.n);
            h->end += b.n;
        } else {
            if (h->z_done) return false;
            // inflate more
            if (h->zs.avail_in == 0) {
                h->zin.clear();
                if (!fill_raw(h, h->zin, 1 << 20)) {
                    h->z_done = true;
                    if (h->z_mid) h->z_err = "truncated gzip stream";
                    return false;
                }
                h->zs.next_in = (Bytef *)h->zin.data();
                h->zs.avail_in = (uInt)h->zin.size();
            }
            h->zs.next_out = (Bytef *)(h->buf.data() + h->end);
            h->zs.avail_out = (uInt)(h->buf.size() - h->end);
            int rc = inflate(&h->zs, Z_NO_FLUSH);
            h->end = h->buf.size() - h->zs.avail_out;
            h->z_mid = true;
            if (rc == Z_STREAM_END) {
                // concatenated gzip members: restart on the remaining input
                h->z_mid = false;
                if (inflateReset(&h->zs) != Z_OK) { h->z_done = true; h->z_err = "zlib reset"; return false; }
            } else if (rc != Z_OK && rc != Z_BUF_ERROR) {
                h->z_done = true;
                h->z_err = "corrupt gzip stream";
                return false;
            }
        }
    }
    return true;
}

// the error that ended the input early, if any (FC2_OK at a clean end of input)
int input_rc(fc2_ingest *h) {
    if (h->in_rc) return fc2::fail(h->in_rc, h->in_err);
    if (!h->z_err.empty()) return fc2::fail(FC2_E_FORMAT, std::string(h->bam ? "BAM" : "SAM") + " input: " + h->z_err);
    return FC2_OK;
}

// SAM: next line as [*s, *e) inside the input buffer (without newline; valid until the next
// call); false at EOF
bool next_line_view(fc2_ingest *h, const char *&ls, const char *&le) {
    for (;;) {
        const char *s = h->buf.data() + h->beg;
        const char *nl = (const char *)memchr(s, '\n', h->end - h->beg);
        if (nl) {
            ls = s;
            le = nl;
            h->beg = (size_t)(nl - h->buf.data()) + 1;
            if (le > ls && le[-1] == '\r') --le;
            return true;
        }
        size_t have = h->end - h->beg;
        if (!ensure(h, have + 1)) {
            if (h->end > h->beg) {
                ls = h->buf.data() + h->beg;
                le = h->buf.data() + h->end;
                h->beg = h->end;
                if (le > ls && le[-1] == '\r') --le;
                return true;
            }
            return false;
        }
    }
}

bool next_line(fc2_ingest *h, std::string &line) {
    const char *s, *e;
    if (!next_line_view(h, s, e)) return false;
    line.assign(s, e);
    return true;
}

// strtoll(field, NULL, 10) semantics; digits-only fields (the normal case) without a copy
int64_t to_i64(const char *b, const char *e) {
    const char *p = b;
    bool neg = false;
    if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
    if (p < e && p - b <= 1) {
        int64_t v = 0;
        const char *q = p;
        while (q < e && *q >= '0' && *q <= '9' && q - p < 18) v = v * 10 + (*q++ - '0');
        if (q == e && q > p) return neg ? -v : v;
    }
    return strtoll(std::string(b, e).c_str(), nullptr, 10);
}

// a SAM text tag value of type ty in [b, e) as pysam returns it: 'i' an int, 'f' the float32 htslib
// stores (strtod, then narrowed), 'B' an array, anything else a str
fc2::ing::PyNum tag_num(char ty, const char *b, const char *e) {
    using fc2::ing::PyNum;
    if (ty == 'i') return PyNum::of_int(to_i64(b, e));
    if (ty == 'f') return PyNum::of_float((double)(float)strtod(std::string(b, e).c_str(), nullptr));
    return PyNum::other(ty == 'B' ? PyNum::ARRAY : PyNum::STR);
}

// AS / XS of one tag in SAM text form "TG:T:value" (first occurrence wins, like get_tag)
void note_tag(Rec &r, const char *t, const char *e) {
    if (e - t < 5 || t[2] != ':' || t[4] != ':') return;
    const bool as = t[0] == 'A' && t[1] == 'S', xs = t[0] == 'X' && t[1] == 'S';
    if (!as && !xs) return;
    const fc2::ing::PyNum v = tag_num(t[3], t + 5, e);
    if (as) {
        if (!r.has_as) { r.has_as = true; r.as = v; }
        r.as_last = v;
    } else {
        if (!r.has_xs) { r.has_xs = true; r.xs = v; }
        r.xs_last = v;
    }
}

void scan_sam_tags(Rec &r, const char *p, const char *end) {
    while (p < end) {
        const char *t = (const char *)memchr(p, '\t', (size_t)(end - p));
        const char *e = t ? t : end;
        note_tag(r, p, e);
        p = e + 1;
    }
}

// the tabs of [b, e) in order, up to maxn of them (16 bytes per SSE2 compare; every x86-64 has it)
int find_tabs(const char *b, const char *e, const char **t, int maxn) {
    int n = 0;
    const char *p = b;
    const __m128i tab = _mm_set1_epi8('\t');
    while (p + 16 <= e && n < maxn) {
        unsigned m = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)p), tab));
        while (m && n < maxn) { t[n++] = p + __builtin_ctz(m); m &= m - 1; }
        p += 16;
    }
    for (; p < e && n < maxn; ++p)
        if (*p == '\t') t[n++] = p;
    return n;
}

int parse_sam_record(fc2_ingest *h, const char *ls, const char *le, Rec &r, fc2_ingest::ParseScratch &ps,
                     bool lazy = false) {
    // every tab of the line in one pass: fields 1-11, then the tags
    constexpr int kMaxTabs = 64;
    const char *tabs[kMaxTabs];
    const int nt = find_tabs(ls, le, tabs, kMaxTabs);
    const char *f[13];
    int nf = 0;
    f[nf++] = ls;
    for (int k = 0; k < nt && nf < 12; ++k) f[nf++] = tabs[k] + 1;
    if (nf < 11) return fc2::fail(FC2_E_FORMAT, "malformed SAM line: " + std::string(ls, std::min<size_t>(80, le - ls)));
    auto fb = [&](int k) { return f[k]; };
    auto fe = [&](int k) { return k < nt ? tabs[k] : le; };
    if (h->need_text || h->bam_out) r.text.assign(ls, le);
    r.qname.assign(fb(0), fe(0));
    r.flag = (uint32_t)to_i64(fb(1), fe(1));
    const char *rb = fb(2), *re = fe(2);
    if (re - rb == 1 && *rb == '*') r.tid = -1;
    else if ((size_t)(re - rb) == ps.last_rn.size() && memcmp(rb, ps.last_rn.data(), ps.last_rn.size()) == 0) {
        r.tid = ps.last_tid;
    } else {
        ps.last_rn.assign(rb, re);
        auto it = h->tid_of.find(ps.last_rn);
        r.tid = ps.last_tid = it == h->tid_of.end() ? -1 : it->second;
    }
    r.pos = to_i64(fb(3), fe(3)) - 1;
    std::vector<std::pair<int, int>> &ops = ps.ops;
    ops.clear();
    const char *cb = fb(5), *ce = fe(5);
    if (!(ce - cb == 1 && *cb == '*')) {
        long n = 0;
        for (const char *c = cb; c < ce; ++c) {
            if (*c >= '0' && *c <= '9') n = n * 10 + (*c - '0');
            else {
                int code = cig_code(*c);
                if (code < 0) return fc2::fail(FC2_E_FORMAT, "bad CIGAR: " + std::string(cb, ce));
                ops.emplace_back(code, (int)n);
                n = 0;
            }
        }
    }
    const char *sb = fb(9), *se = fe(9), *qb = fb(10), *qe = fe(10);
    r.has_seq = !(se - sb == 1 && *sb == '*');
    r.has_qual = !(qe - qb == 1 && *qb == '*');
    r.seq_n = (uint32_t)(se - sb);
    if (lazy) {                                     // decoded if the record is ever needed (Rec::decode)
        r.lz.seq = sb;
        r.lz.qual = qb;
        r.lz.n_seq = (int32_t)(se - sb);
        r.lz.n_qual = (int32_t)(qe - qb);
        r.lz.bam = false;
    } else {
        r.lz.n_seq = -1;
        r.seq.assign(sb, se);
        r.qual.assign(qb, qe);
    }
    r.has_as = r.has_xs = false;
    r.as = r.xs = r.as_last = r.xs_last = fc2::ing::PyNum();
    finish_rec(r, ops, r.has_seq ? (int64_t)r.seq_n : 0);
    if (nf == 12) {                                 // tags: [tabs[k] + 1, next tab or line end), k >= 10
        const int last = nt == kMaxTabs ? nt - 1 : nt;
        for (int k = 10; k < last; ++k) note_tag(r, tabs[k] + 1, k + 1 < nt ? tabs[k + 1] : le);
        if (nt == kMaxTabs) scan_sam_tags(r, tabs[kMaxTabs - 1] + 1, le);   // more tabs than were collected
    }
    return FC2_OK;
}

// Bytes of one aux value of type ty at p (the record ends at end), or -1 where htslib reports
// corrupted aux data: an unknown type, a value running past the record, a Z / H string without its
// NUL, a B array with an unknown element type or a negative count.
ptrdiff_t aux_value_size(char ty, const uint8_t *p, const uint8_t *end) {
    const ptrdiff_t left = end - p;
    ptrdiff_t n;
    switch (ty) {
        case 'c': case 'C': case 'A': n = 1; break;
        case 's': case 'S': n = 2; break;
        case 'i': case 'I': case 'f': n = 4; break;
        case 'Z': case 'H': {
            const uint8_t *z = left > 0 ? (const uint8_t *)memchr(p, 0, (size_t)left) : nullptr;
            return z ? (z - p) + 1 : -1;
        }
        case 'B': {
            if (left < 5) return -1;
            const char sub = (char)p[0];
            const int w = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2
                        : (sub == 'i' || sub == 'I' || sub == 'f') ? 4 : 0;
            int32_t cnt;
            memcpy(&cnt, p + 1, 4);
            if (!w || cnt < 0) return -1;
            n = 5 + (ptrdiff_t)w * cnt;
            break;
        }
        default: return -1;
    }
    return n <= left ? n : -1;
}

// SAM text of the aux fields [p, end), already checked by scan_bam_tags
void append_bam_tags(std::string &t, const uint8_t *p, const uint8_t *end) {
    char tmp[64];
    while (end - p >= 3) {
        const char ty = (char)p[2];
        const ptrdiff_t adv = aux_value_size(ty, p + 3, end);
        if (adv < 0) return;
        t += '\t';
        t.append((const char *)p, 2);
        p += 3;
        auto ival = [&](long long v) { snprintf(tmp, sizeof tmp, ":i:%lld", v); t += tmp; };
        switch (ty) {
            case 'c': ival(*(const int8_t *)p); break;
            case 'C': ival(*(const uint8_t *)p); break;
            case 's': { int16_t v; memcpy(&v, p, 2); ival(v); break; }
            case 'S': { uint16_t v; memcpy(&v, p, 2); ival(v); break; }
            case 'i': { int32_t v; memcpy(&v, p, 4); ival(v); break; }
            case 'I': { uint32_t v; memcpy(&v, p, 4); ival(v); break; }
            // nine significant digits: the Python loop parses back the very float32 (samio._tag_value)
            case 'f': { float v; memcpy(&v, p, 4); snprintf(tmp, sizeof tmp, ":f:%.9g", v); t += tmp; break; }
            case 'A': t += ":A:"; t += (char)*p; break;
            case 'Z': case 'H':
                t += ':'; t += ty; t += ':';
                t.append((const char *)p, (size_t)(adv - 1));
                break;
            case 'B': {
                const char sub = (char)p[0];
                int32_t cnt; memcpy(&cnt, p + 1, 4);
                const uint8_t *q = p + 5;
                t += ":B:"; t += sub;
                for (int32_t k = 0; k < cnt; ++k) {
                    t += ',';
                    switch (sub) {
                        case 'c': snprintf(tmp, sizeof tmp, "%d", *(const int8_t *)q); q += 1; break;
                        case 'C': snprintf(tmp, sizeof tmp, "%u", *(const uint8_t *)q); q += 1; break;
                        case 's': { int16_t v; memcpy(&v, q, 2); snprintf(tmp, sizeof tmp, "%d", v); q += 2; break; }
                        case 'S': { uint16_t v; memcpy(&v, q, 2); snprintf(tmp, sizeof tmp, "%u", v); q += 2; break; }
                        case 'i': { int32_t v; memcpy(&v, q, 4); snprintf(tmp, sizeof tmp, "%d", v); q += 4; break; }
                        case 'I': { uint32_t v; memcpy(&v, q, 4); snprintf(tmp, sizeof tmp, "%u", v); q += 4; break; }
                        default: { float v; memcpy(&v, q, 4); snprintf(tmp, sizeof tmp, "%g", v); q += 4; break; }
                    }
                    t += tmp;
                }
                break;
            }
        }
        p += adv;
    }
}

// AS / XS from binary BAM tags, as pysam's get_tag returns them (fc2::ing::PyNum); false when the
// aux data is corrupt (aux_value_size) or ends inside a tag
bool scan_bam_tags(Rec &r, const uint8_t *p, const uint8_t *end) {
    using fc2::ing::PyNum;
    while (p < end) {
        if (end - p < 3) return false;
        const char t0 = (char)p[0], t1 = (char)p[1], ty = (char)p[2];
        p += 3;
        const ptrdiff_t adv = aux_value_size(ty, p, end);
        if (adv < 0) return false;
        const bool as = t0 == 'A' && t1 == 'S', xs = t0 == 'X' && t1 == 'S';
        if (as || xs) {
            PyNum v;
            switch (ty) {
                case 'c': v = PyNum::of_int(*(const int8_t *)p); break;
                case 'C': v = PyNum::of_int(*(const uint8_t *)p); break;
                case 's': { int16_t x; memcpy(&x, p, 2); v = PyNum::of_int(x); break; }
                case 'S': { uint16_t x; memcpy(&x, p, 2); v = PyNum::of_int(x); break; }
                case 'i': { int32_t x; memcpy(&x, p, 4); v = PyNum::of_int(x); break; }
                case 'I': { uint32_t x; memcpy(&x, p, 4); v = PyNum::of_int(x); break; }
                case 'f': { float x; memcpy(&x, p, 4); v = PyNum::of_float(x); break; }
                case 'B': v = PyNum::other(PyNum::ARRAY); break;
                default: v = PyNum::other(PyNum::STR); break;          // A Z H
            }
            if (as && !r.has_as) { r.has_as = true; r.as = v; }
            if (xs && !r.has_xs) { r.has_xs = true; r.xs = v; }
            if (as) r.as_last = v;
            if (xs) r.xs_last = v;
        }
        p += adv;
    }
    return true;
}

// one BAM record body (b: the bs bytes after block_size) into r; thread-safe (reads only the
// header's reference names), so parser threads can call it.  ops: CIGAR scratch.  A record whose
// fields do not fit its block, with an unterminated query name or corrupt aux data is an error, as
// in htslib's bam_read1 / aux parsing.
int parse_bam_body(const fc2_ingest *h, const uint8_t *b, int32_t bs, Rec &r,
                   std::vector<std::pair<int, int>> &ops, bool need_text, bool keep_raw, bool lazy = false) {
    if (bs < 32) return fc2::fail(FC2_E_FORMAT, "invalid BAM record (block shorter than its fixed fields)");
    const uint8_t *e = b + bs;
    int32_t ref_id, pos, l_seq, nref, npos, tlen;
    uint8_t l_name, mapq;
    uint16_t bin, n_cig, flag;
    memcpy(&ref_id, b, 4); memcpy(&pos, b + 4, 4); l_name = b[8]; mapq = b[9]; memcpy(&bin, b + 10, 2);
    memcpy(&n_cig, b + 12, 2); memcpy(&flag, b + 14, 2); memcpy(&l_seq, b + 16, 4); memcpy(&nref, b + 20, 4);
    memcpy(&npos, b + 24, 4); memcpy(&tlen, b + 28, 4);
    if (l_seq < 0 || 32 + (int64_t)l_name + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2 + (int64_t)l_seq > bs)
        return fc2::fail(FC2_E_FORMAT, "invalid BAM record (its fields exceed its block size)");
    if (l_name == 0 || b[32 + l_name - 1] != 0)
        return fc2::fail(FC2_E_FORMAT, "invalid BAM record (query name not NUL-terminated)");
    if (keep_raw) r.raw.assign((const char *)b - 4, 4 + (size_t)bs);
    const uint8_t *p = b + 32;
    r.qname.assign((const char *)p, l_name - 1);
    p += l_name;
    ops.resize(n_cig);
    for (int k = 0; k < n_cig; ++k) {
        uint32_t c; memcpy(&c, p + 4 * k, 4);
        ops[k] = {(int)(c & 0xF), (int)(c >> 4)};
    }
    const uint8_t *cigp = p;
    p += 4 * n_cig;
    r.lz.seq = (const char *)p;
    r.lz.qual = (const char *)p + (l_seq + 1) / 2;
    r.lz.n_seq = l_seq;
    r.lz.bam = true;
    r.has_seq = l_seq > 0;
    r.has_qual = !(l_seq == 0 || p[(l_seq + 1) / 2] == 0xFF);
    r.seq_n = r.has_seq ? (uint32_t)l_seq : 1u;
    if (!lazy) r.decode_lazy();                 // (else when the record is needed: Rec::decode)
    p += (l_seq + 1) / 2 + l_seq;
    r.flag = flag;
    r.tid = ref_id;
    r.pos = pos;
    finish_rec(r, ops, l_seq);
    r.has_as = r.has_xs = false;
    r.as = r.xs = r.as_last = r.xs_last = fc2::ing::PyNum();
    if (!scan_bam_tags(r, p, e)) return fc2::fail(FC2_E_FORMAT, "corrupted aux data in a BAM record");
    if (!need_text) return FC2_OK;
    const std::string &seq = r.seq, &qual = r.qual;
    std::string cig;
    char tmp[32];
    for (int k = 0; k < n_cig; ++k) {
        uint32_t c; memcpy(&c, cigp + 4 * k, 4);
        snprintf(tmp, sizeof tmp, "%u%c", c >> 4, "MIDNSHP=X"[(c & 0xF) < 9 ? (c & 0xF) : 0]);
        cig += tmp;
    }
    // SAM text (hand-back to the Python caller)
    std::string &t = r.text;
    t = r.qname;
    snprintf(tmp, sizeof tmp, "\t%u\t", flag); t += tmp;
    t += (ref_id >= 0 && ref_id < (int)h->refs.size()) ? h->refs[ref_id] : std::string("*");
    snprintf(tmp, sizeof tmp, "\t%d\t%u\t", pos + 1, mapq); t += tmp;
    t += cig.empty() ? std::string("*") : cig;
    t += "\t*\t0\t0\t";
    t += seq;
    t += '\t';
    t += qual;
    append_bam_tags(t, p, e);
    return FC2_OK;
}

int parse_bam_record(fc2_ingest *h, Rec &r, bool &got) {
    got = false;
    if (!ensure(h, 4)) {
        if (int rc = input_rc(h)) return rc;
        return h->end > h->beg ? fc2::fail(FC2_E_FORMAT, "truncated BAM record") : FC2_OK;
    }
    int32_t bs;
    memcpy(&bs, h->buf.data() + h->beg, 4);
    if (bs < 32 || !ensure(h, 4 + (size_t)bs))
        return fc2::fail(FC2_E_FORMAT, "truncated BAM record" + (h->z_err.empty() ? "" : " (" + h->z_err + ")"));
    if (int rc = parse_bam_body(h, (const uint8_t *)h->buf.data() + h->beg + 4, bs, r, h->ops, h->need_text,
                                h->bam_out != nullptr))
        return rc;
    h->beg += 4 + (size_t)bs;
    got = true;
    return FC2_OK;
}

int read_header(fc2_ingest *h) {
    if (!h->bam) {
        std::string line;
        for (;;) {
            // peek: header lines start with '@'
            if (!ensure(h, 1)) return input_rc(h);
            if (h->buf[h->beg] != '@') return FC2_OK;
            if (!next_line(h, line)) return input_rc(h);
            h->header += line;
            h->header += '\n';
            if (line.compare(0, 3, "@SQ") == 0) {
                size_t p = line.find("\tSN:");
                if (p != std::string::npos) {
                    size_t e = line.find('\t', p + 4);
                    std::string name = line.substr(p + 4, e == std::string::npos ? std::string::npos : e - p - 4);
                    h->tid_of[name] = (int)h->refs.size();
                    h->refs.push_back(name);
                    size_t q = line.find("\tLN:");
                    h->ref_len.push_back(q == std::string::npos ? 0 : strtoll(line.c_str() + q + 4, nullptr, 10));
                }
            }
        }
    }
    if (!ensure(h, 12)) return fc2::fail(FC2_E_FORMAT, "truncated BAM header" + (h->z_err.empty() ? "" : " (" + h->z_err + ")"));
    if (memcmp(h->buf.data() + h->beg, "BAM\1", 4) != 0) return fc2::fail(FC2_E_FORMAT, "not a BAM file");
    int32_t lt;
    memcpy(&lt, h->buf.data() + h->beg + 4, 4);
    if (lt < 0) return fc2::fail(FC2_E_FORMAT, "invalid BAM header (negative text length)");
    if (!ensure(h, 8 + (size_t)lt + 4))
        return fc2::fail(FC2_E_FORMAT, "truncated BAM header" + (h->z_err.empty() ? "" : " (" + h->z_err + ")"));
    h->header.assign(h->buf.data() + h->beg + 8, (size_t)lt);
    while (!h->header.empty() && h->header.back() == '\0') h->header.pop_back();
    h->beg += 8 + (size_t)lt;
    int32_t nref;
    memcpy(&nref, h->buf.data() + h->beg, 4);
    h->beg += 4;
    for (int k = 0; k < nref; ++k) {
        if (!ensure(h, 4)) return fc2::fail(FC2_E_FORMAT, "truncated BAM refs");
        int32_t ln;
        memcpy(&ln, h->buf.data() + h->beg, 4);
        if (ln <= 0) return fc2::fail(FC2_E_FORMAT, "invalid BAM header (reference name length)");
        if (!ensure(h, 4 + (size_t)ln + 4)) return fc2::fail(FC2_E_FORMAT, "truncated BAM refs");
        std::string name(h->buf.data() + h->beg + 4, (size_t)ln - 1);
        int32_t lref;
        memcpy(&lref, h->buf.data() + h->beg + 4 + ln, 4);
        h->ref_len.push_back(lref);
        h->beg += 4 + (size_t)ln + 4;
        h->tid_of[name] = (int)h->refs.size();
        h->refs.push_back(name);
    }
    return FC2_OK;
}

// splitter: the input from where the header ended, in newline-aligned numbered blocks
// (A is handed over, not read from h->ahead: closing resets h->ahead before ~SamAhead joins, and a
// thread that only starts running then must still find its object)
void sam_split_loop(fc2_ingest *h, fc2_ingest::SamAhead *ap) {
    fc2::cpu::Scope acct(fc2::cpu::SPLIT);
    auto &A = *ap;
    std::string carry(h->buf.data() + h->beg, h->end - h->beg);   // bytes read with the header
    h->beg = h->end;
    bool in_eof = h->eof_in;
    for (uint64_t seq = 0;; ++seq) {
        std::unique_ptr<fc2_ingest::SamAhead::Batch> b;
        {
            std::unique_lock<std::mutex> lk(A.m);
            const auto w0 = std::chrono::steady_clock::now();
            A.cv.wait(lk, [&] { return A.stop || A.inflight < A.max_inflight; });
            A.split_block_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
            if (A.stop) return;
            ++A.inflight;
            if (!A.spare.empty()) { b = std::move(A.spare.back()); A.spare.pop_back(); }
        }
        if (!b) b.reset(new fc2_ingest::SamAhead::Batch());
        b->seq = seq;
        b->n = 0;
        b->rc = FC2_OK;
        b->err.clear();
        b->read_rc = FC2_OK;
        b->read_err.clear();
        b->eof = false;
        std::string &blk = b->block;
        blk.swap(carry);
        carry.clear();
        // read until the block holds kBlock bytes and a newline, or the input ends
        bool has_nl = memchr(blk.data(), '\n', blk.size()) != nullptr;
        while (!in_eof && (blk.size() < A.block || !has_nl)) {
            if (A.wake[0] >= 0) {
                pollfd pf[2] = {{h->fd, POLLIN, 0}, {A.wake[0], POLLIN, 0}};
                int pr;
                do { pr = poll(pf, 2, -1); } while (pr < 0 && errno == EINTR);
                if (pr > 0 && pf[1].revents) return;       // the ingest is closing
            }
            const size_t have = blk.size();
            blk.resize(have + A.block);
            ssize_t k;
            do { k = read(h->fd, &blk[have], A.block); } while (k < 0 && errno == EINTR);
            if (k < 0) {
                blk.resize(have);
                b->read_rc = FC2_E_IO;
                b->read_err = std::string("read error: ") + strerror(errno);
                in_eof = true;
                break;
            }
            blk.resize(have + (size_t)k);
            if (k == 0) in_eof = true;
            else if (!has_nl) has_nl = memchr(&blk[have], '\n', (size_t)k) != nullptr;
        }
        if (!in_eof) {                          // whole lines only; the rest starts the next block
            const size_t nl = blk.rfind('\n');   // exists: the loop above read up to one
            carry.assign(blk, nl + 1, std::string::npos);
            blk.resize(nl + 1);
        } else {
            b->eof = true;
            if (b->read_rc) {                   // a line cut short by the failed read is not a record
                const size_t nl = blk.rfind('\n');
                blk.resize(nl == std::string::npos ? 0 : nl + 1);
            }
        }
        const bool last = b->eof;
        {
            std::lock_guard<std::mutex> lk(A.m);
            A.todo.push_back(std::move(b));
        }
        A.cv.notify_all();
        if (last) return;
    }
}

// BAM splitter: the decompressed stream (ensure(): BGZF blocks inflated on their own threads, or
// any gzip stream) cut into numbered blocks of whole records (block_size + body), ~kBlock bytes
// each.  Where the stream ends inside a record, or the input fails, the block ends after the last
// whole record and carries the error parse_bam_record would have reported there.
void bam_split_loop(fc2_ingest *h, fc2_ingest::SamAhead *ap) {
    fc2::cpu::Scope acct(fc2::cpu::SPLIT);
    auto &A = *ap;
    for (uint64_t seq = 0;; ++seq) {
        std::unique_ptr<fc2_ingest::SamAhead::Batch> b;
        {
            std::unique_lock<std::mutex> lk(A.m);
            const auto w0 = std::chrono::steady_clock::now();
            A.cv.wait(lk, [&] { return A.stop || A.inflight < A.max_inflight; });
            A.split_block_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
            if (A.stop) return;
            ++A.inflight;
            if (!A.spare.empty()) { b = std::move(A.spare.back()); A.spare.pop_back(); }
        }
        if (!b) b.reset(new fc2_ingest::SamAhead::Batch());
        b->seq = seq;
        b->n = 0;
        b->rc = FC2_OK;
        b->err.clear();
        b->read_rc = FC2_OK;
        b->read_err.clear();
        b->eof = false;
        std::string &blk = b->block;
        blk.clear();
        auto truncated = [&]() {
            b->read_rc = FC2_E_FORMAT;
            b->read_err = "truncated BAM record" + (h->z_err.empty() ? "" : " (" + h->z_err + ")");
            b->eof = true;
        };
        while (blk.size() < A.block) {
            if (!ensure(h, 4)) {                // end of input (clean, or an input error first)
                if (h->in_rc) { b->read_rc = h->in_rc; b->read_err = h->in_err; }
                else if (!h->z_err.empty()) { b->read_rc = FC2_E_FORMAT; b->read_err = "BAM input: " + h->z_err; }
                else if (h->end > h->beg) truncated();
                b->eof = true;
                break;
            }
            // every whole record in the buffer, in one copy
            const char *base = h->buf.data();
            size_t q = h->beg;
            while (q + 4 <= h->end) {
                int32_t bs;
                memcpy(&bs, base + q, 4);
                if (bs < 32 || q + 4 + (size_t)bs > h->end) break;
                q += 4 + (size_t)bs;
                if (blk.size() + (q - h->beg) >= A.block) break;
            }
            if (q > h->beg) {
                blk.append(base + h->beg, q - h->beg);
                h->beg = q;
                continue;
            }
            int32_t bs;                         // the record at beg is not whole yet
            memcpy(&bs, base + h->beg, 4);
            if (bs < 32 || !ensure(h, 4 + (size_t)bs)) { truncated(); break; }
        }
        const bool last = b->eof;
        {
            std::lock_guard<std::mutex> lk(A.m);
            A.todo.push_back(std::move(b));
        }
        A.cv.notify_all();
        if (last) return;
    }
}

// BGZF input parsed ahead: the inflated batches are cut into blocks of whole records in place --
// a block is a view into its batch's buffer, shared with the parse threads, and the record cut by a
// batch's end moves into the next batch's headroom (kHead) -- so the stream is never copied in bulk
// on this thread (bam_split_loop copies it twice: into the reader's buffer, then into the block).
// The errors are bam_split_loop's, at the same records.
void bgzf_split_loop(fc2_ingest *h, fc2_ingest::SamAhead *ap) {
    fc2::cpu::Scope acct(fc2::cpu::SPLIT);
    auto &A = *ap;
    std::shared_ptr<CharBuf> cur = std::make_shared<CharBuf>(h->buf.begin() + (ptrdiff_t)h->beg,
                                                             h->buf.begin() + (ptrdiff_t)h->end);   // inflated with the header
    size_t beg = 0, end = cur->size();
    h->beg = h->end;
    std::shared_ptr<RecLists> lists;            // the current batch's record lists, its bytes from `base` on
    size_t base = 0;
    // the next batch behind the bytes not yet cut; false at the end of the input or an input error
    auto more = [&]() -> bool {
        if (h->z_done) return false;
        const auto w0 = std::chrono::steady_clock::now();
        BgzfBatch b = h->bgzf_next.get();
        h->inflate_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
        if (!b.err.empty()) { h->z_err = b.err; h->z_done = true; return false; }
        if (b.eof) h->z_done = true;
        else h->bgzf_next = std::async(std::launch::async, bgzf_batch, h->fd, std::vector<uint8_t>(), batch_blocks(h), h->bgzf_nt,
                                       h->gpu_inflate);
        const size_t L = end - beg;
        std::shared_ptr<CharBuf> nb;
        if (L <= kHead) {
            if (L) memcpy(b.out.data() + kHead - L, cur->data() + beg, L);
            nb = std::make_shared<CharBuf>(std::move(b.out));
            beg = kHead - L;
        } else {                                // a record longer than the headroom: joined by copy
            nb = std::make_shared<CharBuf>();
            nb->reserve(L + b.n);
            nb->insert(nb->end(), cur->data() + beg, cur->data() + end);
            nb->insert(nb->end(), b.data(), b.data() + b.n);
            beg = 0;
        }
        end = beg + L + b.n;
        lists = std::move(b.recs);
        base = beg + L;
        cur = std::move(nb);
        return true;
    };
    for (uint64_t seq = 0;; ++seq) {
        std::unique_ptr<fc2_ingest::SamAhead::Batch> b;
        {
            std::unique_lock<std::mutex> lk(A.m);
            const auto w0 = std::chrono::steady_clock::now();
            A.cv.wait(lk, [&] { return A.stop || A.inflight < A.max_inflight; });
            A.split_block_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
            if (A.stop) return;
            ++A.inflight;
            if (!A.spare.empty()) { b = std::move(A.spare.back()); A.spare.pop_back(); }
        }
        if (!b) b.reset(new fc2_ingest::SamAhead::Batch());
        b->seq = seq;
        b->n = 0;
        b->rc = FC2_OK;
        b->err.clear();
        b->read_rc = FC2_OK;
        b->read_err.clear();
        b->eof = false;
        b->block.clear();
        b->vbuf.reset();
        b->voff = b->vlen = 0;
        auto truncated = [&]() {
            b->read_rc = FC2_E_FORMAT;
            b->read_err = "truncated BAM record" + (h->z_err.empty() ? "" : " (" + h->z_err + ")");
            b->eof = true;
        };
        for (;;) {
            // every whole record from beg on, up to a block's worth: the first record end at or past
            // beg + A.block, or the last whole one.  Where the chain of records from beg reaches a start
            // the inflating threads listed, the rest of that BGZF block's records are the list's (the
            // same block sizes, already read): the cut is found there, or the chain continues at the
            // list's exit; elsewhere (no list, a start it missed, a record past the batch's end, a
            // block_size below 32) one record at a time
            const char *bp = cur->data();
            size_t q = beg;
            for (;;) {
                if (lists && q >= base && q - base < lists->n) {
                    const uint64_t bq = q - base;
                    const size_t j = (size_t)(std::upper_bound(lists->ooff.begin(), lists->ooff.end(), (size_t)bq) -
                                              lists->ooff.begin()) - 1;
                    const std::vector<uint32_t> &S = lists->starts[j];
                    const auto it = std::lower_bound(S.begin(), S.end(), (uint32_t)bq);
                    if (it != S.end() && *it == bq) {
                        const uint64_t tb = beg + A.block - base;   // > bq: q - beg < A.block here
                        const auto c = std::lower_bound(it + 1, S.end(), (uint32_t)std::min<uint64_t>(tb, UINT32_MAX));
                        if (c != S.end() && *c >= tb) { q = base + *c; ++A.split_jumps; break; }
                        const uint64_t ex = lists->exit[j];
                        if (ex != kNoExit && base + ex <= end) {
                            q = base + ex;
                            ++A.split_jumps;
                            if (q - beg >= A.block) break;
                            continue;
                        }
                        q = base + S.back();            // its last record on, one at a time
                    }
                }
                if (q + 4 > end) break;
                int32_t bs;
                memcpy(&bs, bp + q, 4);
                if (bs < 32 || q + 4 + (size_t)bs > end) break;
                q += 4 + (size_t)bs;
                ++A.split_steps;
                if (q - beg >= A.block) break;
            }
            if (q > beg) {
                b->vbuf = cur;
                b->voff = beg;
                b->vlen = q - beg;
                beg = q;
                break;
            }
            if (end - beg < 4) {                // no whole record: the input ends here, or more comes
                if (more()) continue;
                if (!h->z_err.empty()) { b->read_rc = FC2_E_FORMAT; b->read_err = "BAM input: " + h->z_err; }
                else if (end > beg) truncated();
                b->eof = true;
                break;
            }
            int32_t bs;                         // the record at beg is not whole yet
            memcpy(&bs, bp + beg, 4);
            if (bs < 32 || !more()) { truncated(); break; }
        }
        const bool last = b->eof;
        {
            std::lock_guard<std::mutex> lk(A.m);
            A.todo.push_back(std::move(b));
        }
        A.cv.notify_all();
        if (last) return;
    }
}

void group_batch(const fc2_ingest_params &p, fc2_ingest::SamAhead::Batch &b);

// parser: blocks to record batches (own RNAME cache and CIGAR scratch)
void sam_parse_loop(fc2_ingest *h, fc2_ingest::SamAhead *ap) {
    fc2::cpu::Scope acct(fc2::cpu::PARSE);
    auto &A = *ap;
    fc2_ingest::ParseScratch ps;
    for (;;) {
        std::unique_ptr<fc2_ingest::SamAhead::Batch> b;
        {
            std::unique_lock<std::mutex> lk(A.m);
            const auto w0 = std::chrono::steady_clock::now();
            A.cv.wait(lk, [&] { return A.stop || !A.todo.empty(); });
            A.parse_idle_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
            if (A.stop) return;
            b = std::move(A.todo.front());
            A.todo.pop_front();
        }
        const char *p = b->vbuf ? b->vbuf->data() + b->voff : b->block.data();
        const char *end = p + (b->vbuf ? b->vlen : b->block.size());
        while (h->bam && p < end && b->rc == FC2_OK) {     // whole BAM records (bam/bgzf_split_loop)
            int32_t bs;
            memcpy(&bs, p, 4);
            if (b->n == b->recs.size()) b->recs.emplace_back();
            const int rc = parse_bam_body(h, (const uint8_t *)p + 4, bs, b->recs[b->n], ps.ops, h->need_text, false,
                                          !h->need_text);
            if (rc) { b->rc = rc; b->err = fc2_last_error(); break; }
            ++b->n;
            p += 4 + (size_t)bs;
        }
        while (!h->bam && p < end && b->rc == FC2_OK) {
            const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
            const char *ls = p, *le = nl ? nl : end;
            p = nl ? nl + 1 : end;
            if (le > ls && le[-1] == '\r') --le;
            bool blank = true;
            for (const char *c = ls; c < le; ++c) if (!isspace((unsigned char)*c)) { blank = false; break; }
            if (blank) continue;
            if (b->n == b->recs.size()) b->recs.emplace_back();
            const int rc = parse_sam_record(h, ls, le, b->recs[b->n], ps, !h->need_text);
            if (rc) { b->rc = rc; b->err = fc2_last_error(); break; }
            ++b->n;
        }
        if (b->rc == FC2_OK && b->read_rc) { b->rc = b->read_rc; b->err = b->read_err; }
        b->gs = b->gt = 0;
        if (A.group) group_batch(A.gp, *b);
        {
            std::lock_guard<std::mutex> lk(A.m);
            const uint64_t seq = b->seq;
            A.done.emplace(seq, std::move(b));
        }
        A.cv.notify_all();
    }
}

// the consumer side of next_record: the next parsed record, in place in its batch (valid until the
// next call; open_mate / add_segment swap it out)
Rec *next_ahead(fc2_ingest *h, int &rc) {
    auto &A = *h->ahead;
    for (;;) {
        if (!A.cur) {
            std::unique_lock<std::mutex> lk(A.m);
            if (!A.done.count(A.next_consume)) {
                const auto w0 = std::chrono::steady_clock::now();
                A.cv.wait(lk, [&] { return A.done.count(A.next_consume) != 0; });
                A.wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
            }
            auto it = A.done.find(A.next_consume);
            A.cur = std::move(it->second);
            A.done.erase(it);
            ++A.next_consume;
            A.pos = 0;
        }
        if (A.pos < A.cur->n) return &A.cur->recs[A.pos++];
        if (A.cur->rc) { rc = fc2::fail(A.cur->rc, A.cur->err); return nullptr; }   // stays: reported again
        if (A.cur->eof) return nullptr;
        {
            std::lock_guard<std::mutex> lk(A.m);
            --A.inflight;
            if (A.pin) A.pinned.push_back(std::move(A.cur));
            else A.spare.push_back(std::move(A.cur));
        }
        A.cv.notify_all();
    }
}

bool next_record(fc2_ingest *h, Rec &r, int &rc) {
    rc = FC2_OK;
    if (h->bam) {
        bool got;
        rc = parse_bam_record(h, r, got);
        return rc == FC2_OK && got;
    }
    const char *ls, *le;
    for (;;) {
        if (!next_line_view(h, ls, le)) { rc = input_rc(h); return false; }
        bool blank = true;
        for (const char *c = ls; c < le; ++c) if (!isspace((unsigned char)*c)) { blank = false; break; }
        if (blank) continue;
        rc = parse_sam_record(h, ls, le, r, h->ps);
        return rc == FC2_OK;
    }
}

// ---- fragment logic ----------------------------------------------------------
// a mate's records stay in place for reuse (RecList): their strings keep their capacity
void recycle(fc2_ingest *h, Mate &m) {
    (void)h;
    m.recs.clear();
    m.proper.clear();
    m.valid = false;
}

// r's record opens / joins the mate; r gets back a recycled record
void open_mate(fc2_ingest *h, Mate &m, Rec &r) {
    h->counts.total_mates++;
    recycle(h, m);
    m.recs.take(r);
    m.proper.push_back(0);
    m.valid = true;
}

void add_segment(Mate &m, Rec &r) {
    const Rec &p = m.recs[0];
    const bool proper = r.tid == p.tid && r.reverse() == p.reverse();
    m.recs.take(r);
    if (proper) m.proper.push_back((int)m.recs.size() - 1);
}

struct MateEval {
    int n_circ = 0, n_lin = 0, too_short = 0;
    bool unspliced = false;
    bool python_must_see = false;   // the reference would fail or compute on it: let the caller do it
};

MateEval eval_mate(const MateRef &m, int asize) {
    MateEval ev;
    if (m.np < 2) { ev.unspliced = true; return ev; }
    const Rec &prim = m.rec(0);
    if (!prim.has_seq) { ev.python_must_see = true; return ev; }   // len(None) in the reference
    for (uint32_t k = 0; k < m.np; ++k) {
        const Rec &s = m.rec((size_t)m.proper[k]);
        if (s.qlen < 0 || s.aend < 0) { ev.python_must_see = true; return ev; }
    }
    int small[16];
    std::vector<int> big;
    int *segs = small;
    const size_t n = m.np;
    if (n > 16) { big.assign(m.proper, m.proper + n); segs = big.data(); }
    else std::copy(m.proper, m.proper + n, small);
    for (size_t i = 1; i < n; ++i) {            // stable insertion sort by query start
        const int v = segs[i];
        size_t j = i;
        while (j > 0 && m.rec((size_t)segs[j - 1]).astart > m.rec((size_t)v).astart) { segs[j] = segs[j - 1]; --j; }
        segs[j] = v;
    }
    for (size_t k = 0; k + 1 < n; ++k) {
        const Rec &a = m.rec((size_t)segs[k]), &b = m.rec((size_t)segs[k + 1]);
        if (a.qlen < asize || b.qlen < asize) { ev.too_short++; continue; }
        // JunctionSpan.__init__ raises on these whether or not the span is ever evaluated
        // (uniqness: AS missing, or a str / array AS or XS, :809-819): the caller must see the
        // fragment even under --no-linear
        if (!a.has_as || !b.has_as || !a.as.number() || !b.as.number() || (a.has_xs && !a.xs.number()) ||
            (b.has_xs && !b.xs.number())) {
            ev.python_must_see = true;
            return ev;
        }
        if (b.pos - a.aend < 0) ev.n_circ++; else ev.n_lin++;
    }
    return ev;
}

// -B: what adjacent_segment_pairs writes while process_mate consumes it (find_circ.py:1134-1140):
// seg_a of every pair that passes the anchor-length filter, then the last pair's seg_b.  A mate
// on which the reference raises (len(None) at :1101 / :1497, A.aend None at :851) stops all
// writing: the run ends there.
int write_anchors(fc2_ingest *h, const Mate &m, int asize) {
    if (m.proper.size() < 2) return FC2_OK;
    const Rec &prim = m.recs[0];
    if (!prim.has_seq) { h->bam_stopped = true; return FC2_OK; }
    for (int k : m.proper)
        if (m.recs[k].qlen < 0) { h->bam_stopped = true; return FC2_OK; }
    std::vector<int> segs(m.proper.begin(), m.proper.end());
    std::stable_sort(segs.begin(), segs.end(), [&](int a, int b) { return m.recs[a].astart < m.recs[b].astart; });
    auto put = [&](const Rec &r) {
        bool ok;
        if (h->bam) ok = fc2::bam::write_raw(h->bam_out, (const uint8_t *)r.raw.data(), r.raw.size());
        else ok = fc2::bam::write_sam(h->bam_out, r.text.data(), r.text.data() + r.text.size(), h->tid_of, h->bam_err);
        if (!ok) return fc2::fail(FC2_E_IO, h->bam_err.empty() ? "IOError: writing spliced_alignments.bam" : h->bam_err);
        return (int)FC2_OK;
    };
    for (size_t k = 0; k + 1 < segs.size(); ++k) {
        const Rec &a = m.recs[segs[k]], &b = m.recs[segs[k + 1]];
        if (a.qlen < asize || b.qlen < asize) continue;
        if (int rc = put(a)) return rc;
        if (a.aend < 0) { h->bam_stopped = true; return FC2_OK; }
    }
    return put(m.recs[segs.back()]);
}

MateRef ref_of(Mate &m) {
    MateRef r;
    r.base = m.recs.begin();
    r.n = (uint32_t)m.recs.size();
    r.proper = m.proper.data();
    r.np = (uint32_t)m.proper.size();
    r.seq_len = m.recs.empty() ? 0 : m.recs[0].seq_n;
    return r;
}

int emit_or_count(fc2_ingest *h, const fc2_ingest_params *p, uint64_t &n_handed,
                  const fc2::ing::FragSink *sink) {
    h->counts.n_reads++;
    if (p->noop) return FC2_OK;
    if (h->bam_out) {
        const Mate *order[2] = {h->have_other ? &h->other : nullptr, &h->current};
        for (const Mate *m : order)
            if (m && !h->bam_stopped)
                if (int rc = write_anchors(h, *m, p->asize)) return rc;
    }
    const Mate *mates[2] = {h->have_other ? &h->other : nullptr, &h->current};
    MateRef refs[2] = {h->have_other ? ref_of(h->other) : MateRef(), ref_of(h->current)};
    MateEval ev[2];
    int circ = 0, lin = 0;
    bool must = false;
    for (int k = 0; k < 2; ++k) {
        if (!mates[k]) continue;
        ev[k] = eval_mate(refs[k], p->asize);
        circ += ev[k].n_circ;
        lin += ev[k].n_lin;
        must |= ev[k].python_must_see;
    }
    bool hand = must || ((circ || lin) && !(circ == 0 && p->nolinear));
    if (!hand) {
        for (int k = 0; k < 2; ++k) {
            if (!mates[k]) continue;
            if (ev[k].unspliced) h->counts.unspliced_mates++;
            h->counts.seg_too_short_skip += (uint64_t)ev[k].too_short;
        }
        return FC2_OK;
    }
    ++n_handed;
    h->counts.handed_back++;
    if (sink) return (*sink)(h->have_other ? &refs[0] : nullptr, &refs[1], must);
    for (int k = 0; k < 2; ++k) {
        if (!mates[k]) continue;
        for (const Rec &r : mates[k]->recs) { h->out += r.text; h->out += '\n'; }
    }
    h->out += '\n';
    return FC2_OK;
}

// ---- grouping on the parse threads ---------------------------------------------------------------
// The loop above closes a fragment at every mapped record whose qname differs from the current
// primary's.  In a batch, let P be the qname of its first mapped record: the first mapped record
// with another qname (gs) closes a fragment whatever came before the batch -- every mapped record
// before it has qname P, so the primary then has qname P too (a continued mate keeps its primary,
// whose qname matched; an opened one has qname P).  From gs on the batch is grouped here, on its
// parse thread, exactly as the loop would: the fragments closed in [gs, gt) with their counts, the
// handed ones listed for the sink; the consumer closes the fragment before gs, takes the list, and
// goes on sequentially from gt (whose record opens the fragment still open at the batch's end).
void group_batch(const fc2_ingest_params &p, fc2_ingest::SamAhead::Batch &b) {
    using Batch = fc2_ingest::SamAhead::Batch;
    b.gs = b.gt = 0;
    b.gfrags.clear();
    b.gidx.clear();
    b.gtotal = fc2_ingest_counts{};
    b.gtotal_frags = 0;
    Rec *R = b.recs.data();
    const size_t n = b.n;
    size_t i = 0;
    while (i < n && R[i].unmapped()) ++i;
    if (i == n) return;
    size_t s = i + 1;
    while (s < n && (R[s].unmapped() || R[s].qname == R[i].qname)) ++s;
    if (s >= n) return;
    struct LM {                                 // a mate: record positions, proper indices
        std::vector<int32_t> r, p;
    };
    thread_local LM cur, oth;
    bool have_oth = false;
    fc2_ingest_counts C{};
    uint64_t F = 0;
    fc2_ingest_counts Ct{};
    uint64_t Ft = 0;
    uint64_t span_cum = 0, arena_cum = 0;
    size_t t = s;
    auto open = [&](LM &m, size_t j) {
        C.total_mates++;
        m.r.clear();
        m.p.clear();
        m.r.push_back((int32_t)j);
        m.p.push_back(0);
    };
    auto ref = [&](LM &m) {
        MateRef x;
        x.base = R;
        x.idx = m.r.data();
        x.n = (uint32_t)m.r.size();
        x.proper = m.p.data();
        x.np = (uint32_t)m.p.size();
        return x;
    };
    // emit_or_count without a -B writer
    auto close = [&]() {
        C.n_reads++;
        ++F;
        if (p.noop) return;
        LM *ms[2] = {have_oth ? &oth : nullptr, &cur};
        MateEval ev[2];
        int circ = 0, lin = 0;
        bool must = false;
        for (int k = 0; k < 2; ++k) {
            if (!ms[k]) continue;
            ev[k] = eval_mate(ref(*ms[k]), p.asize);
            circ += ev[k].n_circ;
            lin += ev[k].n_lin;
            must |= ev[k].python_must_see;
        }
        const bool hand = must || ((circ || lin) && !(circ == 0 && p.nolinear));
        if (!hand) {
            for (int k = 0; k < 2; ++k) {
                if (!ms[k]) continue;
                if (ev[k].unspliced) C.unspliced_mates++;
                C.seg_too_short_skip += (uint64_t)ev[k].too_short;
            }
            return;
        }
        C.handed_back++;
        Batch::GFrag g;
        for (int k = 0; k < 2; ++k) {
            g.r0[k] = g.n[k] = g.p0[k] = g.np[k] = 0;
            g.seq_len[k] = 0;
            if (!ms[k]) continue;
            g.seq_len[k] = R[ms[k]->r[0]].seq_n;
            R[ms[k]->r[0]].decode();            // the primary's SEQ / QUAL, here rather than on the consumer's side
            g.r0[k] = (int32_t)b.gidx.size();
            g.n[k] = (int32_t)ms[k]->r.size();
            b.gidx.insert(b.gidx.end(), ms[k]->r.begin(), ms[k]->r.end());
            g.p0[k] = (int32_t)b.gidx.size();
            g.np[k] = (int32_t)ms[k]->p.size();
            b.gidx.insert(b.gidx.end(), ms[k]->p.begin(), ms[k]->p.end());
        }
        for (int k = 0; k < 2; ++k)
            if (g.np[k] >= 2) {
                span_cum += (uint64_t)(g.np[k] - 1);
                arena_cum += (uint64_t)(g.np[k] - 1) * g.seq_len[k];
            }
        g.span_cum = span_cum;
        g.arena_cum = arena_cum;
        g.must = must;
        g.cum = C;
        g.frags = F;
        b.gfrags.push_back(g);
    };
    C.records++;
    open(cur, s);
    for (size_t j = s + 1; j < n; ++j) {
        const Rec &r = R[j];
        if (r.unmapped()) {
            C.records++;
            C.unmapped_reads++;
            continue;
        }
        const Rec &prim = R[cur.r[0]];
        const bool same = r.qname == prim.qname;
        if (same && r.read1() == prim.read1()) {              // add_segment
            C.records++;
            const bool proper = r.tid == prim.tid && r.reverse() == prim.reverse();
            cur.r.push_back((int32_t)j);
            if (proper) cur.p.push_back((int32_t)cur.r.size() - 1);
        } else if (same) {                                    // the other mate
            C.records++;
            std::swap(oth, cur);
            have_oth = true;
            open(cur, j);
        } else {                                              // r closes the fragment
            close();
            Ct = C;                                           // the region ends before r ...
            Ft = F;
            t = j;
            C.records++;                                      // ... if no later record closes one
            have_oth = false;
            open(cur, j);
        }
    }
    if (t == s) {                                             // no fragment closed after gs's
        b.gfrags.clear();
        b.gidx.clear();
        return;
    }
    b.gs = (uint32_t)s;
    b.gt = (uint32_t)t;
    b.gtotal = Ct;
    b.gtotal_frags = Ft;
}

void add_counts(fc2_ingest_counts &c, const fc2_ingest_counts &to, const fc2_ingest_counts &from) {
    c.n_reads += to.n_reads - from.n_reads;
    c.total_mates += to.total_mates - from.total_mates;
    c.unmapped_reads += to.unmapped_reads - from.unmapped_reads;
    c.unspliced_mates += to.unspliced_mates - from.unspliced_mates;
    c.seg_too_short_skip += to.seg_too_short_skip - from.seg_too_short_skip;
    c.records += to.records - from.records;
    c.handed_back += to.handed_back - from.handed_back;
}

}  // namespace

extern "C" int fc2_ingest_open(const char *path, int is_bam, fc2_ingest **out) {
    // is_bam is the reference's mode hint ('rb' unless the name ends in "sam", find_circ.py:463-466);
    // like htslib's hts_open, reading never trusts it: the format comes from the bytes (the CLI logs a
    // warning when a BAM-named input holds SAM text)
    if (!path || !out) return fc2::fail(FC2_E_PARAM, "fc2_ingest_open: null argument");
    *out = nullptr;
    int fd = strcmp(path, "-") == 0 ? dup(0) : open(path, O_RDONLY);
    if (fd < 0) return fc2::fail(FC2_E_IO, std::string("cannot open '") + path + "': " + strerror(errno));
    fc2_ingest *h = new fc2_ingest();
    h->fd = fd;
    h->buf.resize(1 << 22);
    // 1. the byte source: peek one gzip header's worth (a pipe cannot be rewound, so the peeked
    //    bytes start the first BGZF batch, the zlib stream or the plain buffer)
    std::vector<uint8_t> pre(18);
    size_t got = 0;
    if (!read_full(fd, pre.data(), 18, got)) {
        const std::string e = std::string("read error: ") + strerror(errno);
        close(fd);
        delete h;
        return fc2::fail(FC2_E_IO, e);
    }
    pre.resize(got);
    if (got >= 2 && pre[0] == 0x1f && pre[1] == 0x8b) {
        if (got == 18 && bgzf_block_size(pre.data(), got) != 0) {
            // BGZF (BAM, or bgzip'ed SAM): blocks inflated in parallel, one batch ahead
            h->src = fc2_ingest::SRC_BGZF;
            h->bgzf = true;
            h->bgzf_nt = bgzf_threads();
            if (const char *e = getenv("FC2_BGZF_BATCH"))
                if (atoi(e) > 0) h->bgzf_blocks = std::min(atoi(e), 4096);
            h->bgzf_next = std::async(std::launch::async, bgzf_batch, fd, std::move(pre), std::min(16, h->bgzf_blocks),
                                      h->bgzf_nt, nullptr);
        } else {
            // any other gzip stream (gzip -c, concatenated members)
            h->src = fc2_ingest::SRC_GZIP;
            if (inflateInit2(&h->zs, 15 + 16) != Z_OK) { close(fd); delete h; return fc2::fail(FC2_E_IO, "zlib init"); }
            h->z_init = true;
            h->zin.assign(pre.begin(), pre.end());
            h->zs.next_in = (Bytef *)h->zin.data();
            h->zs.avail_in = (uInt)h->zin.size();
        }
    } else {
        h->src = fc2_ingest::SRC_RAW;
        memcpy(h->buf.data(), pre.data(), got);
        h->end = got;
    }
    // 2. the format, from the first (decompressed) bytes: BAM magic or SAM text
    ensure(h, 4);
    const size_t have = h->end - h->beg;
    const char *b = h->buf.data() + h->beg;
    int rc = FC2_OK;
    if (have >= 4 && memcmp(b, "BAM\1", 4) == 0) h->bam = true;
    else if (have >= 4 && memcmp(b, "CRAM", 4) == 0)
        rc = fc2::fail(FC2_E_FORMAT, std::string("'") + path + "' is CRAM, which this ingest does not read (convert "
                                     "it to BAM or SAM)");
    else if (h->in_rc || !h->z_err.empty()) rc = input_rc(h);
    if (!rc) rc = read_header(h);
    // pysam's Samfile(path, mode) checks the header (check_sq, on by default): an input that declares
    // no reference sequence -- an empty file, e.g. what a crashed aligner leaves as x.bam, or SAM text
    // without @SQ lines -- raises ValueError before the first record (find_circ.py:463-469)
    if (!rc && h->refs.empty())
        rc = fc2::fail(FC2_E_FORMAT, std::string("ValueError: file has no sequences defined (mode='") +
                                         (is_bam ? "rb" : "r") + "') - is it SAM/BAM format? Consider opening with "
                                         "check_sq=False");
    if (rc) { fc2_ingest_close(h); return rc; }
    *out = h;
    return FC2_OK;
}

extern "C" int fc2_ingest_format(const fc2_ingest *h, int *compression) {
    if (!h) return -1;
    if (compression)
        *compression = h->src == fc2_ingest::SRC_BGZF ? FC2_INGEST_BGZF
                     : h->src == fc2_ingest::SRC_GZIP ? FC2_INGEST_GZIP : FC2_INGEST_PLAIN;
    return h->bam ? FC2_INGEST_BAM : FC2_INGEST_SAM;
}

extern "C" int fc2_ingest_set_gpu_inflate_from(fc2_ingest *h, int device, uint64_t after_bytes) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_ingest_set_gpu_inflate: null argument");
    if (h->n_records) return fc2::fail(FC2_E_PARAM, "fc2_ingest_set_gpu_inflate: call before reading");
    const char *e = getenv("FC2_GPU_INFLATE");
    const bool wait = e && atoi(e) == 2;       // (2: the buffers made before the first read, as the tests want)
    if (e && (atoi(e) == 1 || wait)) after_bytes = 0;
    if (device < 0 || !h->bgzf || (e && atoi(e) == 0)) {
        h->gpu_inflate.reset();
        return FC2_OK;
    }
    auto gi = std::make_shared<GpuInflate>();
    gi->device = device;
    // batches of 1024 blocks (64 MiB inflated, four chunks of 256; fc2_inflate.hip) once the GPU
    // inflates; FC2_BGZF_BATCH still rules
    gi->max_blocks = getenv("FC2_BGZF_BATCH") ? (uint32_t)h->bgzf_blocks : 1024u;
    if (after_bytes == 0) {
        // the device's buffers and the first pinned batch buffers: now, or made while the first
        // batches are read and inflated on the CPU
        gi->launch(wait);
        if (wait) {
            auto r = gi->opening.get();
            gi->g = r.first;
            if (!gi->g) gi->failed = true, gi->err = r.second;
        }
    } else {
        gi->launched = false;
        gi->start_after = after_bytes;
    }
    h->gpu_inflate = gi;
    return FC2_OK;
}

extern "C" int fc2_ingest_set_gpu_inflate(fc2_ingest *h, int device, int wait) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_ingest_set_gpu_inflate: null argument");
    if (!wait) return fc2_ingest_set_gpu_inflate_from(h, device, 0);
    const char *e = getenv("FC2_GPU_INFLATE");
    if (e && atoi(e) == 0) return fc2_ingest_set_gpu_inflate_from(h, -1, 0);
    if (h->n_records) return fc2::fail(FC2_E_PARAM, "fc2_ingest_set_gpu_inflate: call before reading");
    if (device < 0 || !h->bgzf) {
        h->gpu_inflate.reset();
        return FC2_OK;
    }
    auto gi = std::make_shared<GpuInflate>();
    gi->device = device;
    gi->max_blocks = getenv("FC2_BGZF_BATCH") ? (uint32_t)h->bgzf_blocks : 1024u;
    gi->launch(true);
    auto r = gi->opening.get();
    gi->g = r.first;
    if (!gi->g) gi->failed = true, gi->err = r.second;
    h->gpu_inflate = gi;
    return FC2_OK;
}

extern "C" int fc2_ingest_inflate_counts(const fc2_ingest *h, uint64_t *gpu_blocks, uint64_t *cpu_blocks) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_ingest_inflate_counts: null argument");
    const GpuInflate *gi = h->gpu_inflate.get();
    if (gpu_blocks) *gpu_blocks = gi ? gi->gpu_blocks.load() : 0;
    if (cpu_blocks) *cpu_blocks = gi ? gi->cpu_blocks.load() : 0;
    return FC2_OK;
}

extern "C" int fc2_ingest_set_bam_out(fc2_ingest *h, const char *path) {
    if (!h || !path) return fc2::fail(FC2_E_PARAM, "fc2_ingest_set_bam_out: null argument");
    if (h->bam_out || h->n_records) return fc2::fail(FC2_E_PARAM, "fc2_ingest_set_bam_out: call once, before reading");
    std::string err;
    h->bam_out = fc2::bam::open_writer(path, h->header, h->refs, h->ref_len, err);
    return h->bam_out ? FC2_OK : fc2::fail(FC2_E_IO, err);
}

extern "C" int fc2_ingest_close_bam_out(fc2_ingest *h) {
    if (!h) return fc2::fail(FC2_E_PARAM, "fc2_ingest_close_bam_out: null argument");
    std::string err;
    const bool ok = fc2::bam::close_writer(h->bam_out, err);
    h->bam_out = nullptr;
    return ok ? FC2_OK : fc2::fail(FC2_E_IO, err);
}

fc2_ingest::~fc2_ingest() { ahead.reset(); }


extern "C" void fc2_ingest_close(fc2_ingest *h) {
    if (!h) return;
    h->ahead.reset();                  // stops the parse-ahead thread before the fd goes
    if (h->bam_out) {
        std::string err;
        fc2::bam::close_writer(h->bam_out, err);
    }
    if (h->bgzf_next.valid()) h->bgzf_next.wait();     // the batch reader uses the fd
    if (h->z_init) inflateEnd(&h->zs);
    if (h->fd >= 0) close(h->fd);
    delete h;
}

extern "C" int fc2_sam_to_bam(const char *sam_path, const char *bam_path) {
    if (!sam_path || !bam_path) return fc2::fail(FC2_E_PARAM, "fc2_sam_to_bam: null argument");
    fc2_ingest *h = nullptr;
    if (int rc = fc2_ingest_open(sam_path, 0, &h)) return rc;
    int rc = FC2_OK;
    if (h->bam) rc = fc2::fail(FC2_E_FORMAT, std::string("fc2_sam_to_bam: '") + sam_path + "' is BAM already");
    std::string err;
    fc2::bam::Writer *w = rc ? nullptr : fc2::bam::open_writer(bam_path, h->header, h->refs, h->ref_len, err, 1);
    if (!rc && !w) rc = fc2::fail(FC2_E_IO, err);
    // lines gathered into batches of ~32 MiB of text, each batch encoded on T threads (contiguous line
    // ranges) and its records written with fc2::bam::write_bulk (blocks deflated on T threads): the file
    // is byte for byte what encoding and writing record by record gives
    int T = (int)std::thread::hardware_concurrency();
    if (const char *env = getenv("OMP_NUM_THREADS")) if (atoi(env) > 0) T = atoi(env);
    T = std::max(1, std::min(T, 32));
    std::string text;
    std::vector<std::pair<size_t, size_t>> lines;        // (offset, length) in text
    auto process = [&]() -> int {
        const size_t nl = lines.size();
        if (!nl) return FC2_OK;
        const int P = (int)std::max<size_t>(1, std::min<size_t>((size_t)T, nl / 1024));
        std::vector<std::string> part((size_t)P), perr((size_t)P);
        std::vector<char> bad((size_t)P, 0);
        std::vector<std::thread> pool;
        auto enc = [&](int r) {
            for (size_t i = nl * (size_t)r / (size_t)P, e = nl * (size_t)(r + 1) / (size_t)P; i < e; ++i) {
                const char *a = text.data() + lines[i].first;
                if (!fc2::bam::encode_sam(a, a + lines[i].second, h->tid_of, part[(size_t)r], perr[(size_t)r])) {
                    bad[(size_t)r] = 1;
                    return;
                }
            }
        };
        for (int r = 1; r < P; ++r) pool.emplace_back(enc, r);
        enc(0);
        for (auto &th : pool) th.join();
        std::string all;                                 // records up to the first failing line
        int r = 0;
        for (; r < P; ++r) {
            all += part[(size_t)r];
            if (bad[(size_t)r]) break;
        }
        if (!fc2::bam::write_bulk(w, all.data(), all.size(), T)) return fc2::fail(FC2_E_IO, "fc2_sam_to_bam: write failed");
        if (r < P) return fc2::fail(FC2_E_FORMAT, perr[(size_t)r]);
        text.clear();
        lines.clear();
        return FC2_OK;
    };
    const char *ls, *le;
    while (!rc && next_line_view(h, ls, le)) {
        bool blank = true;
        for (const char *c = ls; c < le; ++c) if (!isspace((unsigned char)*c)) { blank = false; break; }
        if (blank) continue;
        lines.emplace_back(text.size(), (size_t)(le - ls));
        text.append(ls, le);
        if (text.size() >= ((size_t)32 << 20)) rc = process();
    }
    if (!rc) rc = process();
    if (!rc) rc = input_rc(h);
    if (w && !fc2::bam::close_writer(w, err) && !rc) rc = fc2::fail(FC2_E_IO, err);
    fc2_ingest_close(h);
    return rc;
}

extern "C" int fc2_ingest_n_refs(const fc2_ingest *h) { return h ? (int)h->refs.size() : 0; }
extern "C" const char *fc2_ingest_ref_name(const fc2_ingest *h, int tid) {
    return (h && tid >= 0 && tid < (int)h->refs.size()) ? h->refs[tid].c_str() : nullptr;
}
extern "C" const char *fc2_ingest_header(const fc2_ingest *h) { return h ? h->header.c_str() : ""; }

namespace {
int run_loop(fc2_ingest *h, const fc2_ingest_params *p, uint64_t max_frags, const fc2::ing::FragSink *sink,
             uint64_t *n_handed, int *eof, const fc2::ing::BulkSink *bulk = nullptr) {
    uint64_t handed = 0, frags = 0;
    int rc = FC2_OK;
    bool done = h->finished;
    while (!done && frags < max_frags) {
        if (sink && h->ahead && h->ahead->pin && h->ahead->pinned.size() >= h->ahead->max_pinned)
            break;                              // the chunk ends here (fc2::ing::pin_full)
        // a batch's region grouped on its parse thread (group_batch): its first record closes the
        // current fragment; then the region's handed fragments go to the sink, and its last
        // record opens the fragment the loop goes on with
        if (h->ahead && sink && h->ahead->cur && h->ahead->cur->gt > h->ahead->cur->gs &&
            h->ahead->pos == h->ahead->cur->gs) {
            auto &A = *h->ahead;
            auto &b = *A.cur;
            if (!A.in_region) {
                rc = emit_or_count(h, p, handed, sink);
                ++frags;
                h->have_other = false;
                recycle(h, h->other);
                A.in_region = true;
                A.gnext = 0;
                A.gapplied = fc2_ingest_counts{};
                A.gapplied_frags = 0;
                if (rc) return rc;
                continue;
            }
            if (bulk && A.pin && A.gnext < b.gfrags.size() && frags < max_frags) {
                // a run of the listed fragments at once: as many as the loop below would hand
                // before `frags` reaches max_frags
                const size_t g0 = A.gnext;
                size_t k = g0 + 1;
                while (k < b.gfrags.size() && frags + (b.gfrags[k - 1].frags - A.gapplied_frags) < max_frags) ++k;
                const auto &g = b.gfrags[k - 1];
                add_counts(h->counts, g.cum, A.gapplied);
                h->n_records += g.cum.records - A.gapplied.records;
                frags += g.frags - A.gapplied_frags;
                A.gapplied = g.cum;
                A.gapplied_frags = g.frags;
                handed += k - g0;
                A.grouped += k - g0;
                A.gnext = k;
                fc2::ing::RegionRef rr;
                rr.recs = b.recs.data();
                rr.g = b.gfrags.data() + g0;
                rr.n = k - g0;
                rr.gidx = b.gidx.data();
                rr.span_before = g0 ? b.gfrags[g0 - 1].span_cum : 0;
                rr.arena_before = g0 ? b.gfrags[g0 - 1].arena_cum : 0;
                rc = (*bulk)(rr);
                if (rc) return rc;
            }
            while (A.gnext < b.gfrags.size() && frags < max_frags) {
                const auto &g = b.gfrags[A.gnext++];
                add_counts(h->counts, g.cum, A.gapplied);
                h->n_records += g.cum.records - A.gapplied.records;
                frags += g.frags - A.gapplied_frags;
                A.gapplied = g.cum;
                A.gapplied_frags = g.frags;
                ++handed;
                ++A.grouped;
                MateRef m[2];
                for (int k = 0; k < 2; ++k) {
                    m[k].base = b.recs.data();
                    m[k].idx = b.gidx.data() + g.r0[k];
                    m[k].n = (uint32_t)g.n[k];
                    m[k].proper = b.gidx.data() + g.p0[k];
                    m[k].np = (uint32_t)g.np[k];
                    m[k].seq_len = g.seq_len[k];
                    m[k].stable = A.pin;
                }
                rc = (*sink)(g.n[0] ? &m[0] : nullptr, &m[1], g.must);
                if (rc) return rc;
            }
            if (A.gnext < b.gfrags.size()) continue;          // stopped at max_frags: resumed here
            add_counts(h->counts, b.gtotal, A.gapplied);
            h->n_records += b.gtotal.records - A.gapplied.records;
            frags += b.gtotal_frags - A.gapplied_frags;
            A.in_region = false;
            Rec &rt = b.recs[b.gt];                            // opens the next fragment
            A.pos = (size_t)b.gt + 1;
            h->n_records++;
            h->counts.records++;
            open_mate(h, h->current, rt);
            continue;
        }
        // the next record: in its parse batch, or parsed here into the scratch record
        Rec *rp = nullptr;
        rc = FC2_OK;
        if (h->ahead) rp = next_ahead(h, rc);
        else if (next_record(h, h->scratch, rc)) rp = &h->scratch;
        if (!rp) {
            if (rc) return rc;
            // end of input: the final yield (:1486)
            if (h->started) {
                if (h->n_records == 1)
                    return fc2::fail(FC2_E_FORMAT, "UnboundLocalError: local variable 'line_num' referenced before "
                                                   "assignment (single-record input, find_circ.py:1486)");
                rc = emit_or_count(h, p, handed, sink);
                ++frags;
            }
            h->finished = done = true;
            if (rc) return rc;
            break;
        }
        h->n_records++;
        h->counts.records++;
        Rec &r = *rp;
        if (!h->started) {           // first record always opens a mate (:1462-1463)
            open_mate(h, h->current, r);
            h->started = true;
            continue;
        }
        if (r.unmapped()) { h->counts.unmapped_reads++; continue; }   // r is reused
        const Rec &prim = h->current.recs[0];
        if (r.read1() == prim.read1() && r.qname == prim.qname) {
            add_segment(h->current, r);
        } else if (r.read1() != prim.read1() && r.qname == prim.qname) {
            std::swap(h->other, h->current);
            h->have_other = true;
            open_mate(h, h->current, r);
        } else {
            rc = emit_or_count(h, p, handed, sink);
            ++frags;
            h->have_other = false;
            recycle(h, h->other);
            open_mate(h, h->current, r);
            if (rc) return rc;
        }
    }
    if (n_handed) *n_handed = handed;
    if (eof) *eof = done ? 1 : 0;
    return FC2_OK;
}
}  // namespace

int fc2::ing::pull(fc2_ingest *h, const fc2_ingest_params *p, uint64_t max_frags, const FragSink &sink, int *eof,
                   const BulkSink *bulk) {
    if (!h || !p) return fc2::fail(FC2_E_PARAM, "ingest pull: null argument");
    if (h->need_text) h->need_text = false;     // (written once: the parse thread reads it)
    // plain SAM text and BAM (any compression): parsed on threads of their own; compressed SAM stays
    // on the sequential reader, and so does everything when -B writes records while reading
    if (!h->ahead && (h->bam || h->src == fc2_ingest::SRC_RAW) && !h->bam_out && !h->finished) {
        fc2_ingest::SamAhead *ap = new fc2_ingest::SamAhead();
        h->ahead.reset(ap);
        if (const char *be = getenv("FC2_PARSE_BLOCK"))
            if (atol(be) > 0) ap->block = (size_t)atol(be);
        if (const char *pm = getenv("FC2_PIN_MAX"))
            if (atoi(pm) > 0) ap->max_pinned = (size_t)atoi(pm);
        if (const char *fe = getenv("FC2_PARSE_INFLIGHT"))
            if (atoi(fe) > 0) ap->max_inflight = (size_t)std::min(atoi(fe), 256);
        // BGZF BAM is cut into parse blocks in place in the inflated batches; plain and other gzip BAM
        // through the copying splitter
        ap->splitter = !h->bam                          ? std::thread(sam_split_loop, h, ap)
                       : h->src == fc2_ingest::SRC_BGZF ? std::thread(bgzf_split_loop, h, ap)
                                                        : std::thread(bam_split_loop, h, ap);
        const char *env = getenv("FC2_PARSE_THREADS");
        const int np = env && atoi(env) > 0 ? std::min(atoi(env), 32) : fc2_ingest::SamAhead::kParsers;
        // fragments grouped on the parse threads (the consumer groups those a parse block cuts)
        ap->gp = *p;
        ap->group = true;
        ap->pin = h->pin;
        for (int k = 0; k < np; ++k) ap->parsers.emplace_back(sam_parse_loop, h, ap);
    }
    return run_loop(h, p, max_frags, &sink, nullptr, eof, bulk);
}

bool fc2::ing::writes_records(const fc2_ingest *h) { return h && h->bam_out != nullptr; }

void fc2::ing::set_pin(fc2_ingest *h, bool on) {
    if (!h) return;
    h->pin = on;
    if (h->ahead) h->ahead->pin = on;
    if (!on) release(h);
}

bool fc2::ing::pin_full(const fc2_ingest *h) {
    return h && h->ahead && h->ahead->pin && h->ahead->pinned.size() >= h->ahead->max_pinned;
}

void fc2::ing::release(fc2_ingest *h) {
    if (!h || !h->ahead || h->ahead->pinned.empty()) return;
    auto &A = *h->ahead;
    {
        std::lock_guard<std::mutex> lk(A.m);
        for (auto &b : A.pinned) A.spare.push_back(std::move(b));
    }
    A.pinned.clear();
    A.cv.notify_all();
}

void fc2::ing::take_stage_ms(fc2_ingest *h, double *inflate_wait, double *split_block, double *parse_idle) {
    *inflate_wait = *split_block = *parse_idle = 0;
    if (!h) return;
    *inflate_wait = (double)h->inflate_wait_ns.exchange(0) * 1e-6;
    if (!h->ahead) return;
    *split_block = (double)h->ahead->split_block_ns.exchange(0) * 1e-6;
    *parse_idle = (double)h->ahead->parse_idle_ns.exchange(0) * 1e-6;
}

double fc2::ing::take_wait_ms(fc2_ingest *h, uint64_t *grouped) {
    if (grouped) *grouped = 0;
    if (!h || !h->ahead) return 0;
    const double w = h->ahead->wait_ms;
    h->ahead->wait_ms = 0;
    if (grouped) *grouped = h->ahead->grouped;
    h->ahead->grouped = 0;
    return w;
}

extern "C" int fc2_ingest_next(fc2_ingest *h, const fc2_ingest_params *p, uint64_t max_frags,
                               fc2_ingest_counts *counts, const char **text, uint64_t *text_len, uint64_t *n_handed,
                               int *eof) {
    if (!h || !p) return fc2::fail(FC2_E_PARAM, "fc2_ingest_next: null argument");
    if (h->deferred_rc) {
        const int code = h->deferred_rc;
        h->deferred_rc = FC2_OK;
        return fc2::fail(code, h->deferred_msg);
    }
    h->out.clear();
    const int rc = run_loop(h, p, max_frags, nullptr, n_handed, eof);
    if (rc) {
        if (h->out.empty()) return rc;
        h->deferred_rc = rc;                   // hand out the fragments before it first
        h->deferred_msg = fc2_last_error();
        if (eof) *eof = 0;
    }
    if (counts) *counts = h->counts;
    if (text) *text = h->out.c_str();
    if (text_len) *text_len = h->out.size();
    return FC2_OK;
}

extern "C" int fc2_ingest_counts_get(const fc2_ingest *h, fc2_ingest_counts *counts) {
    if (!h || !counts) return fc2::fail(FC2_E_PARAM, "fc2_ingest_counts_get: null argument");
    *counts = h->counts;
    return FC2_OK;
}
