// fc2_host.cpp -- host side of libfc2.so: FASTA access with the reference's
// indexed_fasta semantics, genome/pair packing into the device layout, and the
// byte-exact arena for rare pairs.  No GPU calls here.
//
// Reference: find_circ.py:103-215 (indexed_fasta), 821-852 (JunctionSpan),
// 854-974 (find_breakpoints).
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "fc2_common.h"
#include "fc2_compact.h"
#include "fc2_hostmem.h"

namespace fc2 {

static thread_local std::string g_err;

void set_error(const std::string &msg) { g_err = msg; }
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int validate_params(const fc2_params *p) {
    if (!p) return fail(FC2_E_PARAM, "null fc2_params");
    // asize <= margin is legal: eff_a <= 0 turns read[eff_a:-eff_a] (find_circ.py:895) into a short or
    // empty slice, and fc2_pack_pairs sends every pair to the byte-exact path, which follows the
    // reference's string / numpy semantics for it
    if ((int64_t)p->asize - p->margin < -65536)
        return fail(FC2_E_RANGE, "asize - margin < -65536 is not supported (windows of over 128k bases per pair)");
    if (p->margin > 255) return fail(FC2_E_RANGE, "margin > 255 is not supported (ov is stored in 8 bits)");
    return FC2_OK;
}

static int n_workers(int n_threads) {
    if (n_threads > 0) return n_threads;
    unsigned h = std::thread::hardware_concurrency();
    const char *env = getenv("OMP_NUM_THREADS");
    if (env && atoi(env) > 0) h = (unsigned)atoi(env);
    if (h == 0) h = 1;
    if (h > 64) h = 64;
    return (int)h;
}

// Run body(begin, end) over [0, n) split into contiguous chunks on `threads` threads.
static void parallel_for(uint64_t n, int threads, const std::function<void(uint64_t, uint64_t)> &body) {
    if (n == 0) return;
    if (threads <= 1 || n < 4096) {
        body(0, n);
        return;
    }
    uint64_t t = (uint64_t)threads;
    if (t > n) t = n;
    std::vector<std::thread> pool;
    pool.reserve(t);
    for (uint64_t k = 0; k < t; ++k) {
        const uint64_t b = n * k / t, e = n * (k + 1) / t;
        pool.emplace_back([&body, b, e] { body(b, e); });
    }
    for (auto &th : pool) th.join();
}

static inline uint8_t upc(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

// base class of an (uppercased) byte: 0..3 = ACGT, 4 = N, 5 = other
static inline int bclass(uint8_t c) {
    switch (upc(c)) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        case 'N': return 4;
        default: return 5;
    }
}

// pack code of a byte: bits 0-1 = ACGT code, bit 2 = N plane (N or exotic), bit 3 = exotic
struct PackTable {
    uint8_t t[256];
    PackTable() {
        for (int c = 0; c < 256; ++c) {
            const int cl = bclass((uint8_t)c);
            t[c] = (uint8_t)(cl < 4 ? cl : cl == 4 ? 4 : 4 | 8);
        }
    }
};
static const PackTable kPackTable;
static inline uint32_t pack_code(uint8_t c) { return kPackTable.t[c]; }

// The bases of up to 64 FASTA bytes as bit masks (bit j = byte j): a/c/g/t/n = the byte upper-cased
// is that letter (the reference's .upper(), find_circ.py:901-902, on the 2-bit pack's classes).
struct BaseMasks {
    uint64_t a, c, g, t, n, nl;                 // nl: '\n' (a line break inside a row: irregular layout)
};

static inline BaseMasks base_masks_scalar(const uint8_t *s, int len) {
    BaseMasks m{0, 0, 0, 0, 0, 0};
    for (int j = 0; j < len; ++j) {
        const uint64_t bit = 1ull << j;
        if (s[j] == '\n') m.nl |= bit;
        switch (s[j] & 0xDF) {
            case 'A': m.a |= bit; break;
            case 'C': m.c |= bit; break;
            case 'G': m.g |= bit; break;
            case 'T': m.t |= bit; break;
            case 'N': m.n |= bit; break;
            default: break;
        }
    }
    return m;
}

// 64 bytes at s (all readable): one compare per letter per 32 bytes.  (b & 0xDF) == 'A' holds for
// 'A' and 'a' only, as upc() + bclass() classify.
__attribute__((target("avx2"))) static BaseMasks base_masks_avx2(const uint8_t *s) {
    const __m256i up = _mm256_set1_epi8((char)0xDF);
    const __m256i r0 = _mm256_loadu_si256((const __m256i *)s), r1 = _mm256_loadu_si256((const __m256i *)(s + 32));
    const __m256i v0 = _mm256_and_si256(r0, up), v1 = _mm256_and_si256(r1, up);
#define FC2_MASK64(x0, x1, ch)                                                                             \
    ((uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(x0, _mm256_set1_epi8(ch))) |                 \
     (uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(x1, _mm256_set1_epi8(ch))) << 32)
    const BaseMasks m{FC2_MASK64(v0, v1, 'A'), FC2_MASK64(v0, v1, 'C'), FC2_MASK64(v0, v1, 'G'),
                      FC2_MASK64(v0, v1, 'T'), FC2_MASK64(v0, v1, 'N'), FC2_MASK64(r0, r1, '\n')};
#undef FC2_MASK64
    return m;
}

#if defined(__HIP_DEVICE_COMPILE__)
static const bool kHaveAvx2 = false;           // (hipcc's device pass over this host-only file)
#else
static const bool kHaveAvx2 = (__builtin_cpu_init(), __builtin_cpu_supports("avx2"));
#endif

// every byte of u (already upper-cased with & 0xDF) is one of 'A' 'C' 'G' 'T' (exact zero-byte tests)
static inline bool acgt8(uint64_t u) {
    auto zero = [](uint64_t y) { return ~(((y & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | y | 0x7F7F7F7F7F7F7F7Full); };
    const uint64_t m = zero(u ^ 0x4141414141414141ull) | zero(u ^ 0x4343434343434343ull) |
                       zero(u ^ 0x4747474747474747ull) | zero(u ^ 0x5454545454545454ull);
    return m == 0x8080808080808080ull;
}

static inline bool py_isspace(uint8_t c) {
    return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
}

}  // namespace fc2

using namespace fc2;

struct fc2_chrom_rec {
    std::string name;
    int64_t ofs = 0, ldata = 0, skip = 0, size = 0;
    std::string skipchar;
    int nfields = 4;   // the reference's chrom_stats list length (5 when complete)
    int regular = -1;  // -1 unknown until packed
    uint64_t gstart = 0;
};

struct fc2_fasta {
    std::string path;
    int fd = -1;
    const uint8_t *data = nullptr;
    size_t n = 0;
    std::vector<fc2_chrom_rec> chroms;
    std::unordered_map<std::string, int> by_name;
    std::vector<uint64_t> exotic;  // sorted global positions of non-ACGTN bases
    bool packed = false;
    // the planes fc2_fasta_prepack made, until a context's fc2_ctx_genome_load takes them
    struct Prepacked {
        fc2::MappedWords units, nplane;
        std::vector<uint32_t> ncoarse;
        uint64_t n_units = 0;
    };
    std::unique_ptr<Prepacked> prepacked;
};

// ---------------------------------------------------------------------------
// index (find_circ.py:120-155) and .byo_index (157-187)
// ---------------------------------------------------------------------------
static int build_index(fc2_fasta *f) {
    std::unordered_map<std::string, int> &idx = f->by_name;
    std::vector<fc2_chrom_rec> &cs = f->chroms;
    int64_t ofs = 0, chrom_ofs = 0, size = 0;
    std::string chrom = "undef";
    const uint8_t *d = f->data;
    const size_t n = f->n;
    size_t i = 0;
    while (i < n) {
        const uint8_t *nl = (const uint8_t *)memchr(d + i, '\n', n - i);
        const size_t j = nl ? (size_t)(nl - d) + 1 : n;
        const uint8_t *line = d + i;
        const int64_t len = (int64_t)(j - i);
        ofs += len;
        if (line[0] == '>') {
            if (size) {  // self.chrom_stats[chrom].append(size)
                auto it = idx.find(chrom);
                if (it == idx.end())
                    return fail(FC2_E_FORMAT, "FASTA header without sequence before '" + chrom +
                                                  "': reference indexed_fasta.index raises KeyError");
                cs[it->second].size = size;
                cs[it->second].nfields += 1;
            }
            int64_t s = 1;
            while (s < len && py_isspace(line[s])) ++s;
            int64_t e = s;
            while (e < len && !py_isspace(line[e])) ++e;
            if (e == s) return fail(FC2_E_FORMAT, "empty FASTA header: reference raises IndexError");
            chrom.assign((const char *)line + s, (size_t)(e - s));
            chrom_ofs = ofs;
        } else {
            int64_t a = 0, b = len;
            while (a < b && py_isspace(line[a])) ++a;
            while (b > a && py_isspace(line[b - 1])) --b;
            const int64_t stripped = b - a;
            if (idx.find(chrom) == idx.end()) {
                size = 0;
                fc2_chrom_rec r;
                r.name = chrom;
                r.ofs = chrom_ofs;
                r.ldata = stripped;
                r.skip = len - stripped;
                r.skipchar.assign((const char *)line + stripped, (size_t)(len - stripped));
                idx[chrom] = (int)cs.size();
                cs.push_back(r);
            }
            size += stripped;
        }
        i = j;
    }
    if (size) {
        auto it = idx.find(chrom);
        if (it != idx.end()) {
            cs[it->second].size = size;
            cs[it->second].nfields += 1;
        }
    }
    for (auto &c : cs)
        if (c.nfields != 5)
            return fail(FC2_E_FORMAT, "chromosome '" + c.name +
                                          "' has an inconsistent index entry (empty or duplicated sequence); "
                                          "the reference's store_index/get_data fail on it");
    return FC2_OK;
}

static std::string py2_repr(const std::string &s) {
    std::string o = "'";
    for (unsigned char c : s) {
        if (c == '\n') o += "\\n";
        else if (c == '\r') o += "\\r";
        else if (c == '\t') o += "\\t";
        else if (c == '\'') o += "\\'";
        else if (c == '\\') o += "\\\\";
        else if (c >= 32 && c < 127) o += (char)c;
        else {
            char buf[8];
            snprintf(buf, sizeof buf, "\\x%02x", c);
            o += buf;
        }
    }
    return o + "'";
}

static bool py2_unescape(const std::string &in, std::string &out) {  // 'string_escape' for repr output
    out.clear();
    for (size_t i = 0; i < in.size(); ++i) {
        char c = in[i];
        if (c != '\\') { out += c; continue; }
        if (++i >= in.size()) return false;
        switch (in[i]) {
            case 'n': out += '\n'; break;
            case 'r': out += '\r'; break;
            case 't': out += '\t'; break;
            case '\\': out += '\\'; break;
            case '\'': out += '\''; break;
            case '"': out += '"'; break;
            case 'x': {
                if (i + 2 >= in.size()) return false;
                out += (char)strtol(in.substr(i + 1, 2).c_str(), nullptr, 16);
                i += 2;
                break;
            }
            default: out += '\\'; out += in[i];
        }
    }
    return true;
}

static int load_index_file(fc2_fasta *f, const std::string &ipath) {
    FILE *fp = fopen(ipath.c_str(), "r");
    if (!fp) return fail(FC2_E_IO, "cannot open index: IOError: [Errno " + std::to_string(errno) + "] " +
                                       strerror(errno) + ": '" + ipath + "'");   // file(ipath), find_circ.py:185
    char *line = nullptr;
    size_t cap = 0;
    ssize_t len;
    int rc = FC2_OK;
    while ((len = getline(&line, &cap, fp)) > 0) {
        std::string s(line, (size_t)len);
        while (!s.empty() && py_isspace((uint8_t)s.back())) s.pop_back();  // rstrip()
        std::vector<std::string> parts;
        size_t st = 0;
        for (;;) {
            size_t t = s.find('\t', st);
            parts.push_back(s.substr(st, t == std::string::npos ? std::string::npos : t - st));
            if (t == std::string::npos) break;
            st = t + 1;
        }
        if (parts.size() != 6 || parts[4].size() < 2) { rc = fail(FC2_E_FORMAT, "malformed .byo_index line: " + s); break; }
        fc2_chrom_rec r;
        r.name = parts[0];
        r.ofs = atoll(parts[1].c_str());
        r.ldata = atoll(parts[2].c_str());
        r.skip = atoll(parts[3].c_str());
        if (!py2_unescape(parts[4].substr(1, parts[4].size() - 2), r.skipchar)) { rc = fail(FC2_E_FORMAT, "bad skipchar in .byo_index"); break; }
        r.size = atoll(parts[5].c_str());
        r.nfields = 5;
        f->by_name[r.name] = (int)f->chroms.size();
        f->chroms.push_back(r);
    }
    free(line);
    fclose(fp);
    // the file lists chromosomes by name; keep FASTA order so that chromosome indices (and
    // everything laid out by them) do not depend on whether an index file existed
    std::stable_sort(f->chroms.begin(), f->chroms.end(),
                     [](const fc2_chrom_rec &a, const fc2_chrom_rec &b) { return a.ofs < b.ofs; });
    f->by_name.clear();
    for (size_t i = 0; i < f->chroms.size(); ++i) f->by_name[f->chroms[i].name] = (int)i;
    return rc;
}

// find_circ.py:157-179: temp file in the index's directory, fsync, chmod 0444, rename.  Every step is
// an os-level call whose failure raises OSError in Python 2 (tempfile's os.open, os.fsync, os.chmod,
// os.rename), which GenomeAccessor does not catch (:340 catches IOError only): FC2_E_OS.
static int store_index_file(const fc2_fasta *f, const std::string &ipath) {
    std::vector<const fc2_chrom_rec *> v;
    for (auto &c : f->chroms) v.push_back(&c);
    std::sort(v.begin(), v.end(), [](const fc2_chrom_rec *a, const fc2_chrom_rec *b) { return a->name < b->name; });
    std::string dir = ipath.substr(0, ipath.find_last_of('/') == std::string::npos ? 0 : ipath.find_last_of('/') + 1);
    std::string tmpl = (dir.empty() ? std::string("./") : dir) + "tmpXXXXXX";
    std::vector<char> buf(tmpl.begin(), tmpl.end());
    buf.push_back(0);
    auto oserror = [&](int err, const char *what) {
        return fail(FC2_E_OS, std::string("OSError: [Errno ") + std::to_string(err) + "] " + strerror(err) + ": '" +
                                  what + "' (writing the FASTA index " + ipath + ")");
    };
    int fd = mkstemp(buf.data());
    if (fd < 0) return oserror(errno, tmpl.c_str());
    std::string body;
    for (auto *c : v) {
        char num[128];
        body += c->name;
        snprintf(num, sizeof num, "\t%lld\t%lld\t%lld\t", (long long)c->ofs, (long long)c->ldata, (long long)c->skip);
        body += num;
        body += py2_repr(c->skipchar);
        snprintf(num, sizeof num, "\t%lld\n", (long long)c->size);
        body += num;
    }
    size_t done = 0;
    while (done < body.size()) {
        const ssize_t w = write(fd, body.data() + done, body.size() - done);
        if (w < 0) {
            if (errno == EINTR) continue;
            const int err = errno;
            close(fd);
            unlink(buf.data());
            return oserror(err, buf.data());
        }
        done += (size_t)w;
    }
    if (fsync(fd) != 0) { const int err = errno; close(fd); unlink(buf.data()); return oserror(err, buf.data()); }
    close(fd);
    if (chmod(buf.data(), S_IRUSR | S_IRGRP | S_IROTH) != 0) { const int err = errno; unlink(buf.data()); return oserror(err, buf.data()); }
    if (rename(buf.data(), ipath.c_str()) != 0) { const int err = errno; unlink(buf.data()); return oserror(err, buf.data()); }
    return FC2_OK;
}

// ---------------------------------------------------------------------------
// get_data(...).upper()  (find_circ.py:189-215, 901-902), Python slice semantics
// ---------------------------------------------------------------------------
static inline int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}
static inline int64_t pyclip(int64_t i, int64_t n) {
    if (i < 0) { i += n; if (i < 0) i = 0; }
    return i > n ? n : i;
}

// get_data(...).upper() of [start, end) (find_circ.py:189-215); at most `limit` bytes of it when the
// caller only needs to know that a window is longer than that (a window far outside its chromosome
// is padded with 'N' to its full, possibly huge, length by the reference)
static int get_upper_impl(const fc2_fasta *f, int ci, int64_t start, int64_t end, std::string &out,
                          size_t limit = SIZE_MAX, int64_t *full_len = nullptr, int tail_char = -1,
                          int64_t *tail_mis = nullptr) {
    // full_len: the window's untruncated length; tail_mis: how many of its bytes past `limit` differ
    // from tail_char (upper-cased) -- a one-base internal part broadcast over the window needs them
    out.clear();
    if (tail_mis) *tail_mis = 0;
    if (!f) {  // GenomeAccessor.get_dummy (find_circ.py:370-371)
        if (end > start) out.assign(std::min((size_t)(end - start), limit), 'N');
        const int64_t full = end > start ? end - start : 0;
        if (full_len) *full_len = full;
        if (tail_mis && tail_char != 'N' && full > (int64_t)limit) *tail_mis = full - (int64_t)limit;
        return FC2_OK;
    }
    if (ci < 0 || ci >= (int)f->chroms.size()) return fail(FC2_E_KEY, "unknown chromosome index");
    const fc2_chrom_rec &c = f->chroms[ci];
    if (c.ldata == 0) return fail(FC2_E_FORMAT, "chromosome '" + c.name + "' has ldata 0: reference raises ZeroDivisionError");
    int64_t pad_start = 0, pad_end = 0;
    if (start < 0) { pad_start = -start; start = 0; }
    if (end > c.size) { pad_end = end - c.size; end = c.size; }
    const int64_t os = pyclip(floordiv(start, c.ldata) * c.skip + start + c.ofs, (int64_t)f->n);
    const int64_t oe = pyclip(floordiv(end, c.ldata) * c.skip + end + c.ofs, (int64_t)f->n);
    const uint64_t full = (uint64_t)pad_start + (uint64_t)pad_end + (uint64_t)(oe > os ? oe - os : 0);
    if (limit == SIZE_MAX && full > (1ull << 32))   // an inconsistent index entry (e.g. a negative size)
        return fail(FC2_E_RANGE, "window of " + std::to_string(full) + " bytes from chromosome '" + c.name +
                                     "': the reference's get_data raises MemoryError");
    out.reserve(std::min((size_t)full, limit));
    out.append(std::min((size_t)pad_start, limit), 'N');
    const size_t sl = c.skipchar.size();
    for (int64_t p = os; p < oe && out.size() < limit;) {
        if (sl && p + (int64_t)sl <= oe && !memcmp(f->data + p, c.skipchar.data(), sl)) { p += (int64_t)sl; continue; }
        out.push_back((char)upc(f->data[p]));
        ++p;
    }
    out.append(std::min((size_t)pad_end, limit - out.size()), 'N');
    if (full_len || tail_mis) {   // the slice's bytes after skip_char removal + the pads
        const int64_t lim = limit == SIZE_MAX ? INT64_MAX : (int64_t)limit;
        int64_t k = pad_start, mis = 0;
        const bool n_differs = tail_char != 'N';
        if (n_differs && pad_start > lim) mis += pad_start - lim;
        for (int64_t p = os; p < oe;) {
            if (sl && p + (int64_t)sl <= oe && !memcmp(f->data + p, c.skipchar.data(), sl)) { p += (int64_t)sl; continue; }
            if (k >= lim && (int)upc(f->data[p]) != tail_char) ++mis;
            ++k;
            ++p;
        }
        if (n_differs) mis += std::max<int64_t>(0, k + pad_end - std::max(k, lim));
        if (full_len) *full_len = k + pad_end;
        if (tail_mis) *tail_mis = mis;
    }
    return FC2_OK;
}

// ---------------------------------------------------------------------------
// C ABI: library info
// ---------------------------------------------------------------------------
extern "C" int fc2_abi_version(void) { return FC2_ABI_VERSION; }
extern "C" const char *fc2_last_error(void) { return g_err.c_str(); }
extern "C" int fc2_max_fast_l(void) { return kMaxFastL; }

extern "C" int fc2_batch_geometry(const fc2_params *p, int32_t max_read_len, uint32_t *rw, uint32_t *nw, uint32_t *tw) {
    int rc = validate_params(p);
    if (rc) return rc;
    int lmax = max_read_len - 2 * eff_anchor(p);
    if (lmax < 0) lmax = 0;
    const int lfast = lmax > kMaxFastL ? kMaxFastL : lmax;
    if (rw) *rw = (uint32_t)std::max(1, (2 * lfast + 63) / 64);
    if (nw) *nw = (uint32_t)std::max(1, (lfast + 63) / 64);
    // the register kernels write (l + 2 + 63) / 64 tie words per strand (fc2_bp_scan_launch checks it)
    if (tw) *tw = (uint32_t)(2 * std::max(1, (lmax + 2 + 63) / 64));
    return FC2_OK;
}

// ---------------------------------------------------------------------------
// C ABI: FASTA
// ---------------------------------------------------------------------------
extern "C" int fc2_fasta_open(const char *path, int write_index, fc2_fasta **out) {
    if (!path || !out) return fail(FC2_E_PARAM, "fc2_fasta_open: null argument");
    *out = nullptr;
    // FC2_E_IO exactly where indexed_fasta() raises IOError (file(fname), find_circ.py:117/124; file(ipath),
    // :185), which GenomeAccessor turns into its all-N dummy mode (:338-345); a failure the reference does
    // not catch there (mmap.error, :118) is FC2_E_OS, a malformed index FC2_E_FORMAT.
    auto ioerror = [&](int err) {
        return fail(FC2_E_IO, std::string("cannot open FASTA: IOError: [Errno ") + std::to_string(err) + "] " +
                                  strerror(err) + ": '" + path + "'");
    };
    int fd = open(path, O_RDONLY);
    if (fd < 0) return ioerror(errno);
    struct stat st;
    if (fstat(fd, &st) != 0) { const int err = errno; close(fd); return ioerror(err); }
    if (S_ISDIR(st.st_mode)) { close(fd); return ioerror(EISDIR); }   // Python 2's file(<directory>)
    fc2_fasta *f = new fc2_fasta();
    f->path = path;
    f->fd = fd;
    f->n = (size_t)st.st_size;
    if (f->n) {
        void *m = mmap(nullptr, f->n, PROT_READ, MAP_SHARED, fd, 0);
        if (m == MAP_FAILED) {
            const int err = errno;
            close(fd);
            delete f;
            return fail(FC2_E_OS, std::string("mmap.error: [Errno ") + std::to_string(err) + "] " + strerror(err) +
                                      " (FASTA '" + path + "')");
        }
        f->data = (const uint8_t *)m;
        madvise(m, f->n, MADV_WILLNEED);
    }
    const std::string ipath = std::string(path) + ".byo_index";
    int rc;
    if (access(ipath.c_str(), R_OK) == 0) {       // find_circ.py:110-112
        rc = load_index_file(f, ipath);
    } else {
        rc = build_index(f);                       // find_circ.py:114-115
        if (rc == FC2_OK && write_index) rc = store_index_file(f, ipath);
    }
    if (rc != FC2_OK) { fc2_fasta_close(f); return rc; }
    *out = f;
    return FC2_OK;
}

extern "C" void fc2_fasta_close(fc2_fasta *f) {
    if (!f) return;
    if (f->data) munmap((void *)f->data, f->n);
    if (f->fd >= 0) close(f->fd);
    delete f;
}

extern "C" int fc2_fasta_n_chrom(const fc2_fasta *f) { return f ? (int)f->chroms.size() : 0; }

extern "C" int fc2_fasta_chrom(const fc2_fasta *f, int i, const char **name, int64_t *size, int64_t *ofs, int64_t *ldata,
                               int64_t *skip, int *regular) {
    if (!f || i < 0 || i >= (int)f->chroms.size()) return fail(FC2_E_PARAM, "fc2_fasta_chrom: bad index");
    const fc2_chrom_rec &c = f->chroms[i];
    if (name) *name = c.name.c_str();
    if (size) *size = c.size;
    if (ofs) *ofs = c.ofs;
    if (ldata) *ldata = c.ldata;
    if (skip) *skip = c.skip;
    if (regular) *regular = c.regular;
    return FC2_OK;
}

extern "C" int fc2_fasta_find(const fc2_fasta *f, const char *name) {
    if (!f || !name) return -1;
    auto it = f->by_name.find(name);
    return it == f->by_name.end() ? -1 : it->second;
}

extern "C" int fc2_fasta_get_upper(const fc2_fasta *f, int chrom, int64_t start, int64_t end, uint8_t *out, int64_t cap,
                                   int64_t *len) {
    std::string s;
    int rc = get_upper_impl(f, chrom, start, end, s);
    if (rc) return rc;
    if (len) *len = (int64_t)s.size();
    if (out && cap > 0) memcpy(out, s.data(), (size_t)std::min<int64_t>(cap, (int64_t)s.size()));
    return FC2_OK;
}

// Unit-aligned genome coordinates of every chromosome; false when the sizes (a damaged .byo_index)
// add up to more than 2^40 bases, which no device table is laid out for.
static bool compute_layout(fc2_fasta *f, uint64_t *n_units) {
    constexpr uint64_t kMaxBases = 1ull << 40;
    uint64_t g = 0;
    for (auto &c : f->chroms) {
        c.gstart = g;
        const uint64_t sz = (uint64_t)std::max<int64_t>(c.size, 0);
        if (sz > kMaxBases || g + sz > kMaxBases) return false;
        g += (sz + 63) & ~63ull;
    }
    *n_units = std::max<uint64_t>(1, g / 64);
    return true;
}

extern "C" int fc2_fasta_layout(const fc2_fasta *cf, uint64_t *n_units, uint64_t *n_coarse_words, uint64_t *chrom_start) {
    if (!cf) return fail(FC2_E_PARAM, "fc2_fasta_layout: null");
    fc2_fasta *f = const_cast<fc2_fasta *>(cf);
    uint64_t nu;
    if (!compute_layout(f, &nu))
        return fail(FC2_E_RANGE, "fc2_fasta_layout: chromosome sizes add up to more than 2^40 bases (a damaged index?)");
    if (n_units) *n_units = nu;
    if (n_coarse_words) *n_coarse_words = (((nu + 15) >> 4) + 31) >> 5;
    if (chrom_start)
        for (size_t i = 0; i < f->chroms.size(); ++i) chrom_start[i] = f->chroms[i].gstart;
    return FC2_OK;
}

// Is the chromosome laid out exactly as the index arithmetic assumes?  Then
// get_data's slice-and-strip yields base p at file offset ofs + (p//ldata)*skip + p.
// The layout checks of a chromosome that need no pass over its bases: its rows (ldata bytes each, then
// the separator skipchar, find_circ.py:204-209) lie inside the file and the separator is whitespace.
// The per-row part -- no '\n' inside a row, the separator present after each full row -- is checked
// by the pack's pass itself (fc2_fasta_pack); a chromosome failing either is irregular: stored as N,
// its pairs restated on the byte path (get_data's string slicing).
static bool chrom_rows_in_file(const fc2_fasta *f, const fc2_chrom_rec &c) {
    if (c.size <= 0) return true;
    if (c.ldata <= 0) return false;
    if ((int64_t)c.skipchar.size() != c.skip) return false;
    // an index entry (.byo_index) that points outside the file: get_data's Python slices clip or wrap
    // there, which only the byte path restates; the pack's pass then never leaves [0, n]
    const int64_t n = (int64_t)f->n;
    if (c.ofs < 0 || c.ofs > n || c.ldata > n || c.size > n) return false;
    for (char ch : c.skipchar)
        if (!py_isspace((uint8_t)ch)) return false;
    const int64_t nfull = c.size / c.ldata, rem = c.size % c.ldata;
    int64_t stride, last;                        // the end of the last row
    if (__builtin_add_overflow(c.ldata, c.skip, &stride) ||
        __builtin_mul_overflow(rem ? nfull : nfull - 1, stride, &last) ||
        __builtin_add_overflow(last, c.ofs + (rem ? rem : c.ldata), &last))
        return false;
    return last <= n;
}

extern "C" int fc2_fasta_pack(const fc2_fasta *cf, uint64_t *units, uint64_t *nplane, uint32_t *ncoarse,
                              uint64_t *n_exotic, int n_threads) {
    if (!cf || !units || !nplane || !ncoarse) return fail(FC2_E_PARAM, "fc2_fasta_pack: null argument");
    fc2_fasta *f = const_cast<fc2_fasta *>(cf);
    uint64_t nu;
    if (!compute_layout(f, &nu))
        return fail(FC2_E_RANGE, "fc2_fasta_pack: chromosome sizes add up to more than 2^40 bases (a damaged index?)");
    const int T = n_workers(n_threads);
    static const bool timing = getenv("FC2_CALLER_TIMING") != nullptr;      // phase times on stderr
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    // the layout checks that need no pass over the bases; the rest is checked while packing
    // (into a local array, published once at the end: a repack -- every device after the first --
    // never shows a row-broken chromosome as regular to a concurrent fc2_pack_pairs, even briefly)
    std::vector<uint8_t> regular(f->chroms.size());
    for (size_t c = 0; c < f->chroms.size(); ++c) regular[c] = chrom_rows_in_file(f, f->chroms[c]) ? 1 : 0;
    std::unique_ptr<std::atomic<uint8_t>[]> broken(new std::atomic<uint8_t>[std::max<size_t>(1, f->chroms.size())]);
    for (size_t c = 0; c < f->chroms.size(); ++c) broken[c].store(0, std::memory_order_relaxed);
    const double t_regular = ms();
    // work items: (chrom, unit range) of <= 2^14 units
    struct Item { int c; uint64_t u0, u1; };
    std::vector<Item> items;
    for (int c = 0; c < (int)f->chroms.size(); ++c) {
        const fc2_chrom_rec &r = f->chroms[c];
        const uint64_t cu = ((uint64_t)std::max<int64_t>(r.size, 0) + 63) / 64;
        for (uint64_t u = 0; u < cu; u += 16384) items.push_back({c, u, std::min(cu, u + 16384)});
    }
    // every unit belongs to one chromosome (they are laid out back to back, compute_layout) and is
    // written once below -- a regular chromosome's from the FASTA, an irregular one's as all-N; only
    // the single unit of a genome without bases is padding
    uint64_t covered = 0;
    for (const fc2_chrom_rec &r : f->chroms) covered += ((uint64_t)std::max<int64_t>(r.size, 0) + 63) / 64;
    for (uint64_t u = covered; u < nu; ++u) { units[2 * u] = 0; units[2 * u + 1] = 0; nplane[u] = ~0ull; }
    std::vector<std::vector<uint64_t>> exo(items.size());
    std::atomic<size_t> next{0};
    std::vector<std::thread> pool;
    for (int t = 0; t < std::max(1, std::min<int>(T, (int)items.size())); ++t)
        pool.emplace_back([&] {
            for (size_t k; (k = next.fetch_add(1)) < items.size();) {
                const Item it = items[k];
                const fc2_chrom_rec &r = f->chroms[it.c];
                const uint64_t gu0 = r.gstart / 64;
                if (regular[(size_t)it.c] != 1) {   // all N; pairs on it take the byte path
                    for (uint64_t u = it.u0; u < it.u1; ++u) {
                        units[2 * (gu0 + u)] = 0;
                        units[2 * (gu0 + u) + 1] = 0;
                        nplane[gu0 + u] = ~0ull;
                    }
                    continue;
                }
                // the item's bases in segments that stay inside one line and one unit: each segment's
                // class masks (64-byte vector compares where 64 bytes are mapped, else byte by byte)
                // shifted into the unit's planes; a unit is written once, when full or at the end
                const int64_t ld = r.ldata;
                int64_t p = (int64_t)it.u0 * 64;
                const int64_t pend = std::min<int64_t>((int64_t)it.u1 * 64, r.size);
                int64_t col = p % ld;
                const uint8_t *src = f->data + r.ofs + (p / ld) * (ld + r.skip) + col;
                const uint8_t *const fend = f->data + f->n;
                uint64_t u = gu0 + it.u0, lo = 0, hi = 0, nn = 0;
                int b = 0;
                bool bad = false;
                while (p < pend) {
                    const int seg = (int)std::min<int64_t>(std::min<int64_t>(ld - col, pend - p), 64 - b);
                    const BaseMasks m = (kHaveAvx2 && fend - src >= 64) ? base_masks_avx2(src) : base_masks_scalar(src, seg);
                    const uint64_t keep = seg == 64 ? ~0ull : (1ull << seg) - 1;
                    bad |= (m.nl & keep) != 0;
                    const uint64_t acgt = m.a | m.c | m.g | m.t;
                    lo |= ((m.c | m.t) & keep) << b;
                    hi |= ((m.g | m.t) & keep) << b;
                    nn |= (~acgt & keep) << b;
                    for (uint64_t ex = ~(acgt | m.n) & keep; ex; ex &= ex - 1)   // rare: not ACGTN
                        exo[k].push_back(r.gstart + (uint64_t)p + (uint64_t)__builtin_ctzll(ex));
                    b += seg;
                    p += seg;
                    src += seg;
                    col += seg;
                    if (col == ld) {
                        // the separator after a full row; the last row may end the file without it
                        const int64_t te = src - f->data;
                        const bool sep = te + r.skip <= (int64_t)f->n &&
                                         memcmp(src, r.skipchar.data(), (size_t)r.skip) == 0;
                        bad |= !(sep || (p == r.size && te == (int64_t)f->n));
                        col = 0;
                        src += r.skip;
                    }
                    if (b == 64 || p == pend) {
                        if (b < 64) nn |= ~0ull << b;      // past the chromosome's end
                        units[2 * u] = lo;
                        units[2 * u + 1] = hi;
                        nplane[u] = nn;
                        ++u;
                        lo = hi = nn = 0;
                        b = 0;
                    }
                }
                if (bad) broken[it.c].store(1, std::memory_order_relaxed);
            }
        });
    for (auto &th : pool) th.join();
    // chromosomes whose rows turned out irregular: all N, no exotic positions (as if known up front)
    for (size_t k = 0; k < items.size(); ++k) {
        const Item it = items[k];
        if (!broken[it.c].load(std::memory_order_relaxed)) continue;
        regular[(size_t)it.c] = 0;
        const uint64_t gu0 = f->chroms[it.c].gstart / 64;
        for (uint64_t u = it.u0; u < it.u1; ++u) {
            units[2 * (gu0 + u)] = 0;
            units[2 * (gu0 + u) + 1] = 0;
            nplane[gu0 + u] = ~0ull;
        }
        exo[k].clear();
    }
    for (size_t c = 0; c < f->chroms.size(); ++c) f->chroms[c].regular = regular[c];
    const double t_planes = ms();
    f->exotic.clear();
    for (auto &v : exo) f->exotic.insert(f->exotic.end(), v.begin(), v.end());
    // irregular chromosomes: every base is "exotic" for routing purposes (handled by chrom flag)
    const uint64_t n_blocks = (nu + 15) >> 4, n_words = (n_blocks + 31) >> 5;
    parallel_for(n_words, T, [&](uint64_t b, uint64_t e) {
        for (uint64_t w = b; w < e; ++w) {
            uint32_t bits = 0;
            for (int k = 0; k < 32; ++k) {
                const uint64_t blk = w * 32 + k;
                if (blk >= n_blocks) break;
                uint64_t acc = 0;
                for (int j = 0; j < 16; ++j) {
                    const uint64_t u = blk * 16 + j;
                    if (u < nu) acc |= nplane[u];
                }
                if (acc) bits |= 1u << k;
            }
            ncoarse[w] = bits;
        }
    });
    if (n_exotic) *n_exotic = f->exotic.size();
    if (timing)
        fprintf(stderr, "fasta pack: layout check %.1f ms, planes + row check %.1f ms, coarse N map %.1f ms (%d threads)\n", t_regular,
                t_planes - t_regular, ms() - t_planes, T);
    f->packed = true;
    return FC2_OK;
}

extern "C" int fc2_fasta_prepack(fc2_fasta *f, int n_threads) {
    if (!f) return fail(FC2_E_PARAM, "fc2_fasta_prepack: null");
    uint64_t nu = 0, ncw = 0;
    if (int rc = fc2_fasta_layout(f, &nu, &ncw, nullptr)) return rc;
    std::unique_ptr<fc2_fasta::Prepacked> pp(new fc2_fasta::Prepacked);
    pp->units = fc2::MappedWords(2 * nu);
    pp->nplane = fc2::MappedWords(nu);
    if (!pp->units.ok() || !pp->nplane.ok())
        return fail(FC2_E_OS, "fc2_fasta_prepack: cannot map host memory for the 2-bit genome");
    pp->ncoarse.assign((size_t)std::max<uint64_t>(ncw, 1), 0);
    uint64_t n_exotic = 0;
    if (int rc = fc2_fasta_pack(f, pp->units.data(), pp->nplane.data(), pp->ncoarse.data(), &n_exotic, n_threads)) return rc;
    pp->n_units = nu;
    f->prepacked = std::move(pp);
    return FC2_OK;
}

bool fc2::take_prepacked(const fc2_fasta *cf, uint64_t n_units, MappedWords &units, MappedWords &nplane,
                         std::vector<uint32_t> &ncoarse) {
    fc2_fasta *f = const_cast<fc2_fasta *>(cf);
    if (!f || !f->prepacked || f->prepacked->n_units != n_units) return false;
    units = std::move(f->prepacked->units);
    nplane = std::move(f->prepacked->nplane);
    ncoarse.swap(f->prepacked->ncoarse);
    f->prepacked.reset();
    return true;
}

// ---------------------------------------------------------------------------
// C ABI: pair packing
// ---------------------------------------------------------------------------
static bool touches_exotic(const fc2_fasta *f, uint64_t g0, uint64_t g1) {
    if (f->exotic.empty() || g1 <= g0) return false;
    auto it = std::lower_bound(f->exotic.begin(), f->exotic.end(), g0);
    return it != f->exotic.end() && *it < g1;
}

extern "C" int fc2_pack_pairs(const fc2_params *p, const fc2_fasta *f, uint64_t n, const uint8_t *reads,
                              const uint64_t *read_off, fc2_pair *pairs, uint64_t *read_words, uint32_t rw,
                              uint64_t *read_nwords, uint32_t nw, uint64_t stride, uint64_t *n_bytepath,
                              int n_threads) {
    int rc = validate_params(p);
    if (rc) return rc;
    if (n && (!reads || !read_off || !pairs || !read_words || !read_nwords)) return fail(FC2_E_PARAM, "fc2_pack_pairs: null argument");
    if (stride < n) return fail(FC2_E_PARAM, "fc2_pack_pairs: stride < n");
    if (f && !f->packed) return fail(FC2_E_PARAM, "fc2_pack_pairs: genome must be packed first (fc2_fasta_pack)");
    const int e = eff_anchor(p);
    const int T = n_workers(n_threads);
    std::atomic<uint64_t> nbp{0};
    std::atomic<int64_t> bad_chrom{-1}, bad_rows{-1}, bad_dist{-1}, bad_len{-1};
    const int nch = f ? (int)f->chroms.size() : 0;
    const int maxdist = p->maxdist;
    parallel_for(n, T, [&](uint64_t b, uint64_t en) {
        uint64_t local_bp = 0;
        constexpr int kW = (kMaxFastL + 63) / 64;
        for (uint64_t i = b; i < en; ++i) {
            fc2_pair &pr = pairs[i];
            uint8_t flags = (uint8_t)(pr.flags & (FC2_PAIR_BACKSPLICE | FC2_PAIR_PRIMARY_REV | FC2_PAIR_SKIP));
            uint8_t npos = 0;
            // the pair's row words, built in registers and stored once at the end (zero unless packed)
            uint64_t row[2 * kW + 1] = {0}, nrow[kW] = {0};
            const int L = pr.read_len;
            const int l = L - 2 * e;
            bool bytepath = false;
            do {
                if (flags & FC2_PAIR_SKIP) break;
                if (L > FC2_MAX_READ_LEN) { int64_t x = -1; bad_len.compare_exchange_strong(x, (int64_t)i); break; }
                if (f && (int)pr.chrom >= nch) { int64_t x = -1; bad_chrom.compare_exchange_strong(x, (int64_t)i); break; }
                if (l < 0) break;  // range(l+1) is empty: no hit, no window use
                if (maxdist > 255 && l > 255) { int64_t x = -1; bad_dist.compare_exchange_strong(x, (int64_t)i); }
                if (e <= 0) { bytepath = true; break; }   // read[e:-e] is not the read's middle (fc2_bytepath_fill)
                if (l > kMaxFastL) { bytepath = true; break; }
                if ((uint64_t)2 * l > (uint64_t)rw * 64 || (uint64_t)l > (uint64_t)nw * 64) {
                    int64_t x = -1; bad_rows.compare_exchange_strong(x, (int64_t)i); break;
                }
                const uint8_t *I = reads + read_off[i] + e;
                // tight bit-sliced row: low code bits at [0, l), high bits at [l, 2l), 'N' = code 00 +
                // an N bit.  Fast path: 8 bases per step (SWAR) while every byte is one of ACGTacgt
                // (code = ((c >> 2) ^ (c >> 1)) & 3: A0 C1 G2 T3 either case); anything else (N, IUPAC,
                // other bytes) takes the per-byte table for the rest of the read.
                uint64_t lo_w[kW] = {0}, hi_w[kW] = {0}, n_w[kW] = {0};
                uint32_t any = 0;
                int j = 0;
                for (; j + 8 <= l; j += 8) {
                    uint64_t x;
                    memcpy(&x, I + j, 8);
                    const uint64_t u = x & 0xDFDFDFDFDFDFDFDFull;            // upper case
                    if (!acgt8(u)) break;
                    const uint64_t v = ((x >> 2) ^ (x >> 1)) & 0x0303030303030303ull;
                    const uint64_t lo8 = ((v & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56;
                    const uint64_t hi8 = (((v >> 1) & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56;
                    lo_w[j >> 6] |= lo8 << (j & 63);
                    hi_w[j >> 6] |= hi8 << (j & 63);
                }
                for (; j < l; ++j) {
                    const uint32_t pc = pack_code(I[j]);
                    const uint64_t bit = 1ull << (j & 63);
                    if (pc & 4u) n_w[j >> 6] |= bit;                        // 'N' (or exotic)
                    else {
                        if (pc & 1u) lo_w[j >> 6] |= bit;
                        if (pc & 2u) hi_w[j >> 6] |= bit;
                    }
                    any |= pc;
                }
                if (any & 8u) { bytepath = true; break; }
                const int nlw = (l + 63) / 64;
                for (int k = 0; k < nlw; ++k) row[k] = lo_w[k];
                const int sh = l & 63, wo = l >> 6;
                for (int k = 0; k < nlw; ++k) {
                    row[wo + k] |= sh ? (hi_w[k] << sh) : hi_w[k];
                    if (sh) row[wo + k + 1] |= hi_w[k] >> (64 - sh);
                }
                if (any & 4u) {
                    int n_count = 0, n_first = 0;
                    for (int k = 0; k < nlw; ++k) {
                        nrow[k] = n_w[k];
                        if (n_w[k]) {
                            if (n_count == 0) n_first = k * 64 + __builtin_ctzll(n_w[k]);
                            n_count += __builtin_popcountll(n_w[k]);
                        }
                    }
                    flags |= FC2_PAIR_READ_N;
                    if (n_count == 1 && n_first < 256) {      // the scan takes it from the record
                        flags |= FC2_PAIR_READ_N1;
                        npos = (uint8_t)n_first;
                    }
                }
                if (f) {
                    const fc2_chrom_rec &c = f->chroms[pr.chrom];
                    const int64_t W = l + 2;
                    const int64_t wsA = (int64_t)pr.a_pos + e, wsB = (int64_t)pr.b_aend - e - W;
                    if (c.regular != 1) bytepath = true;
                    else if (wsA > c.size || wsA + W < 0 || wsB > c.size || wsB + W < 0) bytepath = true;
                    else {
                        auto clampg = [&](int64_t s) { return (uint64_t)std::min<int64_t>(std::max<int64_t>(s, 0), c.size) + c.gstart; };
                        if (touches_exotic(f, clampg(wsA), clampg(wsA + W)) || touches_exotic(f, clampg(wsB), clampg(wsB + W)))
                            bytepath = true;
                    }
                }
            } while (false);
            if (bytepath) {
                flags = (uint8_t)((flags & ~(FC2_PAIR_READ_N | FC2_PAIR_READ_N1)) | FC2_PAIR_BYTEPATH);
                npos = 0;
                for (auto &w : row) w = 0;
                for (auto &w : nrow) w = 0;
                ++local_bp;
            }
            pr.flags = flags;
            pr.npos = npos;
            for (uint32_t j = 0; j < rw; ++j) read_words[(uint64_t)j * stride + i] = j < 2 * kW + 1 ? row[j] : 0;
            for (uint32_t j = 0; j < nw; ++j) read_nwords[(uint64_t)j * stride + i] = j < kW ? nrow[j] : 0;
        }
        nbp += local_bp;
    });
    if (bad_chrom.load() >= 0)
        return fail(FC2_E_KEY, "pair " + std::to_string(bad_chrom.load()) +
                                   ": chromosome not in the genome index (reference KeyError, find_circ.py:193)");
    if (bad_len.load() >= 0)
        return fail(FC2_E_RANGE, "pair " + std::to_string(bad_len.load()) + ": read_part longer than " +
                                     std::to_string(FC2_MAX_READ_LEN) + " bases (fc2_result.best_x is 16-bit)");
    if (bad_rows.load() >= 0) return fail(FC2_E_PARAM, "pair " + std::to_string(bad_rows.load()) + ": read rows too narrow");
    if (bad_dist.load() >= 0) return fail(FC2_E_RANGE, "maxdist > 255 with reads whose l > 255 is not supported");
    if (n_bytepath) *n_bytepath = nbp.load();
    return FC2_OK;
}

extern "C" int fc2_window_geometry(const fc2_params *p, int max_read_len, uint32_t *pw, uint32_t *ww,
                                   uint32_t *wnw) {
    int rc = validate_params(p);
    if (rc) return rc;
    if (!pw || !ww || !wnw) return fail(FC2_E_PARAM, "fc2_window_geometry: null argument");
    const int l = std::max(0, max_read_len - 2 * eff_anchor(p));
    if (l + 2 > 128) return fail(FC2_E_RANGE, "fc2_window_geometry: window rows carry l + 2 <= 128 only");
    *pw = (uint32_t)((l + 2 + 31) / 32);
    *ww = 2 * *pw;
    *wnw = *pw;
    return FC2_OK;
}

// Af / Bf of each evaluated pair from the FASTA text with get_data's semantics (the same bytes the
// byte-exact kernel gets), encoded as the rows fc2_batch_view.win_words describes.
extern "C" int fc2_pack_windows(const fc2_params *p, const fc2_fasta *f, uint64_t n, fc2_pair *pairs,
                                uint64_t *win_words, uint64_t *win_nwords, uint32_t pw, uint64_t stride,
                                int n_threads) {
    int rc = validate_params(p);
    if (rc) return rc;
    if (n && (!f || !pairs || !win_words || !win_nwords)) return fail(FC2_E_PARAM, "fc2_pack_windows: null argument");
    if (pw < 1 || pw > 4) return fail(FC2_E_RANGE, "fc2_pack_windows: pw is 1..4");
    if (stride < n) return fail(FC2_E_PARAM, "fc2_pack_windows: stride < n");
    const int e = eff_anchor(p);
    const int nch = (int)f->chroms.size();
    std::atomic<int> err{0};
    parallel_for(n, n_workers(n_threads), [&](uint64_t b, uint64_t en) {
        std::string A, B;
        for (uint64_t i = b; i < en; ++i) {
            fc2_pair &pr = pairs[i];
            uint32_t w32[16] = {0}, n32[8] = {0};
            bool anyN = false;
            const int l = (int)pr.read_len - 2 * e;
            const int W = l + 2;
            if (!(pr.flags & (FC2_PAIR_SKIP | FC2_PAIR_BYTEPATH)) && l >= 0 && W <= 32 * (int)pw &&
                (int)pr.chrom < nch) {
                const int r1 = get_upper_impl(f, (int)pr.chrom, (int64_t)pr.a_pos + e, (int64_t)pr.a_pos + e + W, A,
                                              (size_t)W + 1);
                const int r2 = get_upper_impl(f, (int)pr.chrom, (int64_t)pr.b_aend - e - W, (int64_t)pr.b_aend - e, B,
                                              (size_t)W + 1);
                if (r1 || r2) { err = r1 ? r1 : r2; continue; }
                const std::string *win[2] = {&A, &B};
                for (int x = 0; x < 2; ++x) {
                    const std::string &S = *win[x];
                    // windows of unexpected length lie outside get_data's range: the scan reports them
                    // (FC2_RES_ERR_WIN) from the coordinates, whatever the rows hold
                    const int m = std::min<int>(W, (int)S.size());
                    for (int j = 0; j < m; ++j) {
                        const uint32_t pc = pack_code((uint8_t)S[j]);
                        const int k = j >> 5, bit = j & 31;
                        if (pc & 12u) {                 // 'N' (or an exotic byte: such pairs are BYTEPATH)
                            n32[x * pw + k] |= 1u << bit;
                            anyN = true;
                            continue;
                        }
                        if (pc & 1u) w32[(2 * x) * pw + k] |= 1u << bit;
                        if (pc & 2u) w32[(2 * x + 1) * pw + k] |= 1u << bit;
                    }
                }
            }
            for (uint32_t j = 0; j < 2 * pw; ++j)
                win_words[(uint64_t)j * stride + i] = (uint64_t)w32[2 * j] | ((uint64_t)w32[2 * j + 1] << 32);
            for (uint32_t j = 0; j < pw; ++j)
                win_nwords[(uint64_t)j * stride + i] = (uint64_t)n32[2 * j] | ((uint64_t)n32[2 * j + 1] << 32);
            pr.flags = (uint8_t)((pr.flags & ~FC2_PAIR_WIN_N) | (anyN ? FC2_PAIR_WIN_N : 0u));
        }
    });
    if (err.load()) return err.load();
    return FC2_OK;
}

// 16-B header + I + A's slot of l+3 bytes + B's slot of 2l+3 bytes (fc2_bytes_view): an irregular
// window pair -- A cut short past the chromosome's end, B padded long before its start -- compares
// B[x+2 : x+2+lenI-lenA] (find_circ.py:907-908), which reaches byte 2l+2 of B
static inline uint64_t block_bytes(int64_t l) {
    const uint64_t lc = (uint64_t)std::max<int64_t>(0, l);
    return (16 + lc + (lc + 3) + (2 * lc + 3) + 3) & ~3ull;
}

// One pair's block of the byte arena at blk: the read part's internal bytes and both windows
// (A, B: scratch strings).  L = len(read_part), e = the effective anchor.
static int fill_block(const fc2_fasta *f, int e, int64_t L, uint32_t chrom, int64_t a_pos, int64_t b_aend,
                      const uint8_t *read, uint8_t *blk, std::string &A, std::string &B) {
    const int64_t l = L - 2 * (int64_t)e;
    // internal = read[e:-e] with Python's slice rules (find_circ.py:895): the read's middle l bases
    // for e > 0; for e <= 0 read[e:-e] is '' (e == 0) or read[max(L+e, 0) : min(-e, L)]
    int64_t i0 = e, i1 = L - e;
    if (e <= 0) { i0 = std::max<int64_t>(L + e, 0); i1 = e == 0 ? 0 : std::min<int64_t>(-e, L); }
    const int32_t lenI = l < 0 ? 0 : (int32_t)std::max<int64_t>(0, i1 - i0);
    int64_t fullA = 0, fullB = 0, tailB = 0;
    A.clear(); B.clear();
    if (l >= 0) {
        const int64_t flank = l + 2;
        // only min(length, slot) bytes of a window are stored (slots of l + 3 and 2l + 3 bytes); the
        // header keeps the full length and, for a one-base internal part, the mismatches of B's bytes
        // past its slot against that base
        const int c1 = lenI == 1 ? (int)upc(read[i0]) : -1;
        int rc = get_upper_impl(f, (int)chrom, a_pos + e, a_pos + e + flank, A, (size_t)flank + 1, &fullA);
        if (rc) return rc;
        rc = get_upper_impl(f, (int)chrom, b_aend - e - flank, b_aend - e, B, (size_t)(2 * flank - 1), &fullB, c1,
                            lenI == 1 ? &tailB : nullptr);
        if (rc) return rc;
    }
    // a window of unexpected length (outside get_data's defined range) keeps its slot's bytes: the
    // kernel compares what the reference's string form reads of them (at most B[:2l+3] when the
    // lengths add up), sees a length mismatch numpy cannot broadcast (ERR_WIN) or, where numpy
    // broadcasts a 1-byte operand, counts B's bytes past the slot through tailB (bp_bytes_kernel)
    const int32_t lenA = (int32_t)std::min<int64_t>(fullA, INT32_MAX);
    const int32_t lenB = (int32_t)std::min<int64_t>(fullB, INT32_MAX);
    const int32_t tail = (int32_t)std::min<int64_t>(tailB, INT32_MAX);
    memcpy(blk, &lenI, 4);
    memcpy(blk + 4, &lenA, 4);
    memcpy(blk + 8, &lenB, 4);
    memcpy(blk + 12, &tail, 4);
    uint8_t *q = blk + 16;
    for (int64_t j = 0; j < lenI; ++j) q[j] = upc(read[i0 + j]);
    q += lenI;
    const uint64_t lc = (uint64_t)std::max<int64_t>(0, l);
    memcpy(q, A.data(), std::min<size_t>(A.size(), lc + 3));
    q += lc + 3;
    memcpy(q, B.data(), std::min<size_t>(B.size(), 2 * lc + 3));
    return FC2_OK;
}

extern "C" int fc2_bytepath_size(const fc2_params *p, uint64_t n, const fc2_pair *pairs, uint64_t *m, uint64_t *arena_bytes) {
    int rc = validate_params(p);
    if (rc) return rc;
    const int e = eff_anchor(p);
    uint64_t mm = 0, bytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (!(pairs[i].flags & FC2_PAIR_BYTEPATH)) continue;
        bytes += block_bytes((int64_t)pairs[i].read_len - 2 * e);
        ++mm;
    }
    if (m) *m = mm;
    if (arena_bytes) *arena_bytes = bytes;
    return FC2_OK;
}

extern "C" int fc2_bytepath_fill(const fc2_params *p, const fc2_fasta *f, uint64_t n, const uint8_t *reads,
                                 const uint64_t *read_off, const fc2_pair *pairs, uint64_t *index, fc2_pair *bpairs,
                                 uint64_t *off, uint8_t *arena) {
    int rc = validate_params(p);
    if (rc) return rc;
    const int e = eff_anchor(p);
    uint64_t k = 0, pos = 0;
    std::string A, B;
    for (uint64_t i = 0; i < n; ++i) {
        const fc2_pair &pr = pairs[i];
        if (!(pr.flags & FC2_PAIR_BYTEPATH)) continue;
        if ((rc = fill_block(f, e, pr.read_len, pr.chrom, pr.a_pos, pr.b_aend, reads + read_off[i], arena + pos, A, B)))
            return rc;
        index[k] = i;
        bpairs[k] = pr;
        off[k] = pos;
        pos += block_bytes((int64_t)pr.read_len - 2 * e);
        ++k;
    }
    return FC2_OK;
}

// ---- long pairs (include/fc2_bp.h fc2_long_pair) ------------------------------------------------
extern "C" int fc2_long_geometry(const fc2_params *p, uint64_t n, const fc2_long_pair *pairs, uint64_t *arena_bytes,
                                 uint64_t *tie_off) {
    int rc = validate_params(p);
    if (rc) return rc;
    if (n && !pairs) return fail(FC2_E_PARAM, "fc2_long_geometry: null pairs");
    const int e = eff_anchor(p);
    uint64_t bytes = 0, words = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const int64_t l = (int64_t)pairs[i].read_len - 2 * e;
        bytes += block_bytes(l);
        if (tie_off) tie_off[i] = words;
        words += 2 * (uint64_t)((std::max<int64_t>(l, 0) + 2 + 63) / 64);   // x in [0, l] per strand
    }
    if (tie_off) tie_off[n] = words;
    if (arena_bytes) *arena_bytes = bytes;
    return FC2_OK;
}

extern "C" int fc2_long_fill(const fc2_params *p, const fc2_fasta *f, uint64_t n, const uint8_t *reads,
                             const fc2_long_pair *pairs, uint64_t *off, uint8_t *arena) {
    int rc = validate_params(p);
    if (rc) return rc;
    if (n && (!reads || !pairs || !off || !arena)) return fail(FC2_E_PARAM, "fc2_long_fill: null argument");
    const int e = eff_anchor(p);
    const int nch = f ? (int)f->chroms.size() : 0;
    uint64_t pos = 0;
    std::string A, B;
    for (uint64_t i = 0; i < n; ++i) {
        const fc2_long_pair &pr = pairs[i];
        if (pr.read_len > (uint32_t)INT32_MAX) return fail(FC2_E_RANGE, "fc2_long_fill: read part of 2^31 bases or more");
        off[i] = pos;
        const int64_t l = (int64_t)pr.read_len - 2 * e;
        if (!(pr.flags & FC2_PAIR_SKIP)) {
            if (f && (int)pr.chrom >= nch)
                return fail(FC2_E_KEY, "long pair " + std::to_string(i) +
                                           ": chromosome not in the genome index (reference KeyError, find_circ.py:193)");
            if ((rc = fill_block(f, e, pr.read_len, pr.chrom, pr.a_pos, pr.b_aend, reads + pr.read_off, arena + pos, A, B)))
                return rc;
        } else {
            memset(arena + pos, 0, 16);
        }
        pos += block_bytes(l);
    }
    return FC2_OK;
}

// ---- compact results (include/fc2_bp.h) --------------------------------------------------------
extern "C" int fc2_result_expand(const fc2_params *p, const void *words, int width, uint64_t n,
                                 const fc2_result_escape *esc, uint64_t n_esc, fc2_result *out, int n_threads) {
    if (int rc = fc2::validate_params(p)) return rc;
    if (p->noncanonical) return fc2::fail(FC2_E_PARAM, "fc2_result_expand: the compact forms hold canonical-mode results only");
    if (width != 2 && width != 4) return fc2::fail(FC2_E_PARAM, "fc2_result_expand: width is 2 or 4");
    if ((n && (!words || !out)) || (n_esc && !esc)) return fc2::fail(FC2_E_PARAM, "fc2_result_expand: bad args");
    std::atomic<uint64_t> flagged{0};
    auto escaped = [&](uint64_t i) {
        return width == 2 ? (((const uint16_t *)words)[i] & 0x7Fu) == FC2_R16_ESCAPE
                          : (((const uint32_t *)words)[i] & FC2_R32_ESCAPE) != 0;
    };
    parallel_for(n, n_workers(n_threads), [&](uint64_t b, uint64_t e) {
        uint64_t f = 0;
        uint64_t *o = (uint64_t *)out;
        if (width == 2) {
            const uint16_t *w = (const uint16_t *)words;
            for (uint64_t i = b; i < e; ++i) {
                const uint16_t c = w[i];
                const bool x = (c & 0x7Fu) == FC2_R16_ESCAPE;
                f += x;
                o[i] = x ? 0 : fc2::r16_unpack(c);
            }
        } else {
            const uint32_t *w = (const uint32_t *)words;
            for (uint64_t i = b; i < e; ++i) {
                const uint32_t c = w[i];
                f += c >> 31;
                o[i] = (c & FC2_R32_ESCAPE) ? 0 : fc2::r32_unpack(c);
            }
        }
        flagged += f;
    });
    if (flagged.load() != n_esc)
        return fc2::fail(FC2_E_FORMAT, "fc2_result_expand: " + std::to_string(flagged.load()) + " escaped words, " +
                                           std::to_string(n_esc) + " escapes");
    std::vector<uint64_t> idx(n_esc);
    for (uint64_t k = 0; k < n_esc; ++k) {
        if (esc[k].index >= n || !escaped(esc[k].index))
            return fc2::fail(FC2_E_FORMAT, "fc2_result_expand: escape " + std::to_string(k) + " has no escaped word");
        idx[k] = esc[k].index;
        out[esc[k].index] = esc[k].result;
    }
    std::sort(idx.begin(), idx.end());
    if (std::adjacent_find(idx.begin(), idx.end()) != idx.end())
        return fc2::fail(FC2_E_FORMAT, "fc2_result_expand: an escaped word has two escapes");
    return FC2_OK;
}
