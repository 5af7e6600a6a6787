// fc2_bamout.cpp -- BGZF/BAM writer for -B/--bam (see fc2_bamout.h).
#include "fc2_bamout.h"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <thread>

namespace fc2 {
namespace bam {

namespace {
constexpr size_t kBlockIn = 0xff00;        // htslib's BGZF_BLOCK_SIZE: input bytes per block
constexpr size_t kBlockMax = 0x10000;      // a block (header + deflate + trailer) is at most 64 KiB

// SAM spec 5.3 (and htslib hts_reg2bin with min_shift 14, 5 levels)
int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

int nt16(char c) {                         // htslib seq_nt16_table (case-insensitive, else N)
    switch (c) {
        case '=': return 0; case 'A': case 'a': return 1; case 'C': case 'c': return 2;
        case 'M': case 'm': return 3; case 'G': case 'g': return 4; case 'R': case 'r': return 5;
        case 'S': case 's': return 6; case 'V': case 'v': return 7; case 'T': case 't': return 8;
        case 'U': case 'u': return 8; case 'W': case 'w': return 9; case 'Y': case 'y': return 10;
        case 'H': case 'h': return 11; case 'K': case 'k': return 12; case 'D': case 'd': return 13;
        case 'B': case 'b': return 14; default: return 15;
    }
}

int cigar_op(char c) {
    const char *ops = "MIDNSHP=X";
    const char *p = strchr(ops, c);
    return (c && p) ? (int)(p - ops) : -1;
}

template <class T> void put(std::string &s, T v) { s.append((const char *)&v, sizeof v); }
}  // namespace

// one BGZF block of n (<= kBlockIn) input bytes into out (kBlockMax bytes); its size, 0 on failure
size_t deflate_block(z_stream &zs, const char *in, size_t n, uint8_t *out) {
    deflateReset(&zs);
    zs.next_in = (Bytef *)in;
    zs.avail_in = (uInt)n;
    zs.next_out = out + 18;
    zs.avail_out = (uInt)(kBlockMax - 18 - 8);
    if (deflate(&zs, Z_FINISH) != Z_STREAM_END) return 0;
    const size_t clen = kBlockMax - 18 - 8 - zs.avail_out;
    const size_t bsize = 18 + clen + 8;
    static const uint8_t hdr[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0};
    memcpy(out, hdr, 16);
    out[16] = (uint8_t)((bsize - 1) & 0xff);
    out[17] = (uint8_t)((bsize - 1) >> 8);
    const uint32_t crc = (uint32_t)crc32(0L, (const Bytef *)in, (uInt)n);
    const uint32_t isize = (uint32_t)n;
    memcpy(out + 18 + clen, &crc, 4);
    memcpy(out + 18 + clen + 4, &isize, 4);
    return bsize;
}

struct Writer {
    FILE *fp = nullptr;
    std::string buf;                       // uncompressed bytes of the current block
    z_stream zs{};
    int level = 6;
    bool ok = true;
    std::vector<uint8_t> out;

    bool flush_block() {
        if (buf.empty()) return ok;
        out.resize(kBlockMax);
        const size_t bsize = deflate_block(zs, buf.data(), buf.size(), out.data());
        if (!bsize) return ok = false;
        if (fwrite(out.data(), 1, bsize, fp) != bsize) ok = false;
        buf.clear();
        return ok;
    }
    bool add(const char *p, size_t n) {
        while (n) {
            const size_t k = std::min(n, kBlockIn - buf.size());
            buf.append(p, k);
            p += k;
            n -= k;
            if (buf.size() == kBlockIn && !flush_block()) return false;
        }
        return ok;
    }
};

Writer *open_writer(const std::string &path, const std::string &text, const std::vector<std::string> &names,
                    const std::vector<int64_t> &lens, std::string &err, int level) {
    FILE *fp = fopen(path.c_str(), "wb");
    if (!fp) {
        err = "IOError: cannot open '" + path + "': " + strerror(errno);
        return nullptr;
    }
    Writer *w = new Writer();
    w->fp = fp;
    w->level = level;
    if (deflateInit2(&w->zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
        fclose(fp);
        delete w;
        err = "zlib init failed";
        return nullptr;
    }
    std::string h("BAM\1", 4);
    put<int32_t>(h, (int32_t)text.size());
    h += text;
    put<int32_t>(h, (int32_t)names.size());
    for (size_t i = 0; i < names.size(); ++i) {
        put<int32_t>(h, (int32_t)names[i].size() + 1);
        h += names[i];
        h += '\0';
        put<int32_t>(h, (int32_t)(i < lens.size() ? lens[i] : 0));
    }
    w->add(h.data(), h.size());
    w->flush_block();                      // htslib writes the header in block(s) of its own
    return w;
}

bool write_raw(Writer *w, const uint8_t *rec, size_t n) { return w->add((const char *)rec, n); }

bool write_bulk(Writer *w, const char *p, size_t n, int threads) {
    if (!w->ok) return false;
    // the current block first (the bytes complete it or stay in it)
    const size_t head = std::min(n, kBlockIn - w->buf.size());
    w->buf.append(p, head);
    p += head;
    n -= head;
    if (w->buf.size() < kBlockIn) return true;
    if (!w->flush_block()) return false;
    const size_t nb = n / kBlockIn;           // whole blocks; the rest starts the next current block
    if (nb) {
        const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), nb));
        std::vector<uint8_t> outb(nb * kBlockMax);
        std::vector<size_t> sz(nb, 0);
        std::atomic<size_t> next{0};
        auto work = [&] {
            z_stream zs{};
            if (deflateInit2(&zs, w->level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return;
            for (size_t b; (b = next.fetch_add(1)) < nb;)
                sz[b] = deflate_block(zs, p + b * kBlockIn, kBlockIn, outb.data() + b * kBlockMax);
            deflateEnd(&zs);
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < T; ++t) pool.emplace_back(work);
        work();
        for (auto &th : pool) th.join();
        for (size_t b = 0; b < nb && w->ok; ++b)
            if (!sz[b] || fwrite(outb.data() + b * kBlockMax, 1, sz[b], w->fp) != sz[b]) w->ok = false;
        p += nb * kBlockIn;
        n -= nb * kBlockIn;
    }
    w->buf.assign(p, n);
    return w->ok;
}

bool write_sam(Writer *w, const char *line, const char *end, const std::unordered_map<std::string, int> &tid_of,
               std::string &err) {
    std::string rec;
    return encode_sam(line, end, tid_of, rec, err) && w->add(rec.data(), rec.size());
}

bool encode_sam(const char *line, const char *end, const std::unordered_map<std::string, int> &tid_of,
                std::string &rec, std::string &err) {
    std::vector<std::pair<const char *, const char *>> f;
    for (const char *p = line;;) {
        const char *t = (const char *)memchr(p, '\t', (size_t)(end - p));
        f.emplace_back(p, t ? t : end);
        if (!t) break;
        p = t + 1;
    }
    if (f.size() < 11) {
        err = "ValueError: SAM line with fewer than 11 fields";
        return false;
    }
    auto str = [&](int k) { return std::string(f[k].first, f[k].second); };
    auto tid = [&](const std::string &s) {
        if (s == "*") return -1;
        auto it = tid_of.find(s);
        return it == tid_of.end() ? -1 : it->second;
    };
    const std::string qname = str(0);
    const uint16_t flag = (uint16_t)strtol(str(1).c_str(), nullptr, 10);
    const int32_t ref = tid(str(2));
    const int32_t pos = (int32_t)(strtol(str(3).c_str(), nullptr, 10) - 1);
    const uint8_t mapq = (uint8_t)strtol(str(4).c_str(), nullptr, 10);
    std::vector<uint32_t> cig;
    int64_t rlen = 0;
    const std::string cs = str(5);
    if (cs != "*") {
        uint32_t n = 0;
        for (char c : cs) {
            if (c >= '0' && c <= '9') { n = n * 10 + (uint32_t)(c - '0'); continue; }
            const int op = cigar_op(c);
            if (op < 0) { err = "ValueError: bad CIGAR " + cs; return false; }
            cig.push_back(n << 4 | (uint32_t)op);
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rlen += n;
            n = 0;
        }
    }
    const std::string rn = str(6);
    const int32_t nref = rn == "=" ? ref : tid(rn);
    const int32_t npos = (int32_t)(strtol(str(7).c_str(), nullptr, 10) - 1);
    const int32_t tlen = (int32_t)strtol(str(8).c_str(), nullptr, 10);
    const std::string seq = str(9) == "*" ? std::string() : str(9);
    const std::string qual = str(10);
    const int64_t e = (!(flag & 4) && !cig.empty() && rlen > 0) ? pos + rlen : pos + 1;
    std::string b;
    put<int32_t>(b, ref);
    put<int32_t>(b, pos);
    put<uint8_t>(b, (uint8_t)(qname.size() + 1));
    put<uint8_t>(b, mapq);
    put<uint16_t>(b, (uint16_t)reg2bin(pos, e));
    put<uint16_t>(b, (uint16_t)cig.size());
    put<uint16_t>(b, flag);
    put<int32_t>(b, (int32_t)seq.size());
    put<int32_t>(b, nref);
    put<int32_t>(b, npos);
    put<int32_t>(b, tlen);
    b += qname;
    b += '\0';
    for (uint32_t c : cig) put<uint32_t>(b, c);
    for (size_t k = 0; k < seq.size(); k += 2)
        put<uint8_t>(b, (uint8_t)(nt16(seq[k]) << 4 | (k + 1 < seq.size() ? nt16(seq[k + 1]) : 0)));
    if (qual == "*") b.append(seq.size(), '\xff');
    else for (size_t k = 0; k < seq.size(); ++k) put<uint8_t>(b, (uint8_t)(k < qual.size() ? qual[k] - 33 : 0xff));
    for (size_t k = 11; k < f.size(); ++k) {   // optional fields TG:T:VALUE
        const char *t = f[k].first, *te = f[k].second;
        if (te - t < 5 || t[2] != ':' || t[4] != ':') { err = "ValueError: bad SAM tag"; return false; }
        b.append(t, 2);
        const std::string v(t + 5, te);
        switch (t[3]) {
            case 'A': b += 'A'; b += v.empty() ? '\0' : v[0]; break;
            case 'i': {                        // the smallest integer type that holds it (sam_parse1)
                const long long x = strtoll(v.c_str(), nullptr, 10);
                if (x < 0) {
                    if (x >= INT8_MIN) { b += 'c'; put<int8_t>(b, (int8_t)x); }
                    else if (x >= INT16_MIN) { b += 's'; put<int16_t>(b, (int16_t)x); }
                    else { b += 'i'; put<int32_t>(b, (int32_t)x); }
                } else {
                    if (x <= UINT8_MAX) { b += 'C'; put<uint8_t>(b, (uint8_t)x); }
                    else if (x <= UINT16_MAX) { b += 'S'; put<uint16_t>(b, (uint16_t)x); }
                    else { b += 'I'; put<uint32_t>(b, (uint32_t)x); }
                }
                break;
            }
            case 'f': b += 'f'; put<float>(b, strtof(v.c_str(), nullptr)); break;
            case 'Z': case 'H': b += t[3]; b += v; b += '\0'; break;
            case 'B': {
                if (v.empty()) { err = "ValueError: bad B tag"; return false; }
                const char sub = v[0];
                std::vector<std::string> xs;
                for (size_t p = 1; p < v.size();) {
                    if (v[p] == ',') ++p;
                    size_t q = v.find(',', p);
                    if (q == std::string::npos) q = v.size();
                    xs.push_back(v.substr(p, q - p));
                    p = q;
                }
                b += 'B';
                b += sub;
                put<int32_t>(b, (int32_t)xs.size());
                for (const std::string &x : xs) {
                    switch (sub) {
                        case 'c': put<int8_t>(b, (int8_t)strtol(x.c_str(), nullptr, 10)); break;
                        case 'C': put<uint8_t>(b, (uint8_t)strtoul(x.c_str(), nullptr, 10)); break;
                        case 's': put<int16_t>(b, (int16_t)strtol(x.c_str(), nullptr, 10)); break;
                        case 'S': put<uint16_t>(b, (uint16_t)strtoul(x.c_str(), nullptr, 10)); break;
                        case 'i': put<int32_t>(b, (int32_t)strtol(x.c_str(), nullptr, 10)); break;
                        case 'I': put<uint32_t>(b, (uint32_t)strtoul(x.c_str(), nullptr, 10)); break;
                        case 'f': put<float>(b, strtof(x.c_str(), nullptr)); break;
                        default: err = "ValueError: bad B tag subtype"; return false;
                    }
                }
                break;
            }
            default: err = "ValueError: bad SAM tag type"; return false;
        }
    }
    put<int32_t>(rec, (int32_t)b.size());
    rec += b;
    return true;
}

bool close_writer(Writer *w, std::string &err) {
    if (!w) return true;
    bool ok = w->flush_block();
    static const uint8_t eof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0, 0x1b, 0,
                                    3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (fwrite(eof, 1, sizeof eof, w->fp) != sizeof eof) ok = false;
    if (fclose(w->fp) != 0) ok = false;
    deflateEnd(&w->zs);
    delete w;
    if (!ok) err = "IOError: writing spliced_alignments.bam failed";
    return ok;
}

}  // namespace bam
}  // namespace fc2
