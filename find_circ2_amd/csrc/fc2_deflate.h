// fc2_deflate.h -- whole-buffer DEFLATE for the loop's hot (de)compression: BGZF blocks inflated
// and CRC-checked (fc2_ingest.cpp), the gzip members of spliced_reads.fastq.gz (fc2_gzpieces.h).
// libdeflate (the image's libdeflate.so.0, 1.10; loaded at run time, its header is not installed,
// so the few entry points are declared here) inflates about twice and checks CRC-32 many times
// faster than zlib; zlib stays the fallback when the library is absent, and FC2_LIBDEFLATE=0
// forces it.  The bytes produced or accepted are the same either way: a BGZF block is taken only
// if it inflates to exactly its ISIZE with its CRC-32, and a gzip member decodes to the same text.
#pragma once
#include <dlfcn.h>
#include <stdint.h>
#include <stdlib.h>
#include <zlib.h>

#include <string>

namespace fc2 {
namespace dfl {

struct Api {
    void *(*alloc_d)() = nullptr;
    int (*inflate_raw)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;   // 0: success
    void (*free_d)(void *) = nullptr;
    uint32_t (*crc32)(uint32_t, const void *, size_t) = nullptr;
    void *(*alloc_c)(int) = nullptr;
    size_t (*gzip_compress)(void *, const void *, size_t, void *, size_t) = nullptr;        // 0: failure
    size_t (*gzip_bound)(void *, size_t) = nullptr;
    void (*free_c)(void *) = nullptr;
    bool ok = false;
};

inline const Api &api() {
    static const Api a = [] {
        Api x;
        const char *e = getenv("FC2_LIBDEFLATE");
        if (e && atoi(e) == 0) return x;
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return x;
        x.alloc_d = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
        x.inflate_raw = (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(h, "libdeflate_deflate_decompress");
        x.free_d = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
        x.crc32 = (uint32_t(*)(uint32_t, const void *, size_t))dlsym(h, "libdeflate_crc32");
        x.alloc_c = (void *(*)(int))dlsym(h, "libdeflate_alloc_compressor");
        x.gzip_compress = (size_t(*)(void *, const void *, size_t, void *, size_t))dlsym(h, "libdeflate_gzip_compress");
        x.gzip_bound = (size_t(*)(void *, size_t))dlsym(h, "libdeflate_gzip_compress_bound");
        x.free_c = (void (*)(void *))dlsym(h, "libdeflate_free_compressor");
        x.ok = x.alloc_d && x.inflate_raw && x.free_d && x.crc32 && x.alloc_c && x.gzip_compress && x.gzip_bound && x.free_c;
        return x;
    }();
    return a;
}

inline uint32_t crc32(const void *p, size_t n) {
    const Api &a = api();
    if (a.ok) return a.crc32(0, p, n);
    uLong c = ::crc32(0L, Z_NULL, 0);
    const Bytef *b = (const Bytef *)p;
    while (n) {                                 // zlib takes uInt lengths
        const uInt k = (uInt)(n > (1u << 30) ? (1u << 30) : n);
        c = ::crc32(c, b, k);
        b += k;
        n -= k;
    }
    return (uint32_t)c;
}

// raw DEFLATE data that must inflate to exactly out_n bytes (a BGZF block's ISIZE)
class Inflater {
  public:
    Inflater() {
        if (api().ok) d_ = api().alloc_d();
        else if (inflateInit2(&zs_, -15) == Z_OK) z_ = true;
    }
    ~Inflater() {
        if (d_) api().free_d(d_);
        if (z_) inflateEnd(&zs_);
    }
    Inflater(const Inflater &) = delete;
    Inflater &operator=(const Inflater &) = delete;
    bool ok() const { return d_ || z_; }
    bool exact(const void *in, size_t in_n, void *out, size_t out_n) {
        if (d_) return api().inflate_raw(d_, in, in_n, out, out_n, nullptr) == 0;
        if (!z_) return false;
        uint8_t none = 0;                       // an empty block (the EOF marker): zlib wants a real pointer
        inflateReset(&zs_);
        zs_.next_in = (Bytef *)in;
        zs_.avail_in = (uInt)in_n;
        zs_.next_out = out_n ? (Bytef *)out : (Bytef *)&none;
        zs_.avail_out = (uInt)out_n;
        return inflate(&zs_, Z_FINISH) == Z_STREAM_END && zs_.avail_out == 0;
    }

  private:
    void *d_ = nullptr;
    z_stream zs_{};
    bool z_ = false;
};

// one gzip member of `in` at `level` into out (replaced); false on failure
inline bool gzip_member(const std::string &in, int level, std::string &out) {
    const Api &a = api();
    if (void *c = a.ok ? a.alloc_c(level) : nullptr) {
        out.resize(a.gzip_bound(c, in.size()));
        const size_t n = a.gzip_compress(c, in.data(), in.size(), &out[0], out.size());
        a.free_c(c);
        out.resize(n);
        return n != 0;
    }
    z_stream zs{};
    if (deflateInit2(&zs, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    out.resize(deflateBound(&zs, (uLong)in.size()) + 64);
    zs.next_in = (Bytef *)in.data();
    zs.avail_in = (uInt)in.size();
    zs.next_out = (Bytef *)&out[0];
    zs.avail_out = (uInt)out.size();
    const int rc = deflate(&zs, Z_FINISH);
    out.resize(zs.total_out);
    deflateEnd(&zs);
    return rc == Z_STREAM_END;
}

}  // namespace dfl
}  // namespace fc2
