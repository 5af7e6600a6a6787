// Per-device context over the breakpoint search (include/fc2_ctx.h): the genome made resident on
// the device with every table of fc2_genome_view (what find_circ2_amd/genome.py builds through
// PyTorch), and a batch pipeline -- host pack (fc2_pack_pairs / fc2_bytepath_fill) into page-locked
// staging, H2D, fc2_bp_scan_launch + fc2_bp_scan_bytes_launch, D2H -- on the context's own stream.
// It replaces the Python host layer for hosts that bind the C ABI directly.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "../../include/fc2_bp.h"
#include "../../include/fc2_ctx.h"
#include "fc2_common.h"
#include "fc2_hostmem.h"

namespace {

int hip_fail(hipError_t e, const char *what) {
    return fc2::fail(FC2_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// a device allocation that only grows
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    // slack: room for later, larger batches (staging); a genome table is allocated exactly
    int reserve(size_t bytes, const char *what, bool slack = true) {
        if (bytes <= cap && p) return FC2_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(slack ? bytes + bytes / 4 : bytes, 256);
        const hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) { p = nullptr; return hip_fail(e, what); }
        cap = want;
        return FC2_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// page-locked host staging that only grows
struct HostBuf {
    void *p = nullptr;
    size_t cap = 0;
    int reserve(size_t bytes, const char *what) {
        if (bytes <= cap && p) return FC2_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 256);
        const hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) { p = nullptr; return hip_fail(e, what); }
        cap = want;
        return FC2_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

}  // namespace

struct fc2_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // genome (borrowed: another context's tables, fc2_ctx_create_sibling)
    bool have_genome = false;
    bool borrowed = false;
    const fc2_fasta *fa = nullptr;
    fc2_genome_view gv{};
    DevBuf units, nplane, ncoarse, cstart, csize, twin, nsuper, wt;
    fc2::MappedWords h_units, h_nplane;             // the host planes the device tables were uploaded from
    // batch
    HostBuf h_pairs, h_words, h_nwords, h_res, h_tm, h_bidx, h_bpairs, h_boff, h_arena;
    DevBuf d_pairs, d_words, d_nwords, d_res, d_tm, d_bidx, d_bpairs, d_boff, d_arena;
    bool pending = false;
    uint64_t n = 0;
    uint32_t tw = 0;
    bool allhits = false;
    fc2_result *out_res = nullptr;
    uint64_t *out_tm = nullptr;

    void free_genome() {
        if (!borrowed)
            for (DevBuf *b : {&units, &nplane, &ncoarse, &cstart, &csize, &twin, &nsuper, &wt}) b->release();
        h_units.release();
        h_nplane.release();
        borrowed = false;
        gv = fc2_genome_view{};
        have_genome = false;
        fa = nullptr;
    }
};

namespace {

// record a failure on the context (fc2_ctx_last_error) and pass the code on
int keep(fc2_ctx *c, int rc) {
    if (rc != FC2_OK && c) {
        const char *m = fc2_last_error();
        c->err = m ? m : "";
    }
    return rc;
}

int use_device(fc2_ctx *c) {
    const hipError_t e = hipSetDevice(c->device);
    return e == hipSuccess ? FC2_OK : hip_fail(e, "hipSetDevice");
}

int h2d(DevBuf &d, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return FC2_OK;
    const hipError_t e = hipMemcpyAsync(d.p, src, bytes, hipMemcpyHostToDevice, s);
    return e == hipSuccess ? FC2_OK : hip_fail(e, "hipMemcpyAsync H2D");
}

}  // namespace

extern "C" int fc2_ctx_create(int device, fc2_ctx **out) {
    if (!out) return fc2::fail(FC2_E_PARAM, "fc2_ctx_create: null argument");
    *out = nullptr;
    if (device < 0) return fc2::fail(FC2_E_PARAM, "fc2_ctx_create: negative device");
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess) return hip_fail(e, "fc2_ctx_create: hipGetDeviceCount");
    if (device >= count)
        return fc2::fail(FC2_E_HIP, "fc2_ctx_create: device " + std::to_string(device) + " of " +
                                        std::to_string(count));
    fc2_ctx *c = new fc2_ctx();
    c->device = device;
    int rc = use_device(c);
    if (rc == FC2_OK) {
        e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        if (e != hipSuccess) rc = hip_fail(e, "hipStreamCreateWithFlags");
    }
    if (rc != FC2_OK) {
        delete c;
        return rc;
    }
    *out = c;
    return FC2_OK;
}

extern "C" int fc2_ctx_create_sibling(const fc2_ctx *src, fc2_ctx **out) {
    if (!src || !out) return fc2::fail(FC2_E_PARAM, "fc2_ctx_create_sibling: null argument");
    *out = nullptr;
    if (!src->have_genome) return fc2::fail(FC2_E_PARAM, "fc2_ctx_create_sibling: the source context has no genome");
    fc2_ctx *c = nullptr;
    if (int rc = fc2_ctx_create(src->device, &c)) return rc;
    c->gv = src->gv;                           // read-only tables: shared, never freed by the sibling
    c->fa = src->fa;
    c->have_genome = true;
    c->borrowed = true;
    *out = c;
    return FC2_OK;
}

extern "C" void fc2_ctx_destroy(fc2_ctx *c) {
    if (!c) return;
    if (hipSetDevice(c->device) == hipSuccess && c->stream) (void)hipStreamSynchronize(c->stream);
    c->free_genome();
    for (HostBuf *b : {&c->h_pairs, &c->h_words, &c->h_nwords, &c->h_res, &c->h_tm, &c->h_bidx, &c->h_bpairs,
                       &c->h_boff, &c->h_arena})
        b->release();
    for (DevBuf *b : {&c->d_pairs, &c->d_words, &c->d_nwords, &c->d_res, &c->d_tm, &c->d_bidx, &c->d_bpairs,
                      &c->d_boff, &c->d_arena})
        b->release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" int fc2_ctx_genome_load(fc2_ctx *c, const fc2_fasta *fa, int n_threads) {
    if (!c) return fc2::fail(FC2_E_PARAM, "fc2_ctx_genome_load: null context");
    c->err.clear();
    if (c->pending) return keep(c, fc2::fail(FC2_E_PARAM, "fc2_ctx_genome_load: a batch is queued (fc2_ctx_sync)"));
    int rc = use_device(c);
    if (rc) return keep(c, rc);
    if (hipStreamSynchronize(c->stream) != hipSuccess) return keep(c, fc2::fail(FC2_E_HIP, "stream sync"));
    c->free_genome();
    if (!fa) {                                 // GenomeAccessor's dummy mode (find_circ.py:340-345)
        c->gv.dummy = 1;
        c->gv.n_chrom = 0xFFFFFFFFu;
        c->have_genome = true;
        return FC2_OK;
    }
    // index + 2-bit planes on the host (find_circ.py:110-155 semantics, fc2_host.cpp); phase times on
    // stderr with FC2_CALLER_TIMING
    static const bool timing = getenv("FC2_CALLER_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    const int nch = fc2_fasta_n_chrom(fa);
    std::vector<int64_t> sizes((size_t)std::max(nch, 1), 0);
    for (int i = 0; i < nch; ++i)
        if ((rc = fc2_fasta_chrom(fa, i, nullptr, &sizes[(size_t)i], nullptr, nullptr, nullptr, nullptr))) return keep(c, rc);
    uint64_t nu = 0, ncw = 0;
    std::vector<uint64_t> cs((size_t)std::max(nch, 1), 0);
    if ((rc = fc2_fasta_layout(fa, &nu, &ncw, cs.data()))) return keep(c, rc);
    // anonymous mappings left untouched: fc2_fasta_pack writes every word (padding units included) on
    // its threads, so the pages are first touched there in parallel; huge pages where the kernel gives
    // them (fewer faults, a cheap unmap).  Kept by the context until its genome is freed: unmapping
    // ~1 GB here would hold the process's memory map while the caller (the read loop, the sibling
    // contexts' HIP queues) waits for this call.  Host cost: every primary context keeps its own copy
    // (2-bit planes + N plane, ~1.2 GB for hg19): only the first load of an fc2_fasta takes the prepacked
    // planes, so a run over N devices (CLI --gpus N, N > 1) holds N such copies until its contexts close.
    fc2::MappedWords &units = c->h_units, &nplane = c->h_nplane;
    std::vector<uint32_t> ncoarse;
    uint64_t n_exotic = 0;
    // planes fc2_fasta_prepack made already (while this context's HIP initialisation ran): upload only
    const bool prepacked = fc2::take_prepacked(fa, nu, units, nplane, ncoarse);
    if (!prepacked) {
        units = fc2::MappedWords(2 * nu);
        nplane = fc2::MappedWords(nu);
    }
    if (!units.ok() || !nplane.ok()) return keep(c, fc2::fail(FC2_E_OS, "fc2_ctx_genome_load: cannot map host memory for the 2-bit genome"));
    const double t_alloc = ms();
    if (!prepacked) {
        ncoarse.assign((size_t)std::max<uint64_t>(ncw, 1), 0);
        if ((rc = fc2_fasta_pack(fa, units.data(), nplane.data(), ncoarse.data(), &n_exotic, n_threads))) return keep(c, rc);
    }
    const double t_pack = ms();
    // device tables (genome.py _upload / _upload_tables)
    const hipStream_t s = c->stream;
    if ((rc = c->units.reserve(units.size() * 8, "genome units", false)) || (rc = c->nplane.reserve(nplane.size() * 8, "genome N plane", false)) ||
        (rc = c->ncoarse.reserve(ncoarse.size() * 4, "genome coarse N map", false)) || (rc = c->cstart.reserve(cs.size() * 8, "chromosome starts", false)) ||
        (rc = c->csize.reserve(sizes.size() * 8, "chromosome sizes", false)) || (rc = c->twin.reserve(2 * (nu + 8) * 8, "genome twin", false)))
        return keep(c, rc);
    if ((rc = h2d(c->units, units.data(), units.size() * 8, s)) || (rc = h2d(c->nplane, nplane.data(), nplane.size() * 8, s)) ||
        (rc = h2d(c->ncoarse, ncoarse.data(), ncoarse.size() * 4, s)) || (rc = h2d(c->cstart, cs.data(), cs.size() * 8, s)) ||
        (rc = h2d(c->csize, sizes.data(), sizes.size() * 8, s)))
        return keep(c, rc);
    if ((rc = fc2_twin_launch(c->units.as<uint64_t>(), nu, c->twin.as<uint64_t>(), s))) return keep(c, rc);
    uint32_t ns_shift = 0, ns_words = 0;
    if ((rc = fc2_nsuper_geometry(nu, &ns_shift, &ns_words))) return keep(c, rc);
    const size_t ns_alloc = ((size_t)ns_words + 3) / 4 * 4;
    if ((rc = c->nsuper.reserve(ns_alloc * 4, "N super map", false))) return keep(c, rc);
    if (hipMemsetAsync(c->nsuper.p, 0, ns_alloc * 4, s) != hipSuccess) return keep(c, fc2::fail(FC2_E_HIP, "memset"));
    if ((rc = fc2_nsuper_launch(c->ncoarse.as<uint32_t>(), nu, c->nsuper.as<uint32_t>(), s))) return keep(c, rc);
    uint64_t wt_bytes = 0, wt_twin_off = 0;
    const bool words = fc2_wtab_geometry(nu, &wt_bytes, &wt_twin_off) == FC2_OK;   // > ~8 Gbp: unit planes only
    if (words) {
        if ((rc = c->wt.reserve(wt_bytes, "word-pair table", false))) return keep(c, rc);
        if ((rc = fc2_wtab_launch(c->units.as<uint64_t>(), nu, c->wt.as<uint32_t>(), s))) return keep(c, rc);
    }
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return keep(c, hip_fail(e, "genome upload"));
    if (timing)
        fprintf(stderr, "genome load: host vectors %.1f ms, 2-bit pack %.1f ms%s, device alloc + upload + tables %.1f ms "
                        "(%llu units)\n", t_alloc, t_pack - t_alloc, prepacked ? " (prepacked)" : "", ms() - t_pack,
                (unsigned long long)nu);
    fc2_genome_view &g = c->gv;
    g.units = c->units.as<const uint64_t>();
    g.nplane = c->nplane.as<const uint64_t>();
    g.ncoarse = c->ncoarse.as<const uint32_t>();
    g.chrom_start = c->cstart.as<const uint64_t>();
    g.chrom_size = c->csize.as<const int64_t>();
    g.n_units = nu;
    g.n_chrom = (uint32_t)nch;
    g.dummy = 0;
    g.units_twin = c->twin.as<const uint64_t>();
    g.nsuper = c->nsuper.as<const uint32_t>();
    g.nsuper_shift = ns_shift;
    g.nsuper_words = ns_words;
    g.wt = words ? c->wt.as<const uint32_t>() : nullptr;
    g.wt_bytes = words ? wt_bytes : 0;
    g.wt_twin_off = words ? wt_twin_off : 0;
    c->fa = fa;
    c->have_genome = true;
    return FC2_OK;
}

extern "C" int fc2_ctx_genome_view(const fc2_ctx *c, fc2_genome_view *out) {
    if (!c || !out) return fc2::fail(FC2_E_PARAM, "fc2_ctx_genome_view: null argument");
    if (!c->have_genome) return fc2::fail(FC2_E_PARAM, "fc2_ctx_genome_view: no genome loaded");
    *out = c->gv;
    return FC2_OK;
}

extern "C" int fc2_ctx_scan_async(fc2_ctx *c, const fc2_params *p, uint64_t n, const uint8_t *reads,
                                  const uint64_t *read_off, const fc2_pair *pairs, fc2_result *results,
                                  uint64_t *tiemask, uint32_t tw, int n_threads) {
    if (!c) return fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_async: null context");
    c->err.clear();
    int rc = fc2::validate_params(p);
    if (rc) return keep(c, rc);
    if (c->pending) return keep(c, fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_async: the previous batch was not synced"));
    if (!c->have_genome)
        return keep(c, fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_async: no genome (fc2_ctx_genome_load; NULL = dummy genome)"));
    if (n && (!reads || !read_off || !pairs || !results))
        return keep(c, fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_async: null argument"));
    if (p->allhits && n && !tiemask) return keep(c, fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_async: --all-hits needs a tie mask"));
    if ((rc = use_device(c))) return keep(c, rc);
    c->n = n;
    c->allhits = p->allhits != 0;
    c->tw = tw;
    c->out_res = results;
    c->out_tm = tiemask;
    if (n == 0) {
        c->pending = true;
        return FC2_OK;
    }
    int max_len = 0;
    for (uint64_t i = 0; i < n; ++i) max_len = std::max<int>(max_len, pairs[i].read_len);
    uint32_t rw = 0, nw = 0, tw_need = 0;
    if ((rc = fc2_batch_geometry(p, max_len, &rw, &nw, &tw_need))) return keep(c, rc);
    if (c->allhits && tw < tw_need)
        return keep(c, fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_async: tie mask of " + std::to_string(tw) + " words per pair, " +
                                                  std::to_string(tw_need) + " needed"));
    const size_t tmw = c->allhits ? (size_t)tw * n : 0;
    if ((rc = c->h_pairs.reserve(n * sizeof(fc2_pair), "pair staging")) || (rc = c->h_words.reserve((size_t)rw * n * 8, "read-row staging")) ||
        (rc = c->h_nwords.reserve((size_t)nw * n * 8, "N-row staging")) || (rc = c->h_res.reserve(n * 8, "result staging")) ||
        (tmw && (rc = c->h_tm.reserve(tmw * 8, "tie-mask staging"))) || (rc = c->d_pairs.reserve(n * sizeof(fc2_pair), "pairs")) ||
        (rc = c->d_words.reserve((size_t)rw * n * 8, "read rows")) || (rc = c->d_nwords.reserve((size_t)nw * n * 8, "N rows")) ||
        (rc = c->d_res.reserve(n * 8, "results")) || (tmw && (rc = c->d_tm.reserve(tmw * 8, "tie mask"))))
        return keep(c, rc);
    // host pack (PairBatch.pack): the pairs gain READ_N / BYTEPATH flags, the reads become 2-bit rows
    memcpy(c->h_pairs.p, pairs, n * sizeof(fc2_pair));
    memset(c->h_words.p, 0, (size_t)rw * n * 8);
    memset(c->h_nwords.p, 0, (size_t)nw * n * 8);
    fc2_pair *hp = c->h_pairs.as<fc2_pair>();
    uint64_t n_bytepath = 0;
    if ((rc = fc2_pack_pairs(p, c->fa, n, reads, read_off, hp, c->h_words.as<uint64_t>(), rw, c->h_nwords.as<uint64_t>(), nw,
                             n, &n_bytepath, n_threads)))
        return keep(c, rc);
    const int e = fc2::eff_anchor(p);
    int max_l = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (!(hp[i].flags & (FC2_PAIR_BYTEPATH | FC2_PAIR_SKIP))) max_l = std::max(max_l, (int)hp[i].read_len - 2 * e);
    const hipStream_t s = c->stream;
    // from the first enqueue on, a failure must not return while copies out of the page-locked
    // staging or the scan are still queued: the next call would rewrite (or HostBuf::reserve free)
    // memory they read, and fc2_ctx_sync would return at once (pending stays false)
    auto abandon = [&](int code) {
        const std::string msg = fc2_last_error();
        (void)hipStreamSynchronize(s);
        return keep(c, fc2::fail(code, msg));
    };
    if ((rc = h2d(c->d_pairs, hp, n * sizeof(fc2_pair), s)) || (rc = h2d(c->d_words, c->h_words.p, (size_t)rw * n * 8, s)) ||
        (rc = h2d(c->d_nwords, c->h_nwords.p, (size_t)nw * n * 8, s)))
        return abandon(rc);
    if (tmw && hipMemsetAsync(c->d_tm.p, 0, tmw * 8, s) != hipSuccess) return abandon(fc2::fail(FC2_E_HIP, "tie-mask memset"));
    fc2_batch_view bv{};
    bv.pairs = c->d_pairs.as<const fc2_pair>();
    bv.read_words = c->d_words.as<const uint64_t>();
    bv.read_nwords = c->d_nwords.as<const uint64_t>();
    bv.n = n;
    bv.stride = n;
    bv.rw = rw;
    bv.nw = nw;
    bv.max_l = max_l;
    bv.layout = 0;
    uint64_t *dtm = tmw ? c->d_tm.as<uint64_t>() : nullptr;
    if ((rc = fc2_bp_scan_launch(p, &c->gv, &bv, c->d_res.as<fc2_result>(), dtm, tw, s))) return abandon(rc);
    if (n_bytepath) {                          // pairs whose windows need the FASTA's bytes
        uint64_t m = 0, arena = 0;
        if ((rc = fc2_bytepath_size(p, n, hp, &m, &arena))) return abandon(rc);
        if ((rc = c->h_bidx.reserve(m * 8, "byte-path index")) || (rc = c->h_bpairs.reserve(m * sizeof(fc2_pair), "byte-path pairs")) ||
            (rc = c->h_boff.reserve(m * 8, "byte-path offsets")) || (rc = c->h_arena.reserve(std::max<uint64_t>(arena, 16), "byte-path arena")) ||
            (rc = c->d_bidx.reserve(m * 8, "byte-path index")) || (rc = c->d_bpairs.reserve(m * sizeof(fc2_pair), "byte-path pairs")) ||
            (rc = c->d_boff.reserve(m * 8, "byte-path offsets")) || (rc = c->d_arena.reserve(std::max<uint64_t>(arena, 16), "byte-path arena")))
            return abandon(rc);
        if ((rc = fc2_bytepath_fill(p, c->fa, n, reads, read_off, hp, c->h_bidx.as<uint64_t>(), c->h_bpairs.as<fc2_pair>(),
                                    c->h_boff.as<uint64_t>(), c->h_arena.as<uint8_t>())))
            return abandon(rc);
        if ((rc = h2d(c->d_bidx, c->h_bidx.p, m * 8, s)) || (rc = h2d(c->d_bpairs, c->h_bpairs.p, m * sizeof(fc2_pair), s)) ||
            (rc = h2d(c->d_boff, c->h_boff.p, m * 8, s)) || (rc = h2d(c->d_arena, c->h_arena.p, arena, s)))
            return abandon(rc);
        fc2_bytes_view v{c->d_bidx.as<const uint64_t>(), c->d_bpairs.as<const fc2_pair>(), c->d_arena.as<const uint8_t>(),
                         c->d_boff.as<const uint64_t>(), m};
        if ((rc = fc2_bp_scan_bytes_launch(p, &v, c->d_res.as<fc2_result>(), dtm, tw, n, s))) return abandon(rc);
    }
    hipError_t he = hipMemcpyAsync(c->h_res.p, c->d_res.p, n * 8, hipMemcpyDeviceToHost, s);
    if (he == hipSuccess && tmw) he = hipMemcpyAsync(c->h_tm.p, c->d_tm.p, tmw * 8, hipMemcpyDeviceToHost, s);
    if (he != hipSuccess) return abandon(hip_fail(he, "hipMemcpyAsync D2H"));
    c->pending = true;
    return FC2_OK;
}

extern "C" int fc2_ctx_sync(fc2_ctx *c) {
    if (!c) return fc2::fail(FC2_E_PARAM, "fc2_ctx_sync: null context");
    c->err.clear();
    if (!c->pending) return FC2_OK;
    c->pending = false;
    int rc = use_device(c);
    if (rc) return keep(c, rc);
    const hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return keep(c, hip_fail(e, "fc2_ctx_sync"));
    if (c->n) {
        memcpy(c->out_res, c->h_res.p, c->n * 8);
        if (c->allhits) memcpy(c->out_tm, c->h_tm.p, (size_t)c->tw * c->n * 8);
    }
    return FC2_OK;
}

extern "C" int fc2_ctx_scan_long(fc2_ctx *c, const fc2_params *p, uint64_t n, const uint8_t *reads,
                                 const fc2_long_pair *pairs, fc2_long_result *results, uint64_t *ties) {
    if (!c) return fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_long: null context");
    c->err.clear();
    int rc = fc2::validate_params(p);
    if (rc) return keep(c, rc);
    if (c->pending) return keep(c, fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_long: a batch is queued (fc2_ctx_sync)"));
    if (!c->have_genome)
        return keep(c, fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_long: no genome (fc2_ctx_genome_load; NULL = dummy genome)"));
    if (n == 0) return FC2_OK;
    if (!reads || !pairs || !results || (p->allhits && !ties))
        return keep(c, fc2::fail(FC2_E_PARAM, "fc2_ctx_scan_long: null argument"));
    if ((rc = use_device(c))) return keep(c, rc);
    uint64_t arena = 0;
    std::vector<uint64_t> tie_off(n + 1), off(n);
    if ((rc = fc2_long_geometry(p, n, pairs, &arena, tie_off.data()))) return keep(c, rc);
    std::vector<uint8_t> h_arena((size_t)std::max<uint64_t>(arena, 16));
    if ((rc = fc2_long_fill(p, c->fa, n, reads, pairs, off.data(), h_arena.data()))) return keep(c, rc);
    const uint64_t nt = p->allhits ? tie_off[n] : 0;
    // device buffers of this call only (long pairs are rare): pairs, offsets, arena, tie offsets,
    // results, ties
    DevBuf d_lp, d_off, d_arena, d_toff, d_res, d_ties;
    auto cleanup = [&] { for (DevBuf *b : {&d_lp, &d_off, &d_arena, &d_toff, &d_res, &d_ties}) b->release(); };
    const hipStream_t s = c->stream;
    if ((rc = d_lp.reserve(n * sizeof(fc2_long_pair), "long pairs", false)) || (rc = d_off.reserve(n * 8, "long offsets", false)) ||
        (rc = d_arena.reserve(h_arena.size(), "long arena", false)) || (rc = d_toff.reserve((n + 1) * 8, "long tie offsets", false)) ||
        (rc = d_res.reserve(n * sizeof(fc2_long_result), "long results", false)) ||
        (nt && (rc = d_ties.reserve(nt * 8, "long ties", false)))) {
        cleanup();
        return keep(c, rc);
    }
    if ((rc = h2d(d_lp, pairs, n * sizeof(fc2_long_pair), s)) || (rc = h2d(d_off, off.data(), n * 8, s)) ||
        (rc = h2d(d_arena, h_arena.data(), h_arena.size(), s)) || (rc = h2d(d_toff, tie_off.data(), (n + 1) * 8, s)) ||
        (rc = fc2_bp_scan_long_launch(p, n, d_lp.as<fc2_long_pair>(), d_off.as<uint64_t>(), d_arena.as<uint8_t>(),
                                      d_toff.as<uint64_t>(), d_res.as<fc2_long_result>(), nt ? d_ties.as<uint64_t>() : nullptr, s))) {
        (void)hipStreamSynchronize(s);      // the host vectors must outlive the queued copies
        cleanup();
        return keep(c, rc);
    }
    hipError_t he = hipMemcpyAsync(results, d_res.p, n * sizeof(fc2_long_result), hipMemcpyDeviceToHost, s);
    if (he == hipSuccess && nt) he = hipMemcpyAsync(ties, d_ties.p, nt * 8, hipMemcpyDeviceToHost, s);
    const hipError_t se = hipStreamSynchronize(s);
    cleanup();
    if (he != hipSuccess) return keep(c, hip_fail(he, "fc2_ctx_scan_long D2H"));
    if (se != hipSuccess) return keep(c, hip_fail(se, "fc2_ctx_scan_long"));
    return FC2_OK;
}

extern "C" void *fc2_ctx_stream(const fc2_ctx *c) { return c ? (void *)c->stream : nullptr; }

extern "C" const char *fc2_ctx_last_error(const fc2_ctx *c) { return c ? c->err.c_str() : ""; }
