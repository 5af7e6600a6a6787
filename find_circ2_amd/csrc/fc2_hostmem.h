// Host memory of the device genome's build (fc2_host.cpp packs, fc2_ctx.cpp uploads).
#pragma once
#include <stdint.h>
#include <sys/mman.h>

#include <algorithm>
#include <vector>

#include "../../include/fc2_bp.h"

namespace fc2 {

// Host words in an anonymous mapping (MADV_HUGEPAGE), unmapped by the owner
class MappedWords {
  public:
    MappedWords() = default;
    explicit MappedWords(size_t k) : n_(k), bytes_(std::max<size_t>(k, 1) * 8) {
        void *m = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) return;
        (void)madvise(m, bytes_, MADV_HUGEPAGE);
        p_ = (uint64_t *)m;
    }
    MappedWords(const MappedWords &) = delete;
    MappedWords &operator=(const MappedWords &) = delete;
    MappedWords(MappedWords &&o) noexcept : p_(o.p_), n_(o.n_), bytes_(o.bytes_) { o.p_ = nullptr, o.n_ = o.bytes_ = 0; }
    MappedWords &operator=(MappedWords &&o) noexcept {
        if (this != &o) {
            release();
            p_ = o.p_, n_ = o.n_, bytes_ = o.bytes_;
            o.p_ = nullptr, o.n_ = o.bytes_ = 0;
        }
        return *this;
    }
    ~MappedWords() { release(); }
    void release() {
        if (p_) munmap(p_, bytes_);
        p_ = nullptr, n_ = bytes_ = 0;
    }
    uint64_t *data() { return p_; }
    size_t size() const { return n_; }
    bool ok() const { return p_ != nullptr; }
  private:
    uint64_t *p_ = nullptr;
    size_t n_ = 0, bytes_ = 0;
};

// The 2-bit planes fc2_fasta_prepack made for f (fc2_fasta_layout's n_units): handed over to the
// caller -- fc2_ctx_genome_load, which then only uploads them -- and dropped from f; false if f
// holds none (or for another layout).
bool take_prepacked(const fc2_fasta *f, uint64_t n_units, MappedWords &units, MappedWords &nplane,
                    std::vector<uint32_t> &ncoarse);

}  // namespace fc2
