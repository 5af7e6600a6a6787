// fc2_inflate.h -- the BAM input's BGZF blocks inflated on a GPU (fc2_inflate.hip), for the ingest's
// batch reader (fc2_ingest.cpp bgzf_batch): a stream and device buffers for batches of up to
// max_blocks blocks, and a pool of pinned batch buffers the inflated bytes are downloaded into.
// One batch at a time per Gpu (the ingest reads one batch ahead); its chunks on several streams.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace fc2 {
namespace inf {

struct Gpu;

// nullptr (err set) if the device or its buffers cannot be had; pool_cap > 0 opens the pinned pool
// with buffers of that many bytes (the batch buffers: fc2_ingest.cpp's allocator takes them)
Gpu *gpu_open(int device, uint32_t max_blocks, size_t pool_cap, std::string &err);
void gpu_close(Gpu *g);
uint32_t gpu_max_blocks(const Gpu *g);
// A batch of up to max_blocks whole BGZF blocks, inflated into dest back to back (block i at the
// sum of the ISIZEs before it; dest holds max_blocks * 64 KiB): gpu_begin, then gpu_add for each
// chunk of blocks [i0, i1) as they are read (raw + boff[i], bsz[i] bytes each; the chunk's bytes are
// copied, then uploaded, inflated -- CRC-32 and ISIZE checked on the device -- and downloaded while
// the next chunk is read), then gpu_finish, which waits: false (err set) if the device failed.
// Afterwards gpu_status(g, i) == 0 for each block whose bytes are in dest; the others are the CPU's.
void gpu_begin(Gpu *g, char *dest);
bool gpu_add(Gpu *g, const uint8_t *raw, const size_t *boff, const size_t *bsz, size_t i0, size_t i1);
bool gpu_finish(Gpu *g, std::string &err);
uint32_t gpu_status(const Gpu *g, size_t i);

// a pinned buffer of >= n bytes from the pool (nullptr: no pool, too large, or none left)
void *pinned_take(size_t n);
// true if b is one of the pool's buffers
bool pinned_owns(const void *b);
// true if b came from the pool (it goes back to it)
bool pinned_give(void *b);

}  // namespace inf
}  // namespace fc2
