// BAM writer for -B/--bam (spliced_alignments.bam, find_circ.py:479-483, 1134-1140):
// BGZF blocks (SAM/BAM spec 4.1) of up to 0xff00 input bytes, raw-deflated with zlib, the
// empty EOF block at close.  Records come either as BAM bytes copied from a BAM input or
// as SAM text lines encoded the way htslib's sam_parse1 does (what pysam writes for a
// record read from SAM).
#pragma once
#include <stdint.h>

#include <string>
#include <unordered_map>
#include <vector>

namespace fc2 {
namespace bam {

struct Writer;

// header: the input's header text and its reference names / lengths (pysam template=); level: zlib
// level of the BGZF blocks (htslib's default is 6)
Writer *open_writer(const std::string &path, const std::string &text, const std::vector<std::string> &names,
                    const std::vector<int64_t> &lens, std::string &err, int level = 6);
// one BAM record: block_size (4 B) + body, as found in a BAM stream
bool write_raw(Writer *w, const uint8_t *rec, size_t n);
// one SAM text line (no newline); tid_of maps RNAME/RNEXT to reference ids
bool write_sam(Writer *w, const char *line, const char *end, const std::unordered_map<std::string, int> &tid_of,
               std::string &err);
// one SAM text line encoded as write_sam does, appended to rec (block_size + body)
bool encode_sam(const char *line, const char *end, const std::unordered_map<std::string, int> &tid_of,
                std::string &rec, std::string &err);
// record bytes in bulk (BAM records, back to back): the full blocks they complete are deflated on
// `threads` threads and written in order; the blocks are cut where the record-by-record calls would
// cut them, so the file is byte for byte what those calls write
bool write_bulk(Writer *w, const char *p, size_t n, int threads);
// flush, EOF block, close; false on an I/O error
bool close_writer(Writer *w, std::string &err);

}  // namespace bam
}  // namespace fc2
