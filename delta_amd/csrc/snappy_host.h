// Host SNAPPY raw-block decompressor (format: varint length preamble, then literal/copy tags).
// Used only for the small non-file-action checkpoint columns decoded on the host
// (protocol/metaData/txn); the file-action columns are decompressed on the GPU.
#pragma once
#include <cstddef>
#include <cstdint>

namespace dr {
// Reads the uncompressed length preamble; returns false on a malformed varint.
bool snappy_uncompressed_length(const uint8_t* in, size_t n, uint64_t* out);
// Decompresses `in[0..n)` into `out[0..out_len)`; returns false on corrupt input.
bool snappy_decompress(const uint8_t* in, size_t n, uint8_t* out, size_t out_len);
}  // namespace dr
