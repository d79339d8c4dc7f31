// Parquet footer / page-header planning on the host (Thrift compact protocol) and a small host
// decoder for the non-file-action checkpoint columns (protocol, metaData, txn), which the
// reference reads through Spark's ParquetFileFormat (D/DeltaLogFileIndex.scala:68). The
// file-action columns (add.*, remove.*) are decoded on the GPU from the plan built here.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace dr {
namespace pq {

enum PhysType { BOOLEAN = 0, INT32 = 1, INT64 = 2, INT96 = 3, FLOAT = 4, DOUBLE = 5, BYTE_ARRAY = 6,
                FIXED_LEN_BYTE_ARRAY = 7 };
enum Repetition { REQUIRED = 0, OPTIONAL = 1, REPEATED = 2 };
enum Codec { UNCOMPRESSED = 0, SNAPPY = 1 };
enum Encoding { PLAIN = 0, PLAIN_DICTIONARY = 2, RLE = 3, BIT_PACKED = 4, RLE_DICTIONARY = 8 };
enum PageType { DATA_PAGE = 0, INDEX_PAGE = 1, DICTIONARY_PAGE = 2, DATA_PAGE_V2 = 3 };

struct SchemaElement {
  int type = -1, type_length = 0, repetition = -1, num_children = 0, converted_type = -1;
  std::string name;
};

// A leaf column with its definition/repetition structure.
struct Leaf {
  std::string path;                 // dotted path, e.g. "add.partitionValues.key_value.key"
  std::vector<std::string> parts;
  int type = -1;
  int max_def = 0, max_rep = 0;
  // def_of[k] = definition level reached when the k-th path component (0-based) is non-null.
  std::vector<int> def_of;
};

struct ColumnChunk {
  int type = -1, codec = 0;
  std::string path;
  int64_t num_values = 0, total_compressed = 0, total_uncompressed = 0;
  int64_t data_page_offset = -1, dictionary_page_offset = -1;
};

struct RowGroup {
  int64_t num_rows = 0;
  std::vector<ColumnChunk> cols;
};

struct FileMeta {
  int64_t num_rows = 0;
  std::vector<SchemaElement> schema;
  std::vector<Leaf> leaves;
  std::vector<RowGroup> row_groups;
  std::string created_by;
  const Leaf* leaf(const std::string& path) const;
  int leaf_index(const std::string& path) const;
};

struct Page {
  int page_type = -1;
  int64_t data_off = 0;            // absolute offset of the (compressed) page body in the file
  int64_t compressed_size = 0, uncompressed_size = 0;
  int32_t num_values = 0;
  int32_t encoding = 0;            // values encoding
  int32_t def_enc = RLE, rep_enc = RLE;
  // DATA_PAGE_V2 only
  int32_t v2_def_len = 0, v2_rep_len = 0, v2_compressed = 1;
};

// Parses the footer of a complete Parquet file (magic "PAR1" at both ends).
FileMeta parse_footer(const uint8_t* file, uint64_t len);
// Walks the page headers of one column chunk.
std::vector<Page> walk_pages(const uint8_t* file, uint64_t len, const ColumnChunk& cc);

// ---- host decode of small columns -----------------------------------------------------------
struct HostColumn {
  std::vector<uint8_t> def, rep;              // one per level
  std::vector<int64_t> ivals;                 // INT32/INT64/BOOLEAN values (non-null only)
  std::vector<std::string> svals;             // BYTE_ARRAY values (non-null only)
};
// Decodes every page of one column chunk (any codec we support: UNCOMPRESSED, SNAPPY).
HostColumn decode_column_host(const uint8_t* file, uint64_t len, const ColumnChunk& cc,
                              const Leaf& leaf);

// Sparse, run-wise decode: one Entry per level whose definition level is >= `thr` (i.e. whose
// ancestor at that level is non-null). Long null runs cost O(1), so a 10M-row checkpoint's
// protocol/metaData/txn columns decode in microseconds.
struct Entry {
  int64_t row;        // row index (row_base + row within the chunk)
  uint8_t def, rep;
  bool has_value;     // def == max_def
  int64_t ival;
  std::string sval;
};
std::vector<Entry> sparse_entries(const uint8_t* file, uint64_t len, const ColumnChunk& cc,
                                  const Leaf& leaf, int thr, int64_t row_base);

}  // namespace pq
}  // namespace dr
