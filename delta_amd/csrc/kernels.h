// Kernel argument blocks and launchers (host <-> device contract of libdeltareplay).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>

namespace dr {

// ---- per-kernel timing hook (dr_set_timing) -------------------------------------------------------
// Every launcher enqueues through DR_LAUNCH; when a hook is installed (thread-local: one dr_ctx per
// host thread) and selects the kernel, the launch carries a HIP event pair in its own dispatch, so
// per-kernel device times are exact and need no profiler.
// Per-launch timing hook (dr_set_timing): for a launch the hook selects, it hands out an event
// pair that the launch carries in its own dispatch (hipExtLaunchKernel: the kernel's start and end
// timestamps, no marker packets between kernels, so the timed steps run as the untimed ones do).
typedef bool (*LaunchHook)(void* user, const char* kernel, hipEvent_t* start, hipEvent_t* stop);
void set_launch_hook(LaunchHook hook, void* user);
bool launch_events(const char* kernel, hipEvent_t* start, hipEvent_t* stop);
void launch_grid_check(const char* kernel, dim3 grid, dim3 block);
// A dispatch's work-item count per dimension is 32-bit: a larger grid would silently run a wrapped
// fraction of itself, so it is refused (launch_grid_check throws).
#define DR_LAUNCH(K, GRID, BLOCK, SHM, ST, ...)                                     \
  do {                                                                              \
    ::dr::launch_grid_check(#K, dim3(GRID), dim3(BLOCK));                           \
    hipEvent_t dr_e0_ = nullptr, dr_e1_ = nullptr;                                  \
    if (::dr::launch_events(#K, &dr_e0_, &dr_e1_))                                  \
      hipExtLaunchKernelGGL(K, GRID, BLOCK, SHM, ST, dr_e0_, dr_e1_, 0u, __VA_ARGS__); \
    else                                                                            \
      hipLaunchKernelGGL(K, GRID, BLOCK, SHM, ST, __VA_ARGS__);                     \
  } while (0)

// Per-action SoA arrays in HBM; action index = checkpoint rows first, then JSON lines (the
// reference's replay order: D/Snapshot.scala:102-104 sorts by input file name).
struct ActionArrays {
  uint8_t* kind;
  uint8_t* flags;
  uint64_t* key;        // xxh64(canonical path) | (==0)
  uint64_t* path_ptr;   // device address of the canonical path bytes
  uint32_t* path_len;
  int64_t* size;
  int64_t* delts;
  uint64_t* src_off;    // JSON: line offset in the JSON buffer; checkpoint: row index
  uint32_t* src_len;    // JSON: line length
  // nullable: the packed path reference (path address | length << 48, 0 for a length >= 0xffff) that
  // k_bucket_verify gathers, written by the producers beside path_ptr / path_len (so K3 need not
  // re-read them); states built without it get it from k_bucket_hist
  uint64_t* path_ref = nullptr;
};

struct JsonParseArgs {
  const uint8_t* buf;
  const uint64_t* nl;
  uint64_t nlines;
  uint64_t base;        // action index of the first JSON line
  uint8_t* kind;
  uint8_t* flags;
  uint64_t* key;
  uint64_t* path_ptr;
  uint32_t* path_len;
  int64_t* size;
  int64_t* delts;
  uint64_t* src_off;
  uint32_t* src_len;
  uint64_t* special_count;
  uint64_t* special_bytes;
  uint64_t* nonfile_count;
  uint64_t* nonfile_idx;          // {line, byte offset} per protocol / metaData / txn line
  uint64_t nonfile_cap;           // entries (pairs)
  uint64_t* error_count;
  uint64_t* hard_idx;             // lines the fast walker defers to the General walker
  unsigned long long* hard_count;
  unsigned long long* phase;      // diagnostics (DR_JSON_PHASES): staged kernel phase clocks, or null
  // a segment of one wave (JSON_FUSE_MAX_LINES lines, one index block): the newline index and the
  // counter reset run inside the parse kernel -- nl and off2 = {0, lines} are written by it and
  // zero[0..nzero) cleared (null zero: launch_json_index1 / the block index ran before)
  uint64_t buf_len;
  uint64_t* zero;
  uint32_t nzero;
  uint64_t* off2;
  uint64_t* nl_out;  // = nl, writable (the fused index)
  uint32_t force_staged;  // (host side) DR_OPT_JSON_STAGED: the staged kernel for every segment
  uint64_t* path_ref;     // nullable: ActionArrays::path_ref
};
constexpr uint64_t JSON_FUSE_MAX_LINES = 64;

uint64_t json_num_blocks(uint64_t len);
// newline index: per-block counts + u16 slots (json_slot_entries), then the global positions
uint64_t json_slot_entries(uint64_t len);
void launch_json_index(const uint8_t* buf, uint64_t len, uint32_t* block_counts, uint16_t* slots, hipStream_t st);
void launch_json_place(const uint8_t* buf, uint64_t len, const uint32_t* block_counts, const uint64_t* block_off,
                       const uint16_t* slots, uint64_t* nl, hipStream_t st);
// one-block segments (len <= 16 KiB): newline positions straight into nl, off2 = {0, count}, and
// zero[0..nzero) cleared
void launch_json_index1(const uint8_t* buf, uint64_t len, uint64_t* nl, uint64_t* off2, uint64_t* zero,
                        uint32_t nzero, hipStream_t st);
void launch_json_parse(const JsonParseArgs& a, hipStream_t st);
void launch_json_hard(const JsonParseArgs& a, hipStream_t st);

// ---- scans ------------------------------------------------------------------------------------
// Exclusive scan of n u32 counts into u64 offsets; out[n] = total. Scratch: scan_scratch_bytes(n);
// a scratch smaller than that is refused (std::runtime_error -> DR_E_INTERNAL) instead of overrun.
uint64_t scan_scratch_bytes(uint64_t n);
struct ScanScratch {
  void* p = nullptr;
  uint64_t bytes = 0;
};
void launch_scan_u32(const uint32_t* in, uint64_t* out, uint64_t n, ScanScratch scratch, hipStream_t st);

// ---- Parquet (K2) -------------------------------------------------------------------------------
enum PageKind : int32_t { PG_DATA_V1 = 0, PG_DICT = 2, PG_DATA_V2 = 3 };

struct PageDesc {
  uint64_t src;          // device address of the page body (compressed)
  uint64_t dst;          // device address of the decompressed body in the arena
  uint32_t csize, usize;
  uint32_t num_values;   // levels in the page (= rows for flat columns)
  int32_t kind;          // PageKind
  int32_t encoding;
  int32_t codec;         // 0 uncompressed, 1 snappy
  int32_t col;           // output column slot
  int32_t phys;          // physical type
  int32_t max_def;
  int32_t max_rep;       // > 0: repeated leaf (map key/value); row_base then counts level entries
  int32_t dict;          // index (into the page table) of this chunk's dictionary page, -1 none
  uint64_t row_base;     // first checkpoint row of the page (flat columns)
  int32_t v2_def_len, v2_rep_len, v2_compressed;
  uint32_t dict_base;    // dictionary pages: first slot in the dictionary pool
  // PLAIN BYTE_ARRAY pages (data or dictionary): parallel boundary detection scratch
  int32_t ba;            // 1 if this page's values are length-prefixed byte arrays
  uint32_t ba_slot;      // index into ba_ok / ba_count
  uint64_t ba_base;      // first u32 slot of this page's value offsets
  uint64_t hit_base;     // index of this page's first 4 KiB boundary tile (ParquetArgs::ba_tiles)
};

// Decoded column: one entry per checkpoint row (flat leaf) or per level entry (repeated leaf).
struct FlatColumn {
  uint8_t* def;          // definition level per row / entry
  uint8_t* rep;          // repetition level per entry (repeated leaves only)
  int64_t* ival;         // INT64/INT32/BOOLEAN value (valid where def == max_def)
  uint64_t* sptr;        // BYTE_ARRAY: device address of the value bytes
  uint32_t* slen;
};

struct ParquetArgs {
  PageDesc* pages;
  uint32_t npages;
  FlatColumn cols[8];
  int32_t ncols;
  uint64_t* dict_ptr;    // dictionary pool (BYTE_ARRAY: address; INT: value)
  uint32_t* dict_len;
  uint32_t* error;       // first error code (0 = ok)
  uint32_t* ba_vals;     // value offsets (relative to the page's decompressed body)
  uint32_t* ba_hit;      // unused (kept for layout)
  uint32_t* ba_ok;       // [pages with ba] 1 = boundaries found and validated
  uint32_t* ba_count;    // [pages with ba] number of values found
  const uint2* ba_tiles; // [nba_tiles] (page index, tile index within the page's value region)
  uint32_t nba_tiles;
  uint32_t* ba_tile_cnt; // [nba_tiles]
  uint64_t* ba_tile_off; // [nba_tiles + 1] exclusive scan of ba_tile_cnt
  uint64_t* ba_kept;     // [nba_tiles * 256] kept-candidate masks (64 positions per thread)
  uint32_t* ba_link;     // [nba_tiles * 3] the tile's first kept offset, its last kept's successor
                         // (0xFFFFFFFF: none) and whether its chain broke inside it
};
uint32_t ba_tile_bytes();
void launch_ba_bounds(const ParquetArgs& a, hipStream_t st, ScanScratch scan_scratch);

// SNAPPY pages (k_snappy.hip). `in` points past the varint length preamble.
struct SnapPage {
  uint64_t in, out;      // device addresses
  uint32_t n_in, n_out;
  uint32_t block_base;   // first 64 KiB output block of this page in the block table
};
struct CopyJob { uint64_t src, dst, n; };
struct SnappyArgs {
  const SnapPage* pages;
  uint32_t npages;
  const uint32_t* chunk_base;   // [npages + 1] first speculation chunk of each page
  uint32_t nchunks;
  uint32_t* spec_exit;          // [nchunks]
  uint32_t* vis;                // [nchunks * 8] visited-position bitmaps
  uint32_t* entry;              // [nchunks] true first element position >= chunk start
  uint32_t* spec_first;         // [nchunks] first speculatively visited position >= chunk start
  uint32_t* assumed_exit;       // [nchunks] exit assuming the previous chunk's speculative exit
  uint8_t* chunk_flag;          // [nchunks] 1: serial resolution from this chunk
  uint32_t* region;             // [npages] pages holding a serially resolved region (k_snap_regions)
  unsigned long long* region_count;
  uint32_t* page_mark;          // [npages] zeroed per replay: the page is listed in region[]
  uint32_t* chunk_out;          // [nchunks] output bytes of the chunk's elements
  uint32_t* chunk_out_start;    // [nchunks] page-relative output offset of the chunk's first element
  uint32_t* chunk_elems;        // [nchunks] elements per chunk (statistics)
  const uint32_t* block_page;   // [nblocks]
  uint32_t* block_chunk;        // [nblocks] chunk holding each output block's first element (k_snap_scan)
  uint32_t nblocks;
  const uint32_t* wg_chunk0;    // [nwg] first chunk (global index) of each chunk-walker workgroup
  uint32_t nwg;
  uint32_t* pages_bad;          // [npages] nonzero -> decoded by the serial fallback
  uint32_t* error;
  const uint32_t* chunk_page;   // [nchunks] page of each chunk
  uint64_t* stamps = nullptr;   // diagnostics: [nblocks * 8] k_snap_exec phase clocks, or null
  uint64_t* rstats = nullptr;   // diagnostics: [regions * 4] k_snap_resolve {clocks, windows, walks, spans}, or null
};
uint32_t snappy_wg_chunks();
uint32_t snappy_chunk_bytes();
void launch_snappy(const SnappyArgs& a, hipStream_t st, ScanScratch scan_scratch);
void launch_page_copy(const CopyJob* jobs, uint32_t njobs, hipStream_t st);

void launch_pq_dict(const ParquetArgs& a, hipStream_t st);
void launch_pq_data(const ParquetArgs& a, hipStream_t st);

// Checkpoint row assembly: flat columns -> action arrays.
struct CkptAssembleArgs {
  FlatColumn add_path, add_size, rm_path, rm_delts;
  int32_t add_def, rm_def;              // def level at which add / remove is non-null
  int32_t add_path_max, add_size_max, rm_path_max, rm_delts_max;
  int32_t has_rm;                       // checkpoint has a remove column
  uint64_t nrows;
  uint64_t row_base;                    // action index of checkpoint row 0
  ActionArrays act;
  uint64_t* special_count;
  uint64_t* special_bytes;
};
void launch_ckpt_assemble(const CkptAssembleArgs& a, hipStream_t st);

// ---- canonicalization of special paths ---------------------------------------------------------
struct CanonArgs {
  ActionArrays act;
  uint64_t n;
  uint8_t* arena;
  uint64_t arena_cap;
  uint64_t* arena_fill;
};
void launch_canon(const CanonArgs& a, hipStream_t st);
// a commit-only segment of at most JSON_TAIL_POST_MAX actions: k_json_hard + k_canon in one workgroup
constexpr uint64_t JSON_TAIL_POST_MAX = 256;
void launch_tail_post(const JsonParseArgs& a, const CanonArgs& c, hipStream_t st);

// ---- K3/K4: partition by hash bucket + per-bucket last-writer-wins ------------------------------
// A partition record is 16 B: {xxh64(path) lo, hi, meta = action index << 2 | class, add.size when it
// fits 32 bits (else ~0u: the reducer reads size[] by index)}. Tiles of PART_TILE actions count
// their buckets in LDS into a bucket-major count matrix; its exclusive scan gives every (bucket,
// tile) its output range, so the scatter needs no global atomics.
struct PartRec {
  uint32_t key_lo;
  uint32_t key_hi;
  uint32_t meta;
  uint32_t size;
};
struct PartitionArgs {
  const uint8_t* kind;
  const uint8_t* flags;
  const uint64_t* key;
  const int64_t* size;
  const int64_t* delts;
  uint64_t n;
  int64_t cutoff;              // minFileRetentionTimestamp
  int32_t bucket_bits;
  uint32_t ntiles;
  uint32_t* tile_count;        // [nbuckets * ntiles] bucket-major counts
  const uint64_t* tile_off;    // [nbuckets * ntiles + 1] exclusive scan of tile_count
  PartRec* rec;                // partitioned records
  const uint64_t* path_ptr;
  const uint32_t* path_len;
  uint64_t* path_ref;          // per action: path address | length << 48 (0: length >= 0xffff)
};
uint32_t part_tiles(uint64_t n);
uint32_t part_max_bucket_bits();
void launch_bucket_hist(const PartitionArgs& a, hipStream_t st);
void launch_bucket_scatter(const PartitionArgs& a, hipStream_t st);
// bucket_off[b] = tile_off[b * ntiles], b in [0, nbuckets]
void launch_bucket_offsets(const uint64_t* tile_off, uint32_t nbuckets, uint32_t ntiles, uint64_t* bucket_off,
                           hipStream_t st);

struct ReduceArgs {
  const PartRec* rec;
  const uint64_t* bucket_off;  // [nbuckets + 1]
  uint32_t nbuckets;
  int32_t bucket_bits;
  const int64_t* size;         // add.size by action index (records whose size field overflowed)
  const uint64_t* path_ptr;    // by action index (fallback reducers only)
  const uint32_t* path_len;
  uint32_t* out_live;          // per-bucket survivors, written at bucket_off[b]
  uint32_t* out_tomb;
  uint2* out_pair;             // per-bucket (loser, winner) action indices for k_bucket_verify
  const uint64_t* path_ref;    // PartitionArgs::path_ref
  uint32_t* live_count;        // [nbuckets]
  uint32_t* tomb_count;        // [nbuckets]
  uint32_t* pair_count;        // [nbuckets]
  unsigned long long* totals;  // [0] live files, [1] size sum, [2] tombstones, [3] buckets for the 64-bit
                               // reducer, [4] buckets for the exact reducer, [5] live / [6] tombstone checksum
  uint32_t* redo_list;         // buckets whose LDS table overflowed
  uint32_t* exact_list;        // buckets with a 64-bit path-hash collision (or an unpackable path)
  unsigned long long* bstats;  // [nbuckets * 5] per-bucket {live, tomb, size, live sum, tomb sum}
  unsigned long long* vstats;  // nullable (timed replays): [nbuckets * 2] k_bucket_verify's {pairs, path bytes compared}
};
// K3 refinement for large replays: bucket b's records into 2^sbits sub-buckets by the next key bits
// (bucket_of(key, bits + sbits)); out_off[b * 2^sbits + j] = the sub-buckets' offsets, [nb << sbits] = end
struct SplitArgs {
  const PartRec* rec;
  const uint64_t* bucket_off;  // [nbuckets + 1]
  int32_t bits, sbits;
  PartRec* out;
  uint64_t* out_off;           // [(nbuckets << sbits) + 1]
};
void launch_bucket_split(const SplitArgs& a, uint32_t nbuckets, hipStream_t st);
// LDS last-writer-wins per bucket on the 64-bit key; losers paired with winners (grouped by winner)
void launch_bucket_reduce(const ReduceArgs& a, hipStream_t st);
// byte-verifies every (loser, winner) pair; mismatching buckets (64-bit collisions) -> exact_list
void launch_bucket_verify(const ReduceArgs& a, hipStream_t st);
// redo_list buckets in finer sub-passes; collisions -> exact_list
// `count` (device, nullable): the list's length when only its bound nb is known on the host
void launch_bucket_reduce64(const ReduceArgs& a, const uint32_t* buckets, uint32_t nb, hipStream_t st,
                            const unsigned long long* count = nullptr);
// exact O(m^2) reducer
void launch_bucket_exact(const ReduceArgs& a, const uint32_t* buckets, uint32_t nb, hipStream_t st,
                         const unsigned long long* count = nullptr);
// sums the per-bucket statistics into totals[0,1,2,5,6]
void launch_sum_stats(const ReduceArgs& a, hipStream_t st);

// Compaction of per-bucket survivor lists into dense arrays.
struct CompactArgs {
  const uint32_t* src;
  const uint64_t* bucket_off;
  const uint32_t* counts;
  const uint64_t* dst_off;   // exclusive scan of counts
  uint32_t nbuckets;
  uint32_t* dst;
};
void launch_compact(const CompactArgs& a, hipStream_t st);
// both survivor lists in one launch (nbuckets must match)
void launch_compact2(const CompactArgs& live, const CompactArgs& tomb, hipStream_t st);
// exclusive scans (+ totals at [nb]) of the live / tombstone counts, one workgroup; with bstats also
// the reducer's per-bucket sums into totals (what k_sum_stats did)
void launch_survivor_scan(const uint32_t* lc, const uint32_t* tc, uint32_t nb, uint64_t* loff, uint64_t* toff,
                          hipStream_t st, const unsigned long long* bstats = nullptr,
                          unsigned long long* totals = nullptr);

// ---- multi-GPU path-hash sharding (k_shard.hip) ------------------------------------------------
struct ShardRec {        // 32 B per exchanged file action (DR_SHARD_REC_BYTES)
  uint64_t key;
  int64_t size;
  int64_t delts;
  uint32_t plen;
  uint8_t kind, flags;
  uint16_t pad;
};
static_assert(sizeof(ShardRec) == 32, "ShardRec layout");

struct ShardArgs {
  const uint8_t* kind;
  const uint8_t* flags;
  const uint64_t* key;
  const int64_t* size;
  const int64_t* delts;
  const uint32_t* path_len;
  uint64_t n;
  uint32_t world;
  uint64_t ntiles;
  uint32_t* blk_count;       // [world * ntiles] owner-major
  const uint64_t* blk_off;   // exclusive scan of blk_count
  uint32_t* send_idx;        // [nsend] local action index of each send slot
  uint64_t nsend;
  uint32_t* blk_bytes;       // [world * ntiles] canonical path bytes per (owner, tile); may be null
};
uint64_t shard_tiles(uint64_t n);
uint32_t shard_max_world();
void launch_shard_count(const ShardArgs& a, hipStream_t st);
void launch_shard_scatter(const ShardArgs& a, hipStream_t st);
void launch_shard_pack(const ShardArgs& a, ShardRec* rec, uint32_t* plen, hipStream_t st);
void launch_shard_plen(const ShardRec* rec, uint64_t n, uint32_t* plen, hipStream_t st);
void launch_shard_unpack(const ShardRec* rec, uint64_t n, const uint8_t* path_base, const uint64_t* poff,
                         const ActionArrays& act, hipStream_t st);
// n_dev: the list's length on the device (<= n), or null for n
void launch_verdict_set(const uint32_t* idx, uint64_t n, const unsigned long long* n_dev, uint8_t v, uint8_t* verdict,
                        hipStream_t st);
// out[d] = records, out[world + d] = path bytes this rank sends to owner d (from the scanned matrices),
// out[2 world] = 1 when a tile's byte count saturated (more than 4 GiB of paths in one tile)
void launch_shard_sizes(const uint32_t* blk_bytes, const uint64_t* blk_off, const uint64_t* byte_off, uint32_t world,
                        uint64_t ntiles, uint64_t* out, hipStream_t st);
// the 8 partial sums of the table-wide counter all-reduce (num_files, size_in_bytes, num_removes,
// num_actions, num_file_actions, malformed_lines, live_key_sum, tomb_key_sum)
void launch_shard_partials(const unsigned long long* totals, const uint64_t* parse_ctr, int64_t n_actions,
                           int64_t* out, hipStream_t st);
void launch_verdict_flags(const uint8_t* verdict, uint64_t n, uint32_t* f_live, uint32_t* f_tomb, hipStream_t st);
void launch_verdict_collect(const uint8_t* verdict, const uint32_t* send_idx, uint64_t n, uint8_t want,
                            const uint64_t* pos, uint32_t* out, hipStream_t st);

// ---- K5: partition pruning (k_filter.hip) -------------------------------------------------------
// Two kernels: k_pv_extract builds, once per state and partition column, the column's values cast to
// the column type for every live AddFile (the state's K5 cache); k_filter_typed evaluates a
// predicate program over those typed columns, so a filter reads 4-12 B per file and column.
constexpr int PV_MAXC = 16;
struct PvColumn {
  int32_t type;        // dr_pred_type (DECIMAL: | precision << 8 | scale << 16)
  uint32_t* w32;       // BYTE / SHORT / INT / DATE (days) / BOOLEAN (0/1) / FLOAT (bits)
  int64_t* w64;        // LONG / DOUBLE (bits) / TIMESTAMP (micros, UTC) / DECIMAL (unscaled, low 64 bits)
  uint64_t* sptr;      // STRING: address of the (unescaped) value bytes
  uint32_t* slen;
  uint8_t* isnull;     // 1: NULL (absent, JSON null, or a failed non-ANSI cast)
  uint64_t* s8;        // STRING: the first 8 bytes, big-endian, zero-padded (compared without a gather)
  int64_t* w64hi;      // DECIMAL: unscaled high 64 bits (two's complement 128-bit value)
  uint64_t* hard;      // FLOAT / DOUBLE: {row, value address, length} of values the host converts
  unsigned long long* nhard;
};
struct PvExtractArgs {
  const uint32_t* live;          // live AddFile action indices (export order)
  uint64_t n_live;
  const uint64_t* src_off;       // JSON: line offset; checkpoint: row
  const uint32_t* src_len;
  uint64_t ck_rows;              // actions below this index are checkpoint rows
  const uint8_t* json;           // staged JSON bytes
  // states built by dr_state_apply: checkpoint rows are told by F_FROM_CKPT and JSON lines are
  // read from the staged bytes of their source (null: single segment, the fields above)
  const uint8_t* act_flags;
  const uint16_t* src_id;
  const uint64_t* json_bases;
  // checkpoint add.partitionValues map (level entries)
  int32_t has_map;
  const uint64_t* row_start;     // [ck_rows + 1]
  const uint8_t* key_def;
  const uint64_t* key_ptr;
  const uint32_t* key_len;
  int32_t key_max_def;
  const uint8_t* val_def;
  const uint64_t* val_ptr;
  const uint32_t* val_len;
  int32_t val_max_def;
  // the columns to build (names = exact map keys)
  int32_t ncols;
  const uint64_t* col_name_off;  // [ncols + 1]
  const uint8_t* col_names;
  PvColumn cols[PV_MAXC];
  // unescaped JSON values (null arena: count the bytes needed into arena_need)
  uint8_t* arena;
  uint64_t arena_cap;
  unsigned long long* arena_fill;
  unsigned long long* arena_need;
  uint32_t* error;
};
struct FilterTypedArgs {
  uint64_t n_live;
  int32_t ncols;
  PvColumn cols[PV_MAXC];        // predicate column k -> its typed cache column
  int32_t nops;
  const int32_t* ops;            // [nops * 2] opcode, arg (lowered program)
  const int32_t* lit_types;
  const int64_t* lit_i64;
  const uint8_t* lit_null;
  const uint64_t* lit_str_off;   // [nlits + 1]
  const uint8_t* lit_str;
  uint32_t* flag;                // [n_live] 1 = selected
};
// Leaf form of a predicate (engine.hip leafify): every leaf compares one partition column with
// literals -- col op lit, col IN (lits), col IS [NOT] NULL -- and AND / OR / NOT combine their
// three-valued results on a 2-bit-per-entry stack held in one register.
struct FilterLeaf {
  int32_t col;       // predicate column
  int32_t op;        // DR_OP_EQ .. DR_OP_GE, DR_OP_NSEQ, DR_OP_IN, DR_OP_ISNULL, DR_OP_ISNOTNULL
  int32_t lit;       // literal index (comparisons) or first entry of the sorted set (IN)
  int32_t nlit;      // IN: entries in the set
  int32_t lit_null;  // comparisons: the literal is NULL; IN: the list holds a NULL
  int32_t pad;       // IN over integers: 1 = a bitmap (literals [min, words, bits...])
  int32_t slot;      // k_filter_leaf: the preloaded column slot holding `col` (-1: loaded per leaf)
  int32_t ctype;     // the column's dr_pred_type
};
enum : int32_t { LEAF_OP_LEAF = 0, LEAF_OP_AND = 1, LEAF_OP_OR = 2, LEAF_OP_NOT = 3 };
struct FilterLeafArgs {
  uint64_t n_live;
  PvColumn cols[PV_MAXC];
  const FilterLeaf* leaves;
  const int32_t* prog;           // [nprog * 2] opcode, arg (leaf index)
  int32_t nprog;
  const int64_t* lit_i64;        // comparison literals, then the IN sets (sorted ascending)
  const uint64_t* lit_str_off;   // string literals / sets (sorted bytewise), offsets into lit_str
  const uint8_t* lit_str;
  const uint64_t* lit_s8;        // per string literal: its first 8 bytes as PvColumn::s8
  int32_t n_i64, n_str;          // literal counts
  uint64_t* mask;                // [filter_leaf_mask_words() per tile] selection bits, one u64 per 64 files in file order
  uint32_t* wg_count;            // [tiles] selected files of each 1024-file tile (zeroed before the launch)
  int32_t nleaves;
  int32_t nucol;                 // distinct columns the leaves read (0: more than FL_UCOLS, loaded per leaf)
  int32_t ucol[4];               // FL_UCOLS: those columns (predicate column indices)
};
constexpr int FL_UCOLS = 4;
uint32_t filter_leaf_max_prog();
uint32_t filter_leaf_max_i64();   // literals k_filter_leaf holds in LDS (more: k_filter_typed)
uint32_t filter_leaf_max_str();
uint32_t filter_leaf_max_leaves();
// 1024-file tiles of k_filter_leaf: the sizes of `mask` (x16) and `wg_count`
uint64_t filter_leaf_groups(uint64_t n_live);
uint32_t filter_leaf_mask_words();  // mask words per tile
void launch_filter_leaf(const FilterLeafArgs& a, hipStream_t st);
// out[wg_off[g] + rank] = ordinal of every selected file (wg_off: exclusive scan of wg_count)
void launch_select_bits(const uint64_t* mask, const uint64_t* wg_off, uint64_t n, int64_t* out, hipStream_t st);
// device-only opcodes of the lowered program (engine.hip lower_program): an IN list is folded
// one element at a time into an accumulator slot above its value
enum : int32_t { FILTER_OP_IN_START = 100, FILTER_OP_IN_STEP = 101, FILTER_OP_IN_END = 102 };
uint32_t filter_max_cols();
// ---- K5 dictionary path: each partition column's distinct values get u16 codes (code 0: NULL), a
// leaf becomes a table over its column's codes, and the per-file pass reads 2 bytes per column.
constexpr uint32_t DICT_SLOTS = 1u << 17;   // global hash table (load <= 1/2)
constexpr uint32_t DICT_MAX = 65535;        // codes 1..DICT_MAX-1 for values, 0 for NULL
struct PvDictArgs {
  uint64_t n;
  PvColumn col;              // the typed column (its type field: the dr_pred_type)
  uint64_t* key_tab;         // [DICT_SLOTS] keys
  uint32_t* tag_tab;         // [DICT_SLOTS] 0 empty, 0xffffffff being written, 1 + representative row
  uint32_t* slot_code;       // [DICT_SLOTS] code of an occupied slot
  uint16_t* code;            // [n]
  uint32_t* rep;             // [DICT_MAX + 1] representative row of each code
  unsigned long long* ctr;   // 0: occupied slots, 1: table full / verification failed
};
void launch_dict_insert(const PvDictArgs& a, hipStream_t st);
void launch_dict_number(const PvDictArgs& a, const uint64_t* scan, hipStream_t st);   // after a scan of occupancy
void launch_dict_occupied(const PvDictArgs& a, uint32_t* occ, hipStream_t st);
void launch_dict_code(const PvDictArgs& a, hipStream_t st);
struct DictLeafArgs {
  const FilterLeaf* leaves;
  int32_t nleaves;
  PvColumn cols[PV_MAXC];
  const uint32_t* rep[PV_MAXC];  // per predicate column: representative rows (null: no dictionary)
  uint32_t ncode[PV_MAXC];       // codes per column (incl. code 0)
  const uint32_t* tab_off;       // [nleaves + 1] table offsets
  uint8_t* tab;                  // leaf results (0 false, 1 true, 2 null) per (leaf, code)
  const int64_t* lit_i64;
  const uint64_t* lit_s8;
  const uint64_t* lit_str_off;
  const uint8_t* lit_str;
  uint64_t n_live;
};
void launch_dict_leaf(const DictLeafArgs& a, uint32_t total, hipStream_t st);
struct FilterDictArgs {
  uint64_t n_live;
  const uint16_t* code[FL_UCOLS];  // per slot: the column's codes
  int32_t nslot;
  const FilterLeaf* leaves;        // leaf.slot: the code slot it reads
  int32_t nleaves;
  const int32_t* prog;
  int32_t nprog;
  const uint32_t* tab_off;
  const uint8_t* tab;
  uint32_t tab_bytes;
  uint64_t* mask;
  uint32_t* wg_count;
};
uint32_t filter_dict_max_tab();   // leaf-table bytes the dictionary kernel holds in LDS
void launch_filter_dict(const FilterDictArgs& a, hipStream_t st);
uint32_t filter_max_stack();
void launch_pv_extract(const PvExtractArgs& a, hipStream_t st);
void launch_filter_typed(const FilterTypedArgs& a, hipStream_t st);
void launch_rep0_flags(const uint8_t* rep, uint64_t n, uint32_t* f, hipStream_t st);
void launch_row_starts(const uint8_t* rep, uint64_t n, const uint64_t* pos, uint64_t* row_start, hipStream_t st);
void launch_select(const uint32_t* flag, const uint64_t* pos, uint64_t n, int64_t* out, hipStream_t st);

}  // namespace dr

namespace dr {
void launch_gather_u64(const uint64_t* src, const uint32_t* idx, uint64_t n, uint64_t* dst, hipStream_t st);
void launch_gather_u32(const uint32_t* src, const uint32_t* idx, uint64_t n, uint32_t* dst, hipStream_t st);
void launch_gather_u8(const uint8_t* src, const uint32_t* idx, uint64_t n, uint8_t* dst, hipStream_t st);
void launch_gather_u16(const uint16_t* src, const uint32_t* idx, uint64_t n, uint16_t* dst, hipStream_t st);
void launch_iota_u32(uint32_t* out, uint64_t n, hipStream_t st);
void launch_gather_u64_by64(const uint64_t* src, const uint64_t* idx, uint64_t n, uint64_t* dst, hipStream_t st);
void launch_gather_bytes(const uint64_t* ptr, const uint32_t* len, const uint64_t* off, uint64_t n, uint8_t* out,
                         hipStream_t st);
// n actions from src to dst (both arrays already offset), dst src_id = sid
struct AppendArgs {
  ActionArrays src, dst;
  uint16_t* src_id;
  uint64_t n;
  uint16_t sid;
  // the index counters the apply's next kernels accumulate into: ctr[0..nctr) = 0 but
  // ctr[ctr_at] = ctr_val (null ctr: none), set by the same launch instead of an upload
  unsigned long long* ctr;
  uint32_t nctr, ctr_at;
  unsigned long long ctr_val;
};
void launch_append_actions(const AppendArgs& a, hipStream_t st);
// Device words into pinned host memory, several spans in one launch (an apply's counters and
// non-file line list: one dispatch instead of a copy per span)
constexpr int READBACK_SPANS = 4;
struct ReadbackArgs {
  const uint64_t* src[READBACK_SPANS];
  uint64_t* dst[READBACK_SPANS];
  uint32_t n[READBACK_SPANS];
  // with flag: *flag = seq once every span is written and fenced to the system (the host spins on
  // it instead of a stream synchronize)
  uint64_t* flag;
  uint64_t seq;
};
void launch_readback(const ReadbackArgs& a, hipStream_t st);
// dst[i] = src[i] - base (n entries)
void launch_rebase_i64(const int64_t* src, uint64_t n, int64_t base, int64_t* dst, hipStream_t st);
// a list of distinct indices below nbits sorted ascending: mark its bits in bm (zeroed, ceil(nbits / 32)
// words), the words' popcounts into cnt, and (after an exclusive scan of cnt into off) every word's
// indices written at its offset
void launch_bits_mark(const uint32_t* list, uint64_t n, uint64_t nbits, uint32_t* bm, hipStream_t st);
void launch_bits_popc(const uint32_t* bm, uint64_t w, uint32_t* cnt, hipStream_t st);
void launch_bits_emit(const uint32_t* bm, uint64_t w, const uint64_t* off, uint32_t* out, hipStream_t st);
// export: valid[i] = flags[i] & F_HAS_DELTS, out[i] = valid ? delts[i] : 0
void launch_delts_fix(const uint8_t* flags, const int64_t* delts, uint64_t n, uint8_t* valid, int64_t* out,
                      hipStream_t st);
// isnull[rows[k]] = nulls[k] and w32[rows[k]] = low 32 bits of bits[k] (w32 given) or w64[rows[k]] = bits[k]
void launch_scatter_fp(const uint64_t* rows, const uint64_t* bits, const uint8_t* nulls, uint64_t n, uint32_t* w32,
                       int64_t* w64, uint8_t* isnull, hipStream_t st);
}  // namespace dr

// ---- incremental tail apply: device-resident path index (k_index.hip) ----------------------------
namespace dr {
// One chain of states built by dr_state_apply shares an append-only action store and an
// open-addressing table {path key -> winning action + 1}. A tail's file actions probe and update
// only their own keys; the counters move by the difference of old and new winners' contributions.
struct IndexArgs {
  const uint8_t* kind;
  const uint8_t* flags;
  const uint64_t* key;
  const uint64_t* path_ptr;
  const uint32_t* path_len;
  const int64_t* size;
  const int64_t* delts;
  unsigned long long* keys;  // table: 0 = empty (path_key is never 0)
  uint32_t* vals;            // winner action + 1 (0: none)
  uint64_t mask;             // capacity - 1 (capacity a power of two, load <= 1/2)
  uint64_t lo, hi;           // the action range being inserted / applied
  uint32_t* t_slot;          // per action in [lo, hi): its slot (0xffffffff: not a file action)
  uint32_t* t_prev;          // per action: the slot's value before it (atomicMax)
  int64_t old_cut, new_cut;  // retention cutoffs of the base and the new state
  unsigned long long* ctr;   // IX_C_* counters
  ulonglong2* tomb_list;     // tombstone candidates {action index, deletionTimestamp}, appended at
                             // ctr[IX_C_TOMB_FILL] (the timestamp inline: the expiry's filter is one load)
  uint64_t tomb_cap;
  uint2* undo;               // first touches of this apply: {action, previous value}
};
enum : int {
  IX_C_FILES = 0, IX_C_SIZE = 1, IX_C_REMOVES = 2, IX_C_LKS = 3, IX_C_TKS = 4, IX_C_COLLIDE = 5,
  IX_C_FILE_ACTIONS = 6, IX_C_NEW_SLOTS = 7, IX_C_TOMB_FILL = 8, IX_C_UNDO_FILL = 9, IX_C_DONE = 10, IX_C_N = 16
};
void launch_ix_build(const IndexArgs& a, hipStream_t st);
void launch_ix_touch(const IndexArgs& a, hipStream_t st);
void launch_ix_delta(const IndexArgs& a, hipStream_t st);
// with rb (spans given): the last workgroup to finish also writes the readback spans (the counters
// are final then), instead of a launch_readback after it
void launch_ix_expire(const IndexArgs& a, uint64_t n_list, hipStream_t st, const ReadbackArgs* rb = nullptr);
// A tail of at most IX_T actions in one workgroup: the parse's deferred work (General walker,
// canonicalisation; skipped when ja is null), the append to the chain store with the counters'
// reset, and both index passes -- k_tail_post + k_append_actions + k_ix_touch_delta in one launch
constexpr uint64_t APPLY_SMALL_MAX = 256;
// the one-launch apply also expires a tombstone-candidate list up to this long (one workgroup)
constexpr uint64_t APPLY_FUSED_EXPIRY_MAX = 8192;
void launch_apply_small(const JsonParseArgs* ja, const CanonArgs& cg, const AppendArgs& ap, const IndexArgs& ix,
                        hipStream_t st);
// ... and the line walk itself, for a segment of one wave (ja in the fused-index form: zero, off2,
// nl_out given; JSON_FUSE_MAX_LINES lines in one index block): the whole apply in one launch, with the
// expiry of the first exp_n tombstone candidates and the readback `rb` (when given) after it
void launch_apply_commit(const JsonParseArgs& ja, const CanonArgs& cg, const AppendArgs& ap, const IndexArgs& ix,
                         hipStream_t st, uint64_t exp_n = 0, const ReadbackArgs* rb = nullptr);
void launch_ix_tomb_compact(const IndexArgs& a, const ulonglong2* list_in, uint64_t n, ulonglong2* list_out,
                            hipStream_t st);
void launch_ix_undo(const IndexArgs& a, uint32_t* vals_out, const uint2* undo, uint64_t n, hipStream_t st);
void launch_ix_classify(const IndexArgs& a, const uint32_t* vals, uint64_t cap, int64_t cutoff, uint32_t* live_flag,
                        uint32_t* tomb_flag, hipStream_t st);
void launch_ix_emit(const uint32_t* vals, uint64_t cap, const uint32_t* live_flag, const uint64_t* live_pos,
                    const uint32_t* tomb_flag, const uint64_t* tomb_pos, uint32_t* live, uint32_t* tomb,
                    hipStream_t st);
void launch_ix_rehash(const unsigned long long* okeys, const uint32_t* ovals, uint64_t ocap,
                      unsigned long long* nkeys, uint32_t* nvals, uint64_t nmask, hipStream_t st);
}  // namespace dr

// ---- scan-side consumers (k_filter.hip): DeltaSourceSnapshot order, TahoeFileIndex grouping ---------
namespace dr {
// add.modificationTime of every live file: its JSON line's add object, or the checkpoint's decoded
// add.modificationTime column (row-indexed values + definition levels).
struct MtimeArgs {
  const uint32_t* live;
  uint64_t n_live;
  const uint64_t* src_off;
  const uint32_t* src_len;
  uint64_t ck_rows;
  const uint8_t* json;
  const uint8_t* act_flags;
  const uint16_t* src_id;
  const uint64_t* json_bases;
  const uint8_t* ck_def;  // null: no checkpoint column
  const int64_t* ck_val;
  int32_t ck_max_def;
  int64_t* out;
  uint32_t* error;
};
void launch_mtime_extract(const MtimeArgs& a, hipStream_t st);
// Sorts live positions keys[0, n) by (mtime, path bytes) (Spark's ordering of (long, string):
// strings compare as unsigned UTF-8 bytes). temp == null: *temp_bytes gets the scratch size.
void launch_sort_scan_order(void* temp, size_t* temp_bytes, uint32_t* keys, uint64_t n, const int64_t* mtime,
                            const uint64_t* path_ptr, const uint32_t* path_len, hipStream_t st);
// Partition-value tuples of the live files (string columns of the K5 cache, by live position).
struct GroupCols {
  int32_t ncols;
  const uint64_t* sptr[PV_MAXC];
  const uint32_t* slen[PV_MAXC];
  const uint8_t* isnull[PV_MAXC];
};
void launch_sort_groups(void* temp, size_t* temp_bytes, uint32_t* keys, uint64_t n, const GroupCols& g,
                        hipStream_t st);
// flag[i] = 1 where keys[i] starts a new tuple (i == 0 or it differs from keys[i - 1]).
void launch_group_flags(const uint32_t* keys, uint64_t n, const GroupCols& g, uint32_t* flag, hipStream_t st);
}  // namespace dr

// ---- device export of allFiles / tombstones (k_filter.hip) ---------------------------------------
namespace dr {
// A decoded checkpoint leaf of one side (flat: per row; def null = column absent).
struct ExpFlat {
  const uint8_t* def;
  const int64_t* ival;
  const uint64_t* sptr;
  const uint32_t* slen;
  int32_t max_def;
};
// A decoded checkpoint map (key/value leaves, level entries; row_start null = absent).
struct ExpMap {
  const uint64_t* row_start;  // [ck_rows + 1] first level entry of each row
  const uint8_t* kdef;
  const uint64_t* kptr;
  const uint32_t* klen;
  const uint8_t* vdef;
  const uint64_t* vptr;
  const uint32_t* vlen;
  int32_t map_def, entry_def, vmax;
};
enum : int { EXC_STATS = 0, EXC_PV_N, EXC_PV_KB, EXC_PV_VB, EXC_TAGS_N, EXC_TAGS_KB, EXC_TAGS_VB, EXC_N };
// One pass per call: pass 1 (write == 0) fills the scalar fields and the EXC_* counts of every
// record; pass 2 writes the byte and entry arrays at the scanned offsets.
struct ExportArgs {
  const uint32_t* idx;  // survivor action indices
  uint64_t n;
  const uint32_t* pos;  // pass 1: the records of this launch (checkpoint ones or JSON ones); null: [0, n)
  uint64_t npos;
  int32_t side;         // 0 add (allFiles), 1 remove (tombstones)
  int32_t write;
  const uint8_t* act_flags;
  const uint16_t* src_id;      // null: one source
  const uint64_t* json_bases;
  const uint8_t* json;
  uint64_t ck_rows;
  const uint64_t* src_off;
  const uint32_t* src_len;
  const int64_t* act_size;
  ExpFlat ck_mtime, ck_size, ck_efm, ck_stats;
  ExpMap ck_pv, ck_tags;
  // pass 1 outputs
  int64_t* size;
  int64_t* mtime;
  uint8_t* efm;
  uint8_t* stats_null;
  uint8_t* pv_null;
  uint8_t* tags_null;
  uint32_t* cnt[EXC_N];        // per record
  uint64_t* stats_src;         // a checkpoint record's stats bytes (pass 2 leaves them to k_gather_bytes)
  uint32_t* stats_srclen;      // their length; 0 for a JSON record
  // pass 2
  const uint64_t* off[EXC_N];  // exclusive scans of cnt
  uint8_t* stats_bytes;
  int64_t* pv_key_off;  // [entries + 1] (entry 0 set by the host)
  int64_t* pv_val_off;
  uint8_t* pv_val_null;
  uint8_t* pv_key_bytes;
  uint8_t* pv_val_bytes;
  int64_t* tags_key_off;
  int64_t* tags_val_off;
  uint8_t* tags_val_null;
  uint8_t* tags_key_bytes;
  uint8_t* tags_val_bytes;
  // pass 2, checkpoint records: each map entry's key / value source and length (zeroed by the host;
  // JSON entries keep length 0), copied afterwards by k_gather_bytes at the entry offsets
  uint64_t* pv_ksrc;
  uint64_t* pv_vsrc;
  uint32_t* pv_klen;
  uint32_t* pv_vlen;
  uint64_t* tags_ksrc;
  uint64_t* tags_vsrc;
  uint32_t* tags_klen;
  uint32_t* tags_vlen;
  uint32_t* error;
};
// pass 1 (a.write == 0): one launch over a.pos (checkpoint records: no line stage) -- call it per
// list with `stage` false / true; pass 2: every record, staged
void launch_export(const ExportArgs& a, bool stage, hipStream_t st);
// json[i] = 1 when survivor i's record is a JSON line (0: a checkpoint row)
void launch_export_flags(const ExportArgs& a, uint32_t* json, hipStream_t st);
// jpos[jscan[i]] = i for JSON records, cpos[i - jscan[i]] = i for checkpoint ones
void launch_export_split(const uint32_t* json, const uint64_t* jscan, uint64_t n, uint32_t* jpos, uint32_t* cpos,
                         hipStream_t st);
// Order-free full-record checksum of one exported side (dr_state_record_sums; the record hash is
// defined in oracle/delta_oracle.py:record_hash): *sum += hash(record) over the n records.
struct RecordHashArgs {
  uint64_t n;
  int32_t side;
  const uint8_t* path_bytes; const uint64_t* path_off;
  const int64_t* size; const int64_t* mtime; const uint64_t* delts; const uint8_t* flags; const uint8_t* efm;
  const uint8_t* stats_null; const uint64_t* stats_off; const uint8_t* stats_bytes;
  const uint8_t* pv_null; const uint64_t* pv_entry; const int64_t* pv_key_off; const uint8_t* pv_key_bytes;
  const int64_t* pv_val_off; const uint8_t* pv_val_bytes; const uint8_t* pv_val_null;
  const uint8_t* tags_null; const uint64_t* tags_entry; const int64_t* tags_key_off; const uint8_t* tags_key_bytes;
  const int64_t* tags_val_off; const uint8_t* tags_val_bytes; const uint8_t* tags_val_null;
  unsigned long long* sum;
  uint64_t* out = nullptr;      // nullable: each record's hash, in export order (dr_state_record_hashes)
  uint32_t field_mask = 0xffu;  // words of the record hash kept (diagnostics: DR_RECORD_FIELDS); others are 0
};
void launch_record_hash(const RecordHashArgs& a, hipStream_t st);
}  // namespace dr

// ---- checkpoint page encoding (k_encode.hip) -----------------------------------------------------
namespace dr {
enum EncKind : int32_t { ENC_STR_PTR = 0, ENC_STR_OFF = 1, ENC_I64 = 2, ENC_I32 = 3, ENC_BOOL = 4, ENC_MAP_KEY = 5,
                         ENC_MAP_VAL = 6,
                         ENC_INT96 = 7,     // TIMESTAMP as Spark's INT96 (nanos of day, Julian day) from i64 micros
                         ENC_FLBA_BE = 8 }; // DECIMAL as FIXED_LEN_BYTE_ARRAY(width), big-endian, from i64 + i64hi
// One leaf column of one side (adds or removes) of a checkpoint: where its records' values are and
// the definition levels it takes. Rows of the row group outside the side's records are a null struct
// (one level, def 0).
struct EncLeaf {
  int32_t kind;
  int32_t def_null, def_present;  // flat: null field / value (maps: def_null = the map-null level)
  const uint8_t* null;            // per record (null pointer: never null)
  const uint64_t* sptr;           // ENC_STR_PTR
  const uint32_t* slen;
  const uint64_t* off;            // ENC_STR_OFF: [n + 1] offsets into bytes
  const uint8_t* bytes;
  const int64_t* i64;
  const uint32_t* i32;
  const uint8_t* b8;
  const uint64_t* entry_off;      // maps: [n + 1] first entry per record
  const int64_t* eoff;            // maps: [entries + 1] key or value byte offsets
  const uint8_t* ebytes;
  const uint8_t* enull;           // map values: per entry
  const uint8_t* vflags;          // non-null: the record is null unless vflags[i] & vbit
  uint32_t vbit;
  const int64_t* i64hi;           // ENC_FLBA_BE: high 64 bits
  uint32_t width;                 // ENC_FLBA_BE: bytes per value
};
struct EncArgs {
  EncLeaf L;
  uint64_t r0, r1;       // row group (global checkpoint rows)
  uint64_t side_lo, n;   // the side's records are rows [side_lo, side_lo + n)
  uint32_t* nlev;        // per row of the group
  uint32_t* vbytes;
  const uint64_t* lev_off;  // fill: exclusive scans
  const uint64_t* val_off;
  uint8_t* def;
  uint8_t* rep;
  uint8_t* vals;
};
void launch_enc_count(const EncArgs& a, hipStream_t st);
void launch_enc_fill(const EncArgs& a, hipStream_t st);
// Bit-packs n one-byte values (< 2^width) in groups of 8 (RLE/bit-packing hybrid body; n padded).
void launch_enc_pack(const uint8_t* in, uint64_t n, int width, uint8_t* out, hipStream_t st);
}  // namespace dr
namespace dr {
// SNAPPY compression of `n` bytes (readable up to 16 bytes past n) in 8 KiB fragments, one
// workgroup per fragment (k_encode.hip; copies never leave their fragment): fragment f's elements go
// to out + f * snap_compress_slot(), their length to out_len[f].
uint64_t snap_compress_slot();
uint64_t snap_compress_frag();
void launch_snap_compress(const uint8_t* in, uint64_t n, uint8_t* out, uint32_t* out_len, hipStream_t st);
// Compacts the fragments: fragment f's out_len[f] bytes to dst + off[f] (off = exclusive scan).
void launch_snap_gather(const uint8_t* slots, const uint32_t* len, const uint64_t* off, uint32_t nfrag, uint8_t* dst,
                        hipStream_t st);
}  // namespace dr
