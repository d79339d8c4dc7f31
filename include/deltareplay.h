/*
 * deltareplay.h -- C ABI of the MI355X-native Delta Lake snapshot state reconstruction.
 *
 * The reference has no FFI on this path; the seam is cut where a JNI shim
 * replaces the body of Snapshot.stateReconstruction / InMemoryLogReplay and
 * DeltaLog.filterFileList. Every entry point below names the reference interface it replaces
 * (paths relative to the reference checkout, D/ = core/src/main/scala/org/apache/spark/sql/delta/).
 *
 * Conventions: plain pointers and sizes only; every call returns an int status (DR_OK = 0) and
 * leaves a message in dr_last_error(ctx). Calls on distinct contexts run concurrently; calls that
 * share a context (directly, or through a state, range, shard or communicator of it) may come from
 * several host threads and run one at a time (a per-context lock; ABI 4) -- dr_last_error then holds
 * the message of the latest failed call of any of them. A host that releases a state must not call
 * with it afterwards (the JNI glue reference-counts states, jni/DeltaReplayStateRDD.scala). The
 * library owns every device and host buffer it returns until the matching *_release call
 * (Snapshot.uncache, D/util/StateCache.scala:104-109).
 */
#ifndef DELTAREPLAY_H
#define DELTAREPLAY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history (a host checks dr_abi_version() == DR_ABI_VERSION at load and refuses a mismatch):
 *   1  round 1-2 entry points
 *   2  dr_state_write_checkpoint gained its 9th parameter (add_rows); dr_pred_type gained
 *      DR_T_FLOAT .. DR_T_DECIMAL (partitionValues_parsed of the checkpoint writer);
 *      dr_state_local_counts, dr_state_last_error, dr_comm_last_error, dr_state_materialize
 *   3  dr_state_export_plan, dr_state_export_range, dr_range_release (row-range exports whose columns
 *      each fit a bound, e.g. a JVM direct buffer's 2^31 - 1 bytes)
 *   4  dr_ctx_set_option / dr_ctx_get_option (every path-changing choice is a context option; the
 *      library reads no environment variable that changes a result or a code path); a context may be
 *      shared by threads; a range outlives its context */
#define DR_ABI_VERSION 4

/* Status codes. The JNI shim rethrows the reference's exception class with dr_last_error():
 *   DR_E_EMPTY_DIR / DR_E_LOG_TRUNCATED -> FileNotFoundException (D/DeltaErrors.scala:451-457,915-917)
 *   DR_E_MISSING_PART / DR_E_NONCONTIGUOUS / DR_E_MISSING_PROTOCOL / DR_E_MISSING_METADATA
 *     -> IllegalStateException (D/DeltaErrors.scala:543-546,548-551,553-560)
 *   DR_E_BAD_SEGMENT -> IllegalArgumentException (require(...) in D/SnapshotManagement.scala:124-131) */
enum dr_status {
  DR_OK = 0,
  DR_E_INVALID_ARG = 1,
  DR_E_IO = 2,
  DR_E_EMPTY_DIR = 3,
  DR_E_LOG_TRUNCATED = 4,
  DR_E_MISSING_PART = 5,
  DR_E_NONCONTIGUOUS = 6,
  DR_E_BAD_SEGMENT = 7,
  DR_E_MISSING_PROTOCOL = 8,
  DR_E_MISSING_METADATA = 9,
  DR_E_PARSE = 10,
  DR_E_PARQUET = 11,
  DR_E_UNSUPPORTED = 12,
  DR_E_OOM = 13,
  DR_E_DEVICE = 14,
  DR_E_INTERNAL = 15,
  DR_E_CHECKSUM = 16,     /* computed state differs from the version's .crc (IllegalStateException) */
  DR_E_NO_CHECKSUM = 17,  /* .crc empty or unparseable: ReadChecksum yields None, nothing to validate */
  DR_E_REBUILD = 18,      /* dr_state_apply cannot extend this base (e.g. its retention cutoff is later than
                             the new one): the caller rebuilds the snapshot from its segment instead */
  DR_E_FOREIGN_FILE = 19  /* a staged file is not in the table's _delta_log: AssertionError
                             (assertLogBelongsToTable, D/Snapshot.scala:334-345) */
};

/* Segment file kinds (D/DeltaLogFileIndex.scala:67-68). */
enum dr_file_kind { DR_FILE_JSON = 0, DR_FILE_CHECKPOINT = 1 };

/* One LogSegment file (D/SnapshotManagement.scala:394-416). Bytes are borrowed for the call. */
typedef struct dr_file {
  int64_t version;     /* commit version, or the checkpoint version for checkpoint parts */
  int32_t kind;        /* dr_file_kind */
  int32_t part;        /* 1-based checkpoint part (0 for JSON / single-part) */
  const uint8_t* data; /* file bytes (host memory) */
  uint64_t len;
} dr_file;

/* computedState counters (D/Snapshot.scala:140-151). */
typedef struct dr_counts {
  int64_t num_files;              /* count(add) */
  int64_t size_in_bytes;          /* coalesce(sum(add.size), 0) */
  int64_t num_removes;            /* count(remove): unexpired tombstones */
  int64_t num_metadata;
  int64_t num_protocol;
  int64_t num_set_transactions;
  int64_t num_actions;            /* actions replayed (JSON lines + checkpoint rows) */
  int64_t num_file_actions;       /* add + remove actions replayed */
  int64_t version;                /* snapshot version */
  int64_t malformed_lines;        /* JSON lines Spark's PERMISSIVE reader would null out */
  uint64_t live_key_sum;          /* sum (mod 2^64) of the top 32 bits of xxh64(path key) over allFiles */
  uint64_t tomb_key_sum;          /* same over tombstones: order-free checksum for parity */
} dr_counts;

/* Replay flags. */
#define DR_FLAG_NO_VALIDATION 0x1u  /* stateReconstructionValidation.enabled=false (D/sources/DeltaSQLConf.scala:86-91) */
#define DR_FLAG_EXACT_REDUCE 0x2u   /* test hook: reduce every bucket with the exact O(m^2) kernel */
#define DR_FLAG_REDUCE64 0x4u       /* test hook: reduce every bucket with the 64-bit-key fallback kernel */

/* Export columns of one side of the state (allFiles or tombstones; D/Snapshot.scala:193-204).
 * Strings: `*_off` has n+1 entries into `*_bytes`. Maps (partitionValues, tags): `*_entry_off`
 * has n+1 entries into the entry arrays; map_null[i] != 0 means the map itself is null.
 * All buffers are owned by the state and valid until dr_state_release. */
typedef struct dr_export {
  int64_t n;
  const int64_t* path_off;   const uint8_t* path_bytes;
  const int64_t* size;
  const int64_t* modification_time;     /* adds */
  const int64_t* deletion_timestamp;    /* removes; valid where deletion_timestamp_valid[i] */
  const uint8_t* deletion_timestamp_valid;
  const uint8_t* extended_file_metadata;/* removes */
  const int64_t* stats_off;  const uint8_t* stats_bytes; const uint8_t* stats_null;
  const int64_t* pv_entry_off; const uint8_t* pv_null;
  const int64_t* pv_key_off; const uint8_t* pv_key_bytes;
  const int64_t* pv_val_off; const uint8_t* pv_val_bytes; const uint8_t* pv_val_null;
  const int64_t* tags_entry_off; const uint8_t* tags_null;
  const int64_t* tags_key_off; const uint8_t* tags_key_bytes;
  const int64_t* tags_val_off; const uint8_t* tags_val_bytes; const uint8_t* tags_val_null;
} dr_export;

enum dr_which { DR_LIVE = 0, DR_TOMBSTONES = 1 };

typedef struct dr_ctx dr_ctx;
typedef struct dr_state dr_state;
typedef struct dr_staged dr_staged;

/* ---- context ------------------------------------------------------------------------------ */
/* Creates a context bound to HIP device `device` with its own stream. */
int dr_ctx_create(int device, dr_ctx** out);
/* Waits for any call running on the context, then frees it. States, staged segments, shards and
 * communicators of the context must be released first; row ranges and checkpoint part files may
 * outlive it (their pinned blocks are then unpinned by dr_range_release / dr_free). */
void dr_ctx_destroy(dr_ctx* ctx);

/* Context options (ABI 4): the per-session configuration of the path, as the reference takes its
 * DeltaSQLConf from the session (D/sources/DeltaSQLConf.scala:29). Set before the calls they should
 * affect; they change code paths and resource use, never results (every choice is parity-tested).
 * DR_E_INVALID_ARG for an unknown option or a value outside its range. Debug-only switches (phase
 * clocks, poisoning, roctx ranges, dumps) stay environment variables and change no result. */
enum dr_option {
  DR_OPT_OVERLAP = 1,          /* 1: K1 line parsing on a second stream beside the checkpoint decode for
                                  segments with a checkpoint and a multi-block JSON part; 0 (default since
                                  r06: the two streams' kernels share the CUs and gained nothing): one stream */
  DR_OPT_SPLIT = 2,            /* 1 (default): replays of more than 2^13 * 2048 actions refine K3's buckets
                                  (k_bucket_split) so K4 reduces each in one pass; 0: K4's sub-passes */
  DR_OPT_BUCKET_BITS = 3,      /* -1 (default): automatic; n in 0..32: at most n K3 bucket bits (fewer,
                                  larger buckets: the reducer's sub-pass paths) */
  DR_OPT_FILTER_EVAL = 4,      /* dr_filter's evaluator: 0 (default) dictionary codes where every column has
                                  one, else typed leaves; 1 typed leaves (k_filter_leaf); 2 the generic
                                  postfix interpreter (k_filter_typed) */
  DR_OPT_APPLY_FULL = 5,       /* 0 (default); 1: dr_state_apply reduces base survivors + tail through K3/K4
                                  instead of the O(tail) path index */
  DR_OPT_CANON_HINT = 6,       /* -1 (default): a segment's first replay sizes the canonicalisation arena
                                  exactly (one read-back); n >= 0: n bytes stand in for that sizing (an
                                  undersized arena is detected and the parse redone) */
  DR_OPT_JSON_STAGED = 7,      /* 0 (default); 1: every JSON segment through the staged, wave-cooperative
                                  K1 kernel (the streamed-commit walker) instead of the lane-per-line one */
  DR_OPT_HOST_CACHE_BYTES = 8  /* bytes of released pinned host blocks kept for reuse (default 64 GiB:
                                  config 4's 36 GB export stays pinned between snapshots); a released
                                  block evicts the largest cached ones to fit, one over the bound is
                                  unpinned at once */
};
int dr_ctx_set_option(dr_ctx* ctx, int32_t option, int64_t value);
int dr_ctx_get_option(dr_ctx* ctx, int32_t option, int64_t* value);
const char* dr_last_error(const dr_ctx* ctx);
/* The message of the last failed call on a state / communicator (its context's dr_last_error), for
 * hosts that keep only the state or communicator handle (the JNI glue, jni/deltareplay_jni.c). */
const char* dr_state_last_error(const dr_state* state);
typedef struct dr_comm dr_comm;
const char* dr_comm_last_error(const dr_comm* comm);
int dr_abi_version(void);

/* ---- log segment (host) -------------------------------------------------------------------
 * Replaces SnapshotManagement.getLogSegmentForVersion + Checkpoints.lastCheckpoint
 * (D/SnapshotManagement.scala:82-179,365-372; D/Checkpoints.scala:148-218).
 * Lists `log_path` (a _delta_log directory) with POSIX I/O. version_to_load < 0 = latest.
 * Writes the segment as a newline-separated list "<kind> <version> <part> <file name>" into
 * `buf` (NUL-terminated; *needed gets the size). */
int dr_log_segment(dr_ctx* ctx, const char* log_path, int64_t version_to_load,
                   char* buf, uint64_t buf_len, uint64_t* needed, int64_t* version_out);

/* ---- staging (host -> HBM) ----------------------------------------------------------------
 * Copies the segment's file bytes into HBM and plans the Parquet page decode (footer + page
 * headers, host). The staged input is reusable across dr_replay_staged calls. */
int dr_stage(dr_ctx* ctx, const dr_file* files, int32_t nfiles, dr_staged** out);
/* dr_stage with each file's name (a path or file: URI; "" = unnamed, as the reference's cached
 * snapshots): every named file must sit directly in `log_path` -- the check Snapshot.stateReconstruction
 * applies to input_file_name() of every row (assertLogBelongsToTable, D/Snapshot.scala:102,334-345) --
 * or the call fails with DR_E_FOREIGN_FILE and the reference's AssertionError text; a name that
 * contradicts its dr_file (not a FileNames delta/checkpoint name of that version and part,
 * D/util/FileNames.scala:27-73) fails with DR_E_INVALID_ARG. */
int dr_stage_named(dr_ctx* ctx, const char* log_path, const dr_file* files, const char* const* names,
                   int32_t nfiles, dr_staged** out);
/* Lists + reads the latest (or version_to_load) segment of `log_path` and stages it. */
int dr_stage_log(dr_ctx* ctx, const char* log_path, int64_t version_to_load, dr_staged** out);
int dr_staged_release(dr_staged* staged);
/* Bytes staged in HBM (JSON + checkpoint). */
int dr_staged_bytes(const dr_staged* staged, uint64_t* json_bytes, uint64_t* checkpoint_bytes);
/* Decode plan figures (for roofline accounting): out[0] JSON bytes, [1] checkpoint bytes,
 * [2] checkpoint rows, [3] planned pages, [4] their compressed bytes, [5] their decompressed bytes,
 * [6] dictionary entries, [7] SNAPPY input bytes, [8] SNAPPY output bytes, [9] SNAPPY 256-byte
 * speculation chunks, [10] SNAPPY 64 KiB output blocks, [11] SNAPPY elements (0 until a replay with
 * timing on has counted them), [12] bytes of uncompressed pages copied, [13] JSON lines (newline-terminated). *n receives the number of
 * figures written (<= cap). */
int dr_staged_plan(const dr_staged* staged, uint64_t* out, int32_t cap, int32_t* n);

/* ---- replay (device) ----------------------------------------------------------------------
 * Replaces Snapshot.stateReconstruction (D/Snapshot.scala:88-111) and the per-partition
 * InMemoryLogReplay.append/checkpoint (D/actions/InMemoryLogReplay.scala:43-77): parse,
 * canonicalize, hash, partition+sort, last-writer-wins, tombstone retention
 * (delTimestamp > min_file_retention_timestamp), compaction, computedState counters.
 * The result stays resident in HBM. */
int dr_replay_staged(dr_ctx* ctx, const dr_staged* staged, int64_t min_file_retention_timestamp,
                     uint32_t flags, dr_state** out);
/* dr_stage + dr_replay_staged + dr_staged_release. */
int dr_replay(dr_ctx* ctx, const dr_file* files, int32_t nfiles,
              int64_t min_file_retention_timestamp, uint32_t flags, dr_state** out);
int dr_state_release(dr_state* state);

/* Incremental update: the state of `base`'s segment extended by the commit files staged in
 * `tail` (dr_stage with JSON files of versions base+1, base+2, ... contiguous), with a new
 * retention cutoff (not earlier than the base's: DR_E_REBUILD otherwise). Replaces the full rebuild of
 * SnapshotManagement.update (D/SnapshotManagement.scala:286-330) with K3/K4 over the base's
 * survivors followed by the tail's lines; equal to dr_replay over the whole segment. `base` and
 * `tail` stay owned by the caller and may be released afterwards (the new state keeps what it
 * needs). DR_E_NONCONTIGUOUS when the tail's versions do not follow the base's. */
int dr_state_apply(dr_ctx* ctx, dr_state* base, const dr_staged* tail, int64_t min_file_retention_timestamp,
                   uint32_t flags, dr_state** out);

/* ---- results ------------------------------------------------------------------------------ */
int dr_state_counts(dr_state* state, dr_counts* out);
/* A rank's own counters of a dr_replay_sharded state before they were all-reduced (the actions this
 * rank parsed and reduced, its local survivors); equal to dr_state_counts for any other state. The
 * bench prices each rank's K3/K4 kernels with it. */
int dr_state_local_counts(dr_state* state, dr_counts* out);
/* Latest protocol / metaData and the set transactions as JSON text in the reference's action
 * encoding ({"protocol":{...}} etc., one per line; D/actions/actions.scala:71). */
int dr_state_nonfile_json(dr_state* state, const char** json, uint64_t* len);

/* Snapshot.validateChecksum's comparison (D/Checksum.scala:155-191): `crc` is the first line of the
 * version's `%020d.crc` (FileNames.checksumFile, D/util/FileNames.scala:36). Returns DR_OK when the
 * five counters match, DR_E_CHECKSUM with checkMismatch's text ("Table size (bytes) - Expected: X
 * Computed: Y" lines joined by '\n') in msg (NUL-terminated, *msg_len = full length), or
 * DR_E_NO_CHECKSUM when the line is empty or does not parse as a VersionChecksum. */
int dr_state_check_checksum(dr_state* state, const char* crc, uint64_t crc_len, char* msg, uint64_t msg_cap,
                            uint64_t* msg_len);
/* Materialises allFiles (DR_LIVE) or tombstones (DR_TOMBSTONES) on the host, dataChange=false. */
int dr_state_export(dr_state* state, int32_t which, dr_export* out);

/* Row-range export (ABI 3): allFiles / tombstones as a sequence of row ranges, for a host that cannot
 * take a side as one set of columns -- the JVM's direct buffers hold at most 2^31 - 1 bytes, and
 * config 4's 100M-file side holds ~9 GB of paths alone -- or that builds the reference's partitioned
 * state (Snapshot.state is a partitioned, cached RDD, D/Snapshot.scala:103-120; D/util/StateCache.scala:
 * 45-68) with one partition per range.
 *
 * dr_state_export_plan: row boundaries bounds[0] = 0 < ... < bounds[*nranges] = the side's rows such
 * that every range holds at most max_rows rows and every one of its dr_export columns (offset arrays
 * included) at most max_bytes bytes (freed with dr_free). DR_E_UNSUPPORTED when a single row exceeds
 * max_bytes in some column.
 * dr_state_export_range: rows [row_begin, row_end) of the side in dr_state_export's order, as columns
 * whose offsets are rebased to the range (path_off[0] = 0, entry offsets count from the range's first
 * entry, byte offsets from its first byte): the concatenation of consecutive ranges' columns, offsets
 * shifted back, equals dr_state_export's. The columns are host memory owned by *range until
 * dr_range_release (independent of the state and of the context: either may be released first).
 * dr_range_release of a range that is not live (released twice) returns DR_E_INVALID_ARG. */
typedef struct dr_range dr_range;
int dr_state_export_plan(dr_state* state, int32_t which, int64_t max_rows, uint64_t max_bytes, int64_t** bounds,
                         int64_t* nranges);
int dr_state_export_range(dr_state* state, int32_t which, int64_t row_begin, int64_t row_end, dr_range** range,
                          dr_export* out);
int dr_range_release(dr_range* range);

/* The full-record state resident in HBM: every field of allFiles and tombstones (path, size,
 * modificationTime / deletionTimestamp, extendedFileMetadata, stats, partitionValues, tags) extracted
 * on the device into columns kept with the state until dr_state_release -- the reference's cached
 * SingleAction rows (cacheDS(stateReconstruction), D/Snapshot.scala:116-120, D/util/StateCache.scala:45-68).
 * dr_state_export then only copies them to the host, dr_state_record_sums only hashes them.
 * *bytes (may be NULL): the device bytes the columns hold. */
int dr_state_materialize(dr_state* state, uint64_t* bytes);

/* Order-free full-record checksums of allFiles and tombstones, computed on the device from the export
 * columns: the sum mod 2^64 over the records of one 64-bit hash of every field of the record
 * (path, size, modificationTime / deletionTimestamp + presence, extendedFileMetadata, stats,
 * partitionValues, tags; dataChange is false on both sides). The record hash is defined once in
 * DESIGN.md §2; the CPU restatements compute the same sums, so two states with equal sums hold the
 * same record sets (D/actions/InMemoryLogReplay.scala:55-77 winners, not only the same paths).
 * For a sharded state: this rank's records (sum the ranks' values). */
int dr_state_record_sums(dr_state* state, uint64_t* live_sum, uint64_t* tomb_sum);
/* The same per-record hashes one by one: out[i] = the hash of row i of side `which` in dr_state_export's
 * order (n = the side's row count, else DR_E_INVALID_ARG). Sorted, they are the side's record multiset,
 * which the full-size parity test compares element by element with the CPU restatement's
 * (replay_oracle --record-hashes): equality of every record up to a 64-bit collision of the record
 * hash, not only of a sum. */
int dr_state_record_hashes(dr_state* state, int32_t which, uint64_t* out, int64_t n);

/* ---- per-line commit decode (device) --------------------------------------------------------
 * The hot fields of DeltaLog.getChanges' per-line Action.fromJson (D/DeltaLog.scala:222-238,
 * D/actions/actions.scala:57-59) for a streaming host: K1 over the staged commit (JSON) files, one
 * record per newline-terminated line in file order (blank lines included, kind DR_KIND_NONE), with
 * the replay's reading of a line (Spark's PERMISSIVE JSON reader over Action.logSchema: a line it
 * cannot read is DR_KIND_MALFORMED). Paths are the raw JSON string bodies (DR_LF_PATH_ESCAPED
 * when they hold escapes) at `bytes + path_off`; `size` reads 0 and the deletion timestamp is
 * absent (no DR_LF_HAS_DELETION_TS) when the line has none. Owned by `parsed` until
 * dr_parsed_release. */
enum dr_action_kind { DR_KIND_NONE = 0, DR_KIND_ADD = 1, DR_KIND_REMOVE = 2, DR_KIND_METADATA = 3,
                      DR_KIND_TXN = 4, DR_KIND_PROTOCOL = 5, DR_KIND_CDC = 6, DR_KIND_COMMITINFO = 7,
                      DR_KIND_MALFORMED = 15 };
#define DR_LF_HAS_DELETION_TS 0x1u
#define DR_LF_PATH_ESCAPED 0x4u
#define DR_LF_PATH_NULL 0x8u
typedef struct dr_lines {
  int64_t n;
  const int64_t* version;                          /* commit version of the line's file */
  const uint64_t* line_off; const uint32_t* line_len;  /* the line in `bytes` (no newline) */
  const uint8_t* kind;                             /* dr_action_kind, SingleAction.unwrap priority */
  const uint8_t* flags;                            /* DR_LF_* */
  const uint64_t* path_off; const uint32_t* path_len;  /* add / remove path in `bytes` */
  const int64_t* size;
  const int64_t* deletion_timestamp;
  const uint8_t* bytes; uint64_t nbytes;           /* the staged commit bytes, files newline-terminated */
} dr_lines;
typedef struct dr_parsed dr_parsed;
int dr_parse_commits(dr_ctx* ctx, const dr_staged* staged, dr_parsed** parsed, dr_lines* lines);
int dr_parsed_release(dr_parsed* parsed);

/* ---- partition pruning (device) -----------------------------------------------------------
 * Replaces DeltaLog.filterFileList + rewritePartitionFilters (D/DeltaLog.scala:500-547) for
 * PartitionFiltering.filesForScan (D/PartitionFiltering.scala:27-42): the metadata-only
 * conjuncts, lowered by the shim to the postfix program below, are evaluated over the live
 * AddFiles with Spark's non-ANSI Cast(string AS type) and three-valued logic.
 *
 * Program: `ops[nops]` (dr_pred_op). Columns are indices into `col_names` / `col_types`
 * (the partitionSchema; names are the exact map keys). Literals are indices into `lit_*`:
 * lit_types[k] (dr_pred_type), integer/date/boolean literals in lit_i64[k], strings as
 * lit_str_off[k]..lit_str_off[k+1] into lit_str_bytes; lit_null[k] marks a NULL literal.
 * The program must leave one boolean on the stack; rows where it is TRUE are selected.
 * Output: selected live-file ordinals (indices into the DR_LIVE export order). */
enum dr_pred_type { DR_T_STRING = 0, DR_T_BYTE = 1, DR_T_SHORT = 2, DR_T_INT = 3, DR_T_LONG = 4,
                    DR_T_DATE = 5, DR_T_BOOLEAN = 6,
                    /* partitionValues_parsed of the checkpoint writer only (not in predicate programs):
                       Cast(string AS float / double / timestamp (session zone UTC) / binary /
                       decimal(p, s)); a decimal's code carries p << 8 | s << 16 */
                    DR_T_FLOAT = 7, DR_T_DOUBLE = 8, DR_T_TIMESTAMP = 9, DR_T_BINARY = 10, DR_T_DECIMAL = 11 };
enum dr_pred_opcode {
  DR_OP_COL = 0,      /* arg = column index: push Cast(partitionValues[col] AS type) */
  DR_OP_LIT = 1,      /* arg = literal index */
  DR_OP_EQ = 2, DR_OP_NE = 3, DR_OP_LT = 4, DR_OP_LE = 5, DR_OP_GT = 6, DR_OP_GE = 7,
  DR_OP_NSEQ = 8,     /* <=> */
  DR_OP_IN = 9,       /* arg = number of literals pushed after the value */
  DR_OP_ISNULL = 10, DR_OP_ISNOTNULL = 11,
  DR_OP_AND = 12, DR_OP_OR = 13, DR_OP_NOT = 14
};
typedef struct dr_pred_op { int32_t opcode; int32_t arg; } dr_pred_op;

typedef struct dr_predicate {
  int32_t nops; const dr_pred_op* ops;
  int32_t ncols; const char* const* col_names; const int32_t* col_types;
  int32_t nlits; const int32_t* lit_types; const int64_t* lit_i64; const uint8_t* lit_null;
  const int64_t* lit_str_off; const uint8_t* lit_str_bytes;
} dr_predicate;

int dr_filter(dr_state* state, const dr_predicate* pred, int64_t** selected, int64_t* nselected);
void dr_free(void* p);

/* ---- checkpoint writer --------------------------------------------------
 * Checkpoints.writeCheckpoint / buildCheckpoint (D/Checkpoints.scala:229-365): part `part` (1-based)
 * of `parts` of the state's checkpoint -- rows protocol, metaData, txns, allFiles, tombstones
 * (dataChange=false), split into contiguous slices -- as a complete Parquet file in *bytes (freed
 * with dr_free). The file-action columns are encoded on the device (SNAPPY-compressed on the device
 * with DR_CKPT_SNAPPY, else uncompressed);
 * `row_group_rows` 0 = 2^20. opts: DR_CKPT_STATS writes add.stats (delta.checkpoint.writeStatsAsJson),
 * DR_CKPT_PARSED adds add.partitionValues_parsed (the partition schema's types; writeStatsAsStruct /
 * checkpointV2). The caller writes the file (temp + rename) and `_last_checkpoint`.
 * A sharded replay's state (dr_replay_sharded / dr_shard_finish) writes its own part of a multi-part
 * checkpoint from the GPU shards: all of its survivors, plus the protocol / metaData / txn rows when
 * part == 1 (rank r writes part r + 1 of world; PROTOCOL.md lets parts split the rows any way). */
#define DR_CKPT_STATS 0x1u
#define DR_CKPT_PARSED 0x2u
#define DR_CKPT_SNAPPY 0x4u   /* SNAPPY pages for the device-encoded columns (Spark's default codec) */
/* *rows: the part's row count; *add_rows (may be NULL): its add rows, which the caller sums over the
 * parts and compares with numOfFiles before writing _last_checkpoint (D/Checkpoints.scala:325-328). */
int dr_state_write_checkpoint(dr_state* state, int32_t part, int32_t parts, uint32_t opts, uint64_t row_group_rows,
                              uint8_t** bytes, uint64_t* len, int64_t* rows, int64_t* add_rows);
/* A sharded state's table-wide protocol / metaData / txn winners from every rank's local winners
 * (dr_state_nonfile_json of each rank, concatenated in rank order, one action per line), reduced as
 * InMemoryLogReplay does (D/actions/InMemoryLogReplay.scala:47-53); dr_replay_sharded does this itself
 * over RCCL, a host that exchanges through its own collectives calls it after dr_shard_finish.
 * flags: DR_FLAG_NO_VALIDATION skips the missing protocol / metadata errors. */
int dr_state_set_nonfile_json(dr_state* state, const char* lines, uint64_t len, uint32_t flags);

/* ---- scan-side consumers of the resident state -----------------------
 * DeltaSourceSnapshot.initialFiles (D/files/DeltaSourceSnapshot.scala:53-95): allFiles.sort(
 * "modificationTime", "path") computed on the device (modificationTime decoded from the live files'
 * JSON lines / the checkpoint's add.modificationTime column; strings compare as unsigned UTF-8
 * bytes). *order = the dr_state_export(DR_LIVE) positions in that order (freed with dr_free); the
 * caller's zipWithIndex is the position in *order. */
int dr_state_scan_order(dr_state* state, int64_t** order, int64_t* n);
/* TahoeFileIndex.listFiles grouping (D/files/TahoeFileIndex.scala:58-81, groupBy(partitionValues)):
 * `rows` (live positions, e.g. a dr_filter selection; NULL = every live file) grouped on the device
 * by the raw values of the metadata's partitionColumns (null distinct from every string). *order
 * holds the rows group by group (groups ordered by their values, nulls first; rows ascending in a
 * group), *group_off the *ngroups + 1 group boundaries into it; both freed with dr_free. */
int dr_state_partition_groups(dr_state* state, const int64_t* rows, int64_t nrows, int64_t** order,
                              int64_t** group_off, int64_t* ngroups);

/* ---- multi-GPU shards (one process per GPU) ------------------------------------
 * Replaces Snapshot.stateReconstruction's repartition(50, coalesce(add.path, remove.path)) shuffle
 * (D/Snapshot.scala:103-104) across GPUs. The segment's replay order (checkpoint row groups, then
 * commits) is cut into `world` contiguous slices by estimated device cost; rank r stages slice r.
 * After the local parse, each file action goes to owner(path) = low32(xxh64(path)) * world >> 32;
 * every owner runs the last-writer-wins reduction on its shard alone and returns a verdict per
 * received record (0 dropped, 1 live AddFile, 2 kept tombstone) to the sender, which owns the
 * record bytes for export. The exchange itself is the caller's (RCCL all-to-all over xGMI through
 * torch.distributed): the library only reads/writes the device buffers it is handed.
 *
 *   dr_shard_plan       host only: the unit -> rank plan as text lines
 *                       "<rank> <kind> <version> <part> <rg_lo> <rg_hi> <weight> <file name>"
 *   dr_stage_log_shard  stage rank's slice (checkpoint row groups [rg_lo, rg_hi) + commits)
 *   dr_shard_begin      K1/K2/canonicalise the slice, partition its file actions by owner; returns
 *                       the records (send_counts[d]) and path bytes (send_bytes[d]) per owner d
 *   dr_shard_pack       writes the records (DR_SHARD_REC_BYTES each, grouped by owner, replay
 *                       order inside a group) and the path bytes into caller device buffers
 *   dr_shard_reduce     owner side: the records received from ranks 0..world-1 concatenated in rank
 *                       order; writes one verdict byte per record into `verdict` (device)
 *   dr_shard_finish     sender side: verdicts returned in send order -> dr_state of this rank's
 *                       surviving records (export as usual). Its counts hold this rank's owner-side
 *                       partial sums (files, bytes, tombstones, key sums, file actions) and its
 *                       local num_actions; non-file winners are local (merge in rank order). */
#define DR_SHARD_REC_BYTES 32
typedef struct dr_shard dr_shard;
int dr_shard_plan(dr_ctx* ctx, const char* log_path, int64_t version_to_load, int32_t world, char* buf,
                  uint64_t buf_len, uint64_t* needed);
int dr_stage_log_shard(dr_ctx* ctx, const char* log_path, int64_t version_to_load, int32_t world, int32_t rank,
                       dr_staged** out);
int dr_shard_begin(dr_ctx* ctx, const dr_staged* staged, int32_t world, dr_shard** out, uint64_t* send_counts,
                   uint64_t* send_bytes);
int dr_shard_pack(dr_shard* shard, void* send_rec, void* send_path);
int dr_shard_reduce(dr_shard* shard, const void* recv_rec, uint64_t n_recv, const void* recv_path,
                    uint64_t recv_path_bytes, int64_t min_file_retention_timestamp, uint8_t* verdict);
int dr_shard_finish(dr_shard* shard, const uint8_t* verdict_back, dr_state** out);
int dr_shard_release(dr_shard* shard);

/* The whole sharded replay inside the library, over RCCL (xGMI): no host framework is needed (the
 * JNI host has no torch). Same semantics as the dr_shard_* steps driven by delta_amd/sharded.py:
 * every rank stages its slice (dr_stage_log_shard) and calls dr_replay_sharded collectively; the
 * exchange is grouped ncclSend/ncclRecv on the context's stream, counts and non-file winners go
 * through ncclAllGather, the counters through ncclAllReduce. The returned state exports this rank's
 * surviving records; its counters and non-file winners are table-wide. The communicator comes from
 * one dr_comm_unique_id shared by the caller's own means (e.g. the Spark driver) and one
 * dr_comm_create per rank; librccl is loaded on first use (DR_E_UNSUPPORTED when absent). */
int dr_comm_unique_id(uint8_t* id /* 128 bytes */);
int dr_comm_create(dr_ctx* ctx, const uint8_t* id, int32_t world, int32_t rank, dr_comm** out);
/* Test hook: an id whose communicator is an in-process loopback instead of RCCL -- the `world` ranks
 * are threads of this process (one dr_ctx each, any device), and every collective of dr_replay_sharded
 * becomes device copies between the ranks' buffers at a barrier. Runs the sharded replay's own control
 * flow at world > 1 on one GPU (RCCL refuses two ranks on one device). */
int dr_comm_loopback_id(uint8_t* id /* 128 bytes */);
int dr_comm_release(dr_comm* comm);
int dr_replay_sharded(dr_comm* comm, const dr_staged* staged, int64_t min_file_retention_timestamp, uint32_t flags,
                      dr_state** out);

/* ---- measurement hooks (bench.py) ----------------------------------------------------------
 * Per-stage device time of the last dr_replay_staged on this context (HIP events on the
 * context's stream), in milliseconds; names are returned NUL-separated. */
int dr_last_timings(dr_ctx* ctx, char* names, uint64_t names_len, float* ms, int32_t cap,
                    int32_t* n);
/* Enable/disable per-stage event timing (off by default; small overhead when on). */
int dr_set_timing(dr_ctx* ctx, int32_t on);
/* Restricts the per-kernel events of dr_set_timing to one kernel (by name, e.g. "k_snap_exec";
 * NULL or "" = every kernel): the bench times its roofline kernel inside the timed steps without
 * an event pair on every other launch. */
int dr_set_timing_only(dr_ctx* ctx, const char* kernel);

#ifdef __cplusplus
}
#endif
#endif /* DELTAREPLAY_H */
