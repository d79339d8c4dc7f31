"""ctypes binding of libdeltareplay (include/deltareplay.h).

The library is built in-tree (`make`, or `__graft_entry__.build()`); importing this module fails
loudly when it is missing -- there is no CPU fallback for the replay path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DR_LIB (tests): an in-tree variant of the library, e.g. libdeltareplay_bounds.so (LDS index checks)
LIB_PATH = os.path.join(_HERE, os.environ.get("DR_LIB", "libdeltareplay.so"))

DR_OK = 0
STATUS = {
    1: "DR_E_INVALID_ARG", 2: "DR_E_IO", 3: "DR_E_EMPTY_DIR", 4: "DR_E_LOG_TRUNCATED",
    5: "DR_E_MISSING_PART", 6: "DR_E_NONCONTIGUOUS", 7: "DR_E_BAD_SEGMENT",
    8: "DR_E_MISSING_PROTOCOL", 9: "DR_E_MISSING_METADATA", 10: "DR_E_PARSE", 11: "DR_E_PARQUET",
    12: "DR_E_UNSUPPORTED", 13: "DR_E_OOM", 14: "DR_E_DEVICE", 15: "DR_E_INTERNAL",
    16: "DR_E_CHECKSUM", 17: "DR_E_NO_CHECKSUM", 18: "DR_E_REBUILD", 19: "DR_E_FOREIGN_FILE",
}
DR_E_REBUILD = 18
DR_CKPT_STATS, DR_CKPT_PARSED, DR_CKPT_SNAPPY = 0x1, 0x2, 0x4
DR_E_FOREIGN_FILE = 19
DR_E_CHECKSUM, DR_E_NO_CHECKSUM = 16, 17
DR_FILE_JSON, DR_FILE_CHECKPOINT = 0, 1
DR_LIVE, DR_TOMBSTONES = 0, 1
DR_FLAG_NO_VALIDATION = 0x1
DR_FLAG_EXACT_REDUCE = 0x2
DR_FLAG_REDUCE64 = 0x4
ABI_VERSION = 4  # include/deltareplay.h DR_ABI_VERSION
# context options (include/deltareplay.h enum dr_option)
OPTIONS = {"overlap": 1, "split": 2, "bucket_bits": 3, "filter_eval": 4, "apply_full": 5, "canon_hint": 6,
           "json_staged": 7, "host_cache_bytes": 8}

# Exported symbols (checked by tests/test_native_abi.py against include/deltareplay.h).
SYMBOLS = [
    "dr_abi_version", "dr_ctx_create", "dr_ctx_destroy", "dr_ctx_set_option", "dr_ctx_get_option", "dr_last_error", "dr_state_last_error",
    "dr_comm_last_error", "dr_log_segment",
    "dr_stage", "dr_stage_named", "dr_stage_log", "dr_comm_unique_id", "dr_comm_loopback_id", "dr_comm_create",
    "dr_comm_release",
    "dr_replay_sharded", "dr_staged_release", "dr_staged_bytes", "dr_staged_plan",
    "dr_replay_staged",
    "dr_replay", "dr_state_release", "dr_state_apply", "dr_state_counts", "dr_state_local_counts", "dr_state_nonfile_json", "dr_state_check_checksum",
    "dr_state_export", "dr_state_export_plan", "dr_state_export_range", "dr_range_release", "dr_state_materialize", "dr_state_record_sums", "dr_state_record_hashes", "dr_state_write_checkpoint", "dr_state_set_nonfile_json", "dr_filter", "dr_state_scan_order", "dr_state_partition_groups", "dr_free", "dr_last_timings", "dr_set_timing", "dr_set_timing_only",
    "dr_shard_plan", "dr_stage_log_shard", "dr_shard_begin", "dr_shard_pack", "dr_shard_reduce",
    "dr_shard_finish", "dr_shard_release", "dr_parse_commits", "dr_parsed_release",
]
DR_SHARD_REC_BYTES = 32


class dr_file(C.Structure):
    _fields_ = [("version", C.c_int64), ("kind", C.c_int32), ("part", C.c_int32),
                ("data", C.c_void_p), ("len", C.c_uint64)]


class dr_counts(C.Structure):
    _fields_ = [("num_files", C.c_int64), ("size_in_bytes", C.c_int64), ("num_removes", C.c_int64),
                ("num_metadata", C.c_int64), ("num_protocol", C.c_int64),
                ("num_set_transactions", C.c_int64), ("num_actions", C.c_int64),
                ("num_file_actions", C.c_int64), ("version", C.c_int64),
                ("malformed_lines", C.c_int64), ("live_key_sum", C.c_uint64),
                ("tomb_key_sum", C.c_uint64)]


_P64 = C.POINTER(C.c_int64)
_PU8 = C.POINTER(C.c_uint8)


class dr_export(C.Structure):
    _fields_ = [("n", C.c_int64),
                ("path_off", _P64), ("path_bytes", _PU8),
                ("size", _P64), ("modification_time", _P64),
                ("deletion_timestamp", _P64), ("deletion_timestamp_valid", _PU8),
                ("extended_file_metadata", _PU8),
                ("stats_off", _P64), ("stats_bytes", _PU8), ("stats_null", _PU8),
                ("pv_entry_off", _P64), ("pv_null", _PU8),
                ("pv_key_off", _P64), ("pv_key_bytes", _PU8),
                ("pv_val_off", _P64), ("pv_val_bytes", _PU8), ("pv_val_null", _PU8),
                ("tags_entry_off", _P64), ("tags_null", _PU8),
                ("tags_key_off", _P64), ("tags_key_bytes", _PU8),
                ("tags_val_off", _P64), ("tags_val_bytes", _PU8), ("tags_val_null", _PU8)]


class dr_lines(C.Structure):
    _fields_ = [("n", C.c_int64), ("version", _P64), ("line_off", C.POINTER(C.c_uint64)),
                ("line_len", C.POINTER(C.c_uint32)), ("kind", _PU8), ("flags", _PU8),
                ("path_off", C.POINTER(C.c_uint64)), ("path_len", C.POINTER(C.c_uint32)),
                ("size", _P64), ("deletion_timestamp", _P64), ("bytes", _PU8), ("nbytes", C.c_uint64)]


class dr_pred_op(C.Structure):
    _fields_ = [("opcode", C.c_int32), ("arg", C.c_int32)]


class dr_predicate(C.Structure):
    _fields_ = [("nops", C.c_int32), ("ops", C.POINTER(dr_pred_op)),
                ("ncols", C.c_int32), ("col_names", C.POINTER(C.c_char_p)),
                ("col_types", C.POINTER(C.c_int32)),
                ("nlits", C.c_int32), ("lit_types", C.POINTER(C.c_int32)),
                ("lit_i64", _P64), ("lit_null", _PU8),
                ("lit_str_off", _P64), ("lit_str_bytes", _PU8)]


def hip_runtimes() -> list:
    """Distinct libamdhip64 files mapped into this process."""
    seen = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1]
                if "libamdhip64" in p:
                    seen.add(os.path.realpath(p))
    except OSError:
        pass
    return sorted(seen)


def load(path: str = LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise ImportError("libdeltareplay.so is not built (%s); run `make` or __graft_entry__.build()" % path)
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 (DT_NEEDED
    # "libamdhip64.so"), which the loader does not match against /opt/rocm's copy. Loading torch
    # first makes libdeltareplay's DT_NEEDED "libamdhip64.so.7" resolve to torch's runtime, so
    # device buffers can be shared with torch.distributed (RCCL) in the multi-GPU path.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    vp, i32, i64, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    sig = {
        "dr_state_last_error": ([vp], C.c_char_p),
        "dr_comm_last_error": ([vp], C.c_char_p),
        "dr_state_materialize": ([vp, C.POINTER(C.c_uint64)], C.c_int),
        "dr_abi_version": ([], C.c_int),
        "dr_ctx_create": ([C.c_int, C.POINTER(vp)], C.c_int),
        "dr_ctx_destroy": ([vp], None),
        "dr_ctx_set_option": ([vp, i32, i64], C.c_int),
        "dr_ctx_get_option": ([vp, i32, C.POINTER(i64)], C.c_int),
        "dr_last_error": ([vp], C.c_char_p),
        "dr_log_segment": ([vp, C.c_char_p, i64, C.c_char_p, u64, C.POINTER(u64), C.POINTER(i64)], C.c_int),
        "dr_stage": ([vp, C.POINTER(dr_file), i32, C.POINTER(vp)], C.c_int),
        "dr_comm_unique_id": ([C.c_char_p], C.c_int),
        "dr_comm_loopback_id": ([C.c_char_p], C.c_int),
        "dr_comm_create": ([vp, C.c_char_p, i32, i32, C.POINTER(vp)], C.c_int),
        "dr_comm_release": ([vp], C.c_int),
        "dr_replay_sharded": ([vp, vp, i64, C.c_uint32, C.POINTER(vp)], C.c_int),
        "dr_stage_named": ([vp, C.c_char_p, C.POINTER(dr_file), C.POINTER(C.c_char_p), i32, C.POINTER(vp)], C.c_int),
        "dr_stage_log": ([vp, C.c_char_p, i64, C.POINTER(vp)], C.c_int),
        "dr_staged_release": ([vp], C.c_int),
        "dr_staged_bytes": ([vp, C.POINTER(u64), C.POINTER(u64)], C.c_int),
        "dr_staged_plan": ([vp, C.POINTER(u64), i32, C.POINTER(i32)], C.c_int),
        "dr_replay_staged": ([vp, vp, i64, C.c_uint32, C.POINTER(vp)], C.c_int),
        "dr_replay": ([vp, C.POINTER(dr_file), i32, i64, C.c_uint32, C.POINTER(vp)], C.c_int),
        "dr_state_release": ([vp], C.c_int),
        "dr_state_counts": ([vp, C.POINTER(dr_counts)], C.c_int),
        "dr_state_local_counts": ([vp, C.POINTER(dr_counts)], C.c_int),
        "dr_state_nonfile_json": ([vp, C.POINTER(C.c_char_p), C.POINTER(u64)], C.c_int),
        "dr_state_apply": ([vp, vp, vp, C.c_int64, C.c_uint32, C.POINTER(vp)], C.c_int),
        "dr_state_check_checksum": ([vp, C.c_char_p, u64, C.c_char_p, u64, C.POINTER(u64)], C.c_int),
        "dr_state_export": ([vp, i32, C.POINTER(dr_export)], C.c_int),
        "dr_state_record_sums": ([vp, C.POINTER(u64), C.POINTER(u64)], C.c_int),
        "dr_state_record_hashes": ([vp, i32, vp, i64], C.c_int),
        "dr_state_export_plan": ([vp, i32, i64, u64, C.POINTER(_P64), _P64], C.c_int),
        "dr_state_export_range": ([vp, i32, i64, i64, C.POINTER(vp), C.POINTER(dr_export)], C.c_int),
        "dr_range_release": ([vp], C.c_int),
        "dr_filter": ([vp, C.POINTER(dr_predicate), C.POINTER(_P64), _P64], C.c_int),
        "dr_state_write_checkpoint": ([vp, i32, i32, C.c_uint32, C.c_uint64, C.POINTER(C.POINTER(C.c_uint8)),
                                       C.POINTER(C.c_uint64), _P64, _P64], C.c_int),
        "dr_state_scan_order": ([vp, C.POINTER(_P64), _P64], C.c_int),
        "dr_state_set_nonfile_json": ([vp, C.c_char_p, u64, C.c_uint32], C.c_int),
        "dr_state_partition_groups": ([vp, _P64, i64, C.POINTER(_P64), C.POINTER(_P64), _P64], C.c_int),
        "dr_free": ([vp], None),
        "dr_last_timings": ([vp, C.c_char_p, u64, C.POINTER(C.c_float), i32, C.POINTER(i32)], C.c_int),
        "dr_set_timing_only": ([vp, C.c_char_p], C.c_int),
        "dr_set_timing": ([vp, i32], C.c_int),
        "dr_shard_plan": ([vp, C.c_char_p, i64, i32, C.c_char_p, u64, C.POINTER(u64)], C.c_int),
        "dr_stage_log_shard": ([vp, C.c_char_p, i64, i32, i32, C.POINTER(vp)], C.c_int),
        "dr_shard_begin": ([vp, vp, i32, C.POINTER(vp), C.POINTER(u64), C.POINTER(u64)], C.c_int),
        "dr_shard_pack": ([vp, vp, vp], C.c_int),
        "dr_shard_reduce": ([vp, vp, u64, vp, u64, i64, vp], C.c_int),
        "dr_shard_finish": ([vp, vp, C.POINTER(vp)], C.c_int),
        "dr_shard_release": ([vp], C.c_int),
        "dr_parse_commits": ([vp, vp, C.POINTER(vp), C.POINTER(dr_lines)], C.c_int),
        "dr_parsed_release": ([vp], C.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


_LIB = None


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = load()
    return _LIB
