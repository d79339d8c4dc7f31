"""K1 line walker (delta_amd/csrc/json_lane.h), host build, fuzzed against Python's json module.

The walker is the device code of k_json_lines; here it is compiled with g++ and run on seeded
corpora: real Delta log lines (the reference's golden fixtures and the synthetic generator's
formats) and byte-level mutations of them. Expected results restate Spark's PERMISSIVE JSON reader
over Action.logSchema (D/DeltaLogFileIndex.scala:67, D/actions/actions.scala:514-541): invalid JSON
or a non-object root -> error row; unwrap priority; add/remove must be objects; path a string or
null; size / deletionTimestamp integral longs or null. Lines the walker flags `hard` go to the
general parser and are not compared here (they are counted, and must stay rare).
"""
import ctypes as C
import glob
import json
import os
import random
import subprocess

import pytest

from tests.conftest import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "build", "libjsonlane_host.so")

K_NONE, K_ADD, K_REMOVE, K_METADATA, K_TXN, K_PROTOCOL, K_CDC, K_COMMITINFO, K_ERROR = 0, 1, 2, 3, 4, 5, 6, 7, 15
F_HAS_DELTS, F_PATH_ESCAPED, F_PATH_NULL = 1, 4, 8
ORDER = [("add", K_ADD), ("remove", K_REMOVE), ("metaData", K_METADATA), ("txn", K_TXN),
         ("protocol", K_PROTOCOL), ("cdc", K_CDC), ("commitInfo", K_COMMITINFO)]


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", LIB,
                               os.path.join(ROOT, "tests", "native", "json_lane_host.cpp")])
    L = C.CDLL(LIB)
    L.jl_parse.restype = C.c_int
    return L


def walk(lib, line: bytes, align: int, general: bool = False):
    kind, flags = C.c_ubyte(), C.c_ubyte()
    po, pl = C.c_uint(), C.c_uint()
    size, delts = C.c_longlong(), C.c_longlong()
    hard = lib.jl_parse(line, len(line), align, int(general), C.byref(kind), C.byref(flags), C.byref(po), C.byref(pl),
                        C.byref(size), C.byref(delts))
    if hard:
        return None
    out = {"kind": kind.value}
    if kind.value in (K_ADD, K_REMOVE):
        f = flags.value
        if f & F_PATH_NULL:
            path = None
        else:
            raw = line[po.value:po.value + pl.value]
            path = json.loads(b'"' + raw + b'"') if f & F_PATH_ESCAPED else raw.decode("utf-8")
        out.update(path=path, size=size.value, delts=delts.value if f & F_HAS_DELTS else None)
    return out


def _reject_constant(s):
    raise ValueError(s)


class Pairs(list):
    """A JSON object as its (key, value) members in order."""


def expected(line: bytes):
    """Token-stream semantics: every occurrence of a member is converted when it is read (a bad
    value fails the row even if a later duplicate replaces it); the last occurrence is kept."""
    if not line.strip(b" \t\r"):  # Jackson sees no token: the reader emits no row
        return {"kind": K_NONE}
    try:
        obj = json.loads(line, parse_constant=_reject_constant, object_pairs_hook=Pairs)
    except (ValueError, UnicodeDecodeError):
        return {"kind": K_ERROR}
    if not isinstance(obj, Pairs):
        return {"kind": K_ERROR}

    def is_long(v):
        return type(v) is int and -(1 << 63) <= v < (1 << 63)

    top = {}
    for name, v in obj:
        if name in ("add", "remove") and v is not None:
            if not isinstance(v, Pairs):
                return {"kind": K_ERROR}
            rec = {}
            for f, x in v:
                if f == "path" and x is not None and not isinstance(x, str):
                    return {"kind": K_ERROR}
                if f in ("size", "deletionTimestamp") and x is not None and not is_long(x):
                    return {"kind": K_ERROR}
                rec[f] = x
            v = rec
        top[name] = v
    for name, k in ORDER:
        v = top.get(name)
        if v is None:
            continue
        if k in (K_ADD, K_REMOVE):
            return {"kind": k, "path": v.get("path"), "size": v.get("size") or 0,
                    "delts": v.get("deletionTimestamp")}
        return {"kind": k}
    return {"kind": K_NONE}


def corpus():
    lines = []
    for fn in sorted(glob.glob(os.path.join(GOLDEN, "ref", "*", "_delta_log", "*.json"))):
        with open(fn, "rb") as f:
            lines += [l for l in f.read().split(b"\n") if l]
    from delta_amd.testing import synth as S
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        S.build_config(1, d, scale=0.01)
        for fn in sorted(glob.glob(os.path.join(d, "_delta_log", "*.json")))[:3]:
            with open(fn, "rb") as f:
                lines += [l for l in f.read().split(b"\n") if l][:20]
    with tempfile.TemporaryDirectory() as d:
        S.build_config(3, d, scale=0.0002)
        for fn in sorted(glob.glob(os.path.join(d, "_delta_log", "*.json")))[:2]:
            with open(fn, "rb") as f:
                lines += [l for l in f.read().split(b"\n") if l][:20]
    hand = [
        b'', b'   ', b'{}', b'[]', b'1', b'"x"', b'null', b'{"add":null}', b'{"add":{}}', b'{"add":1}',
        b'{"add":[]}', b'{"add":"x"}', b'{"remove":{"path":null}}', b'{"add":{"path":"a","size":null}}',
        b'{"add":{"path":"a","size":1.5}}', b'{"add":{"path":"a","size":"1"}}', b'{"add":{"path":1}}',
        b'{"add":{"path":"a","size":9223372036854775807}}', b'{"add":{"path":"a","size":9223372036854775808}}',
        b'{"add":{"path":"a","size":-9223372036854775808}}', b'{"add":{"path":"a","size":-0}}',
        b'{"add":{"path":"a","size":01}}', b'{"add":{"path":"a\\"b","size":1}}', b'{"add":{"path":"a\\\\","size":1}}',
        b'{"add":{"path":"a\\u0041","size":1}}', b'{"add":{"path":"a\\x","size":1}}', b'{"add":{"path":"\\/"}}',
        b'{"remove":{"path":"p","deletionTimestamp":null}}', b'{"remove":{"path":"p","deletionTimestamp":5}}',
        b'{"add":{"path":"a"},"add":null}', b'{"add":null,"remove":{"path":"b"}}',
        b'{"add":{"path":"a","path":"b"}}', b'{"add":{"path":"a"},"remove":{"path":"b"}}',
        b'{"metaData":{"id":"x"},"protocol":{"minReaderVersion":1}}', b'{"txn":{"appId":"a","version":3}}',
        b'{"commitInfo":{}}', b'{"cdc":{"path":"c"}}', b'{"unknown":{"add":{"path":"x"}}}',
        b'{"add":{"path":"a"}} ', b' {"add":{"path":"a"}}', b'{"add":{"path":"a"}}x', b'{"add":{"path":"a"}}}',
        b'{"add":{"path":"a"}', b'{"add":{"path":"a}}', b'{"add" {"path":"a"}}', b'{"add":{"path":"a",}}',
        b'{"add":{"path":"a" "size":1}}', b'{"add":{"path":"a","size":1 2}}', b'{"a":tru}', b'{"a":true}',
        b'{"a":truex}', b'{"a":[1,2,{"b":[]}]}', b'{"a":[1,]}', b'{"a":[,1]}', b'{"a":{"b":1,"c":[true,false,null]}}',
        b'{"a":1e5}', b'{"a":1E+5}', b'{"a":1.}', b'{"a":.5}', b'{"a":-}', b'{"a":"\x01"}', b'{"a":NaN}',
        b'{"add":{"path":"a","size":1e3}}', b'{"add":{"path":"' + b"x" * 300 + b'","size":7}}',
        b'{"add":{"stats":"' + b'\\"' * 40 + b'","path":"q"}}', b'{"add":{"path":"' + b'\\\\' * 17 + b'"}}',
        b'{"' + b"k" * 40 + b'":1,"add":{"path":"z"}}', b'{"add":{"partitionValues":{"path":"no"},"path":"yes"}}',
        b'{"add":{"tags":{"size":"x"},"size":3,"path":"t"}}', b'{"add":{"path":"a","size":5,"size":null}}',
        # decided by the General walker (k_json_hard): tabs / CR, escaped member names, deep nesting
        b'{\t"add":{"path":"a","size":1}}\r', b'{"a\\u0064d":{"p\\u0061th":"x","size":2}}',
        b'{"add":{"\\u0070ath":"y","si\\u007Ae":3}}', b'{"re\\u006dove":{"path":"z","deletionTimestamp":4}}',
        b'{"x":' + b"[" * 70 + b"]" * 70 + b',"add":{"path":"d"}}', b'{"x":' + b"[" * 70 + b"]" * 69 + b'}',
        b'{"x":' + b"[{}," * 40 + b"0" + b"]" * 40 + b',"remove":{"path":"e"}}', b'{"a":\x0b1}',
        # integer decoding at every digit count and sign (word-load fast path vs the byte loop)
        b'{"add":{"path":"a","size":-01}}', b'{"add":{"path":"a","size":-}}', b'{"add":{"path":"a","size":00}}',
        b'{"add":{"path":"a","size":9999999999999999999}}', b'{"add":{"path":"a","size":18446744073709551615}}',
        b'{"add":{"path":"a","size":18446744073709551616}}', b'{"add":{"path":"a","size":-9223372036854775809}}',
        b'{"add":{"path":"a","size":1234567890123456789}}', b'{"add":{"path":"a","size":-1234567890123456789}}',
        b'{"add":{"path":"a","size":-0.0}}', b'{"add":{"path":"a","size":1x}}', b'{"add":{"path":"a","size":nul}}',
        b'{"add":{"path":"a","size":nulll}}', b'{"add":{"path":"a","size":falsey}}', b'{"add":{"path":"a","size":truE}}',
        # strings of 4096+ bytes (open/close token pair instead of one string token), unclosed strings
        b'{"add":{"path":"' + b"y" * 5000 + b'","size":9}}', b'{"add":{"stats":"' + b'\\"' * 2100 + b'","path":"w"}}',
        b'{"' + b"k" * 4095 + b'":1,"remove":{"path":"v"}}', b'{"' + b"k" * 4096 + b'":1,"remove":{"path":"v"}}',
        b'{"add":{"path":"a"}}"', b'{"a":"xyz', b'"', b'{"a":"b","', b'{"add":{"path":"a\\"}}',
    ] + [b'{"remove":{"path":"r","deletionTimestamp":%s%s}}' % (sg, b"123456789012345678901"[:k])
         for k in range(1, 22) for sg in (b"", b"-")]
    return lines + hand


MUT_CHARS = b'"\\{}[]:, 0123456789aentrulsfx-.e\x01\t\r'


def mutate(rng: random.Random, line: bytes) -> bytes:
    b = bytearray(line)
    for _ in range(rng.choice([1, 1, 1, 2, 3])):
        if not b:
            b.extend(rng.choice([b"{", b'"', b"}"]))
            continue
        op = rng.randrange(5)
        i = rng.randrange(len(b))
        if op == 0:
            del b[i]
        elif op == 1:
            b.insert(i, rng.choice(MUT_CHARS))
        elif op == 2:
            b[i] = rng.choice(MUT_CHARS)
        elif op == 3:
            j = min(len(b), i + rng.randrange(1, 12))
            b[i:i] = b[i:j]
        else:
            j = min(len(b), i + rng.randrange(1, 20))
            del b[i:j]
    return bytes(b)


def _check(lib, line, align, stats):
    exp = expected(line)
    gen = walk(lib, line, align, general=True)
    assert gen == exp, ("general", line, align, gen, exp)
    got = walk(lib, line, align)
    if got is None:
        stats["hard"] += 1
        return
    assert got == exp, (line, align, got, exp)
    stats[exp["kind"]] = stats.get(exp["kind"], 0) + 1


def test_corpus_all_alignments(lib):
    stats = {"hard": 0}
    lines = corpus()
    for line in lines:
        for align in range(16):
            _check(lib, line, align, stats)
    assert stats["hard"] <= 16 * 8, stats  # only the General-mode cases at the end of the corpus
    assert stats.get(K_ADD, 0) > 0 and stats.get(K_REMOVE, 0) > 0 and stats.get(K_ERROR, 0) > 0


def test_mutations(lib):
    rng = random.Random(0xDE17A)
    base = corpus()
    stats = {"hard": 0}
    n = 0
    for _ in range(int(os.environ.get("JL_FUZZ", "40000"))):
        line = mutate(rng, rng.choice(base))
        if b"\n" in line:
            continue
        try:
            line.decode("utf-8")
        except UnicodeDecodeError:
            continue
        _check(lib, line, rng.randrange(16), stats)
        n += 1
    # mutations stay mostly decidable by the walker itself
    assert stats["hard"] < n // 10, stats
    assert stats.get(K_ERROR, 0) > n // 10 and stats.get(K_ADD, 0) > n // 20, stats


def test_classify_masks(lib):
    """The window classifier (nibble-transposed class masks) equals a per-byte restatement of the
    quote / backslash / structural / space / control classes on 1M random windows."""
    lib.jl_classify_check.restype = C.c_longlong
    lib.jl_classify_check.argtypes = [C.c_ulonglong, C.c_longlong]
    assert lib.jl_classify_check(0x5EED, 1_000_000) == 0
