"""Partition-pruning predicates: the host side of K5 (`dr_filter`).

Mirrors the reference's metadata-predicate handling:
  split_metadata_and_data_predicates <- DeltaTableUtils.splitMetadataAndDataPredicates /
                                        isPredicatePartitionColumnsOnly (D/DeltaTable.scala:198-294)
  build_program                      <- DeltaLog.rewritePartitionFilters + filterFileList
                                        (D/DeltaLog.scala:500-547): every partition column becomes
                                        Cast(partitionValues[col] AS partitionSchema(col).type), the
                                        filters are ANDed
  partition_schema                   <- Metadata.partitionSchema (D/actions/actions.scala:370-373)

Expressions are nested tuples (the oracle's format): ("col", name), ("lit", type, value),
(op, a, b) for = != < <= > >= <=>, ("in", a, [lits]), ("isnull", a), ("isnotnull", a),
("and", a, b), ("or", a, b), ("not", a). Types: "string", "byte", "short", "integer", "long",
"date", "boolean". The program is evaluated on the GPU; nothing here evaluates it.
"""
from __future__ import annotations

import ctypes as C
import datetime as _dt
import json
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from . import _native as N

TYPE_CODE = {"string": 0, "byte": 1, "short": 2, "integer": 3, "long": 4, "date": 5, "boolean": 6}
OP_COL, OP_LIT = 0, 1
OP_CODE = {"=": 2, "!=": 3, "<": 4, "<=": 5, ">": 6, ">=": 7, "<=>": 8, "in": 9, "isnull": 10,
           "isnotnull": 11, "and": 12, "or": 13, "not": 14}
_EPOCH = _dt.date(1970, 1, 1)


class PredicateError(ValueError):
    pass


def partition_schema(metadata: Optional[dict]) -> Dict[str, str]:
    """Metadata.partitionSchema: partition column -> Spark type name (ordered as partitionColumns)."""
    if not metadata:
        return {}
    schema = json.loads(metadata["schemaString"])
    fields = {f["name"]: f["type"] for f in schema["fields"]}
    return {c: fields[c] for c in metadata.get("partitionColumns") or []}


def _refs(expr) -> List[str]:
    op = expr[0]
    if op == "col":
        return [expr[1]]
    if op == "lit":
        return []
    if op == "in":
        return _refs(expr[1]) + [r for l in expr[2] for r in _refs(l)]
    return [r for a in expr[1:] for r in _refs(a)]


def _conjuncts(expr) -> List:
    if expr[0] == "and":
        return _conjuncts(expr[1]) + _conjuncts(expr[2])
    return [expr]


def _resolve(name: str, partition_cols: Sequence[str]) -> Optional[str]:
    # rewritePartitionFilters (D/DeltaLog.scala:531-533): backticks stripped, then the session
    # resolver (spark.sql.caseSensitive=false: case-insensitive) finds the partition field
    name = name.strip("`")
    for c in partition_cols:
        if c.lower() == name.lower():
            return c
    return None


def is_partition_only(expr, partition_cols: Sequence[str]) -> bool:
    """DeltaTableUtils.isPredicatePartitionColumnsOnly: every column the expression references is
    a partition column (resolved case-insensitively, as the session resolver does)."""
    return all(_resolve(r, partition_cols) is not None for r in _refs(expr))


def split_metadata_and_data_predicates(expr, partition_cols: Sequence[str]) -> Tuple[List, List]:
    """(metadata-only conjuncts, the rest): a conjunct is metadata-only when every column it
    references is a partition column (D/DeltaTable.scala:198-230)."""
    meta, data = [], []
    for c in _conjuncts(expr):
        refs = _refs(c)
        if all(_resolve(r, partition_cols) is not None for r in refs):
            meta.append(c)
        else:
            data.append(c)
    return meta, data


@dataclass
class Program:
    ops: List[Tuple[int, int]] = field(default_factory=list)
    cols: List[Tuple[str, int]] = field(default_factory=list)      # (exact map key, type code)
    lits: List[Tuple[int, object]] = field(default_factory=list)   # (type code, value | None)


_DATE_RE = re.compile(r"(\d{4})(?:-(\d{1,2})(?:-(\d{1,2})(?:[ T].*)?)?)?")


def _date_days(s: str) -> Optional[int]:
    """Cast(string AS date) of a literal, the same grammar the device applies to partition values."""
    m = _DATE_RE.fullmatch(s.strip(" \t\n\r\x0b\x0c"))
    if not m:
        return None
    try:
        return (_dt.date(int(m.group(1)), int(m.group(2) or 1), int(m.group(3) or 1)) - _EPOCH).days
    except ValueError:
        return None


_INT_BITS = {"byte": 8, "short": 16, "integer": 32, "long": 64}
_WS = " \t\n\r\x0b\x0c"


def cast_partition_value(s: Optional[str], typ: str):
    """Cast(Literal(partitionValues(col)), partition type) on the host, non-ANSI (a failed cast is
    null), as TahoeFileIndex.listFiles builds a partition row (D/files/TahoeFileIndex.scala:61-64):
    integral types from trimmed decimal text in range, booleans from t/true/y/yes/1 and
    f/false/n/no/0, dates as datetime.date, strings unchanged. Same grammar as the device cast."""
    if s is None:
        return None
    if typ == "string":
        return s
    t = s.strip(_WS)
    if typ in _INT_BITS:
        if not re.fullmatch(r"[+-]?\d+", t):
            return None
        v, b = int(t), _INT_BITS[typ]
        return v if -(1 << (b - 1)) <= v < (1 << (b - 1)) else None
    if typ == "boolean":
        tl = t.lower()
        return True if tl in ("t", "true", "y", "yes", "1") else False if tl in ("f", "false", "n", "no", "0") else None
    if typ == "date":
        d = _date_days(t)
        return None if d is None else _EPOCH + _dt.timedelta(days=d)
    if typ in ("float", "double"):
        return java_parse_fp(s, typ == "float")
    if typ == "binary":
        return s.encode("utf-8")
    if typ == "timestamp":
        us = timestamp_micros(s)
        return None if us is None else _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc) + _dt.timedelta(microseconds=us)
    dm = re.fullmatch(r"decimal(?:\((\d+),(\d+)\))?", typ)
    if dm:
        p, sc = (int(dm.group(1)), int(dm.group(2))) if dm.group(1) else (10, 0)
        return decimal_value(s, p, sc)
    raise PredicateError("unsupported partition type %r" % typ)


# ---- the checkpoint's other partitionValues_parsed casts (the device grammar, k_filter.hip) ------
_FP_RE = re.compile(r"[+-]?(?:NaN|Infinity|(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?[fFdD]?)")
_HEXFP_RE = re.compile(r"([+-]?)0[xX]([0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)[pP]([+-]?\d+)[fFdD]?")


def _jtrim(s: str) -> str:
    b, e = 0, len(s)
    while b < e and ord(s[b]) <= 32:
        b += 1
    while e > b and ord(s[e - 1]) <= 32:
        e -= 1
    return s[b:e]


def _round_f32(x):
    """Nearest binary32 to the exact rational x (round half to even), as Float.parseFloat."""
    import struct
    from fractions import Fraction
    if x == 0:
        return 0.0
    if abs(x) >= (Fraction(2) - Fraction(1, 1 << 24)) * Fraction(2) ** 127:  # rounds past FLT_MAX
        return float("inf") if x > 0 else float("-inf")
    fmax = float((Fraction(2) - Fraction(1, 1 << 23)) * Fraction(2) ** 127)
    f = struct.unpack("<f", struct.pack("<f", min(max(float(x), -fmax), fmax)))[0]
    bits = struct.unpack("<I", struct.pack("<f", f))[0]
    best = None
    for b in (bits - 1, bits, bits + 1):
        if b < 0 or b >= 1 << 32:
            continue
        c = struct.unpack("<f", struct.pack("<I", b))[0]
        if c != c or c in (float("inf"), float("-inf")):
            continue
        d = abs(Fraction(c) - x)
        if best is None or d < best[0] or (d == best[0] and b % 2 == 0):
            best = (d, c)
    return best[1]


def java_parse_fp(s: str, is_float: bool):
    """Double.parseDouble / Float.parseFloat, else Spark's special literals (inf, nan, ...)."""
    from fractions import Fraction
    t = _jtrim(s)
    hm = _HEXFP_RE.fullmatch(t)
    if hm:  # Java's hexadecimal significand with a binary exponent
        ip, _, fp = hm.group(2).partition(".")
        x = Fraction(int((ip or "0") + fp, 16), 16 ** len(fp)) * Fraction(2) ** int(hm.group(3))
        v = _round_f32(x) if is_float else (float(x) if x < Fraction(2) ** 1025 else float("inf"))
        return -v if hm.group(1) == "-" else v
    if _FP_RE.fullmatch(t):
        body = t.rstrip("fFdD") if not t.endswith(("NaN", "Infinity")) else t
        if body.lstrip("+-") == "NaN":
            return float("nan")
        if body.lstrip("+-") == "Infinity":
            return float("-inf") if body.startswith("-") else float("inf")
        if is_float:
            v = _round_f32(Fraction(body))
            return -0.0 if v == 0 and body.startswith("-") else v
        return float(body)
    tl = t.lower()
    if tl in ("inf", "+inf", "infinity", "+infinity"):
        return float("inf")
    if tl in ("-inf", "-infinity"):
        return float("-inf")
    if tl == "nan":
        return float("nan")
    return None


def decimal_value(s: str, precision: int, scale: int):
    """Decimal.fromString + changePrecision: BigDecimal of the trimmed text, HALF_UP to `scale`,
    null beyond `precision` digits."""
    import decimal
    t = _jtrim(s)
    if not re.fullmatch(r"[+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?", t):
        return None
    ctx = decimal.Context(prec=100000, rounding=decimal.ROUND_HALF_UP)
    try:
        v = decimal.Decimal(t).quantize(decimal.Decimal(1).scaleb(-scale), context=ctx)
    except decimal.InvalidOperation:
        return None
    unscaled = abs(int(v.scaleb(scale, context=ctx)))
    return None if unscaled >= 10 ** precision else (v if v != 0 else abs(v))


_TS_RE = re.compile(r"([+-]?)(\d{4,6})(?:-(\d{1,2})(?:-(\d{1,2})(?:[ T](\d{1,2}):(\d{1,2})"
                    r"(?::(\d{1,2})(?:\.(\d*))?)?(.*))?)?)?")
_TZ_RE = re.compile(r"(?:Z|(?:UTC|GMT|UT)?(?:([+-])(\d{1,2})(?::?(\d{1,2})(?::?(\d{1,2}))?)?)?)")


def timestamp_micros(s: str) -> Optional[int]:
    """DateTimeUtils.stringToTimestamp with the session zone UTC, the subset the device reads."""
    t = _jtrim(s)
    m = _TS_RE.fullmatch(t)
    if not m:
        return None
    sign, y, mo, d, hh, mi, ss, frac, zone = m.groups()
    y = int(y) * (-1 if sign == "-" else 1)
    try:
        day = (_dt.date(y, int(mo or 1), int(d or 1)) - _EPOCH).days
    except ValueError:
        return None
    hh, mi, ss = int(hh or 0), int(mi or 0), int(ss or 0)
    if hh > 23 or mi > 59 or ss > 59:
        return None
    us = int(((frac or "") + "000000")[:6])
    off = 0
    if zone:
        z = _TZ_RE.fullmatch(_jtrim(zone))
        if not z or not zone.strip():
            return None
        if z.group(1):
            h, mn, sc = int(z.group(2)), int(z.group(3) or 0), int(z.group(4) or 0)
            if h > 18 or mn > 59 or sc > 59:
                return None
            off = (h * 3600 + mn * 60 + sc) * (-1 if z.group(1) == "-" else 1)
    return ((day * 86400 + hh * 3600 + mi * 60 + ss) - off) * 1_000_000 + us


def _lit(typ: str, v):
    """Literal value as the device sees it (the oracle's _lit_value): dates as days since the
    epoch, booleans as 0/1, strings as bytes."""
    if typ not in TYPE_CODE:
        raise PredicateError("unsupported literal type %r" % typ)
    if v is None:
        return None
    if typ == "date":
        if isinstance(v, str):
            days = _date_days(v)
            if days is None:
                raise PredicateError("bad date literal %r" % v)
            return days
        if isinstance(v, _dt.date):
            return (v - _EPOCH).days
        return int(v)
    if typ == "boolean":
        return 1 if v else 0
    if typ == "string":
        return str(v).encode("utf-8")
    return int(v)


def build_program(schema: Dict[str, str], preds: Sequence) -> Program:
    """AND of `preds` lowered to the postfix program of include/deltareplay.h (dr_pred_op)."""
    if not preds:
        raise PredicateError("no predicates")
    p = Program()
    colidx: Dict[str, int] = {}
    parts = list(schema)

    def col(name):
        exact = _resolve(name, parts)
        if exact is None:
            raise PredicateError("%s is not a partition column" % name)
        typ = schema[exact]
        if typ not in TYPE_CODE:
            raise PredicateError("partition column %s has unsupported type %s" % (exact, typ))
        if exact not in colidx:
            colidx[exact] = len(p.cols)
            p.cols.append((exact, TYPE_CODE[typ]))
        p.ops.append((OP_COL, colidx[exact]))

    def lit(typ, v):
        p.lits.append((TYPE_CODE[typ], _lit(typ, v)))
        p.ops.append((OP_LIT, len(p.lits) - 1))

    def emit(e):
        op = e[0]
        if op == "col":
            col(e[1])
        elif op == "lit":
            lit(e[1], e[2])
        elif op == "in":
            emit(e[1])
            for l in e[2]:
                emit(l)
            p.ops.append((OP_CODE["in"], len(e[2])))
        elif op in ("isnull", "isnotnull", "not"):
            emit(e[1])
            p.ops.append((OP_CODE[op], 0))
        elif op in OP_CODE:
            emit(e[1])
            emit(e[2])
            p.ops.append((OP_CODE[op], 0))
        else:
            raise PredicateError("unsupported expression %r" % (op,))

    emit(preds[0])
    for e in preds[1:]:
        emit(e)
        p.ops.append((OP_CODE["and"], 0))
    return p


def lower_program(prog: Program):
    """ctypes dr_predicate for `prog` (+ the buffers that must outlive the call)."""
    keep = []
    nops = len(prog.ops)
    ops = (N.dr_pred_op * max(nops, 1))()
    for i, (o, a) in enumerate(prog.ops):
        ops[i] = N.dr_pred_op(o, a)
    ncols = len(prog.cols)
    names = (C.c_char_p * max(ncols, 1))()
    ctypes_ = (C.c_int32 * max(ncols, 1))()
    for i, (n, t) in enumerate(prog.cols):
        b = C.create_string_buffer(n.encode("utf-8"))
        keep.append(b)
        names[i] = C.cast(b, C.c_char_p)
        ctypes_[i] = t
    nl = len(prog.lits)
    lt = (C.c_int32 * max(nl, 1))()
    li = (C.c_int64 * max(nl, 1))()
    ln = (C.c_uint8 * max(nl, 1))()
    lo = (C.c_int64 * (nl + 1))()
    blob = b""
    for i, (t, v) in enumerate(prog.lits):
        lt[i] = t
        lo[i] = len(blob)
        if v is None:
            ln[i] = 1
        elif isinstance(v, bytes):
            blob += v
        else:
            li[i] = int(v)
    lo[nl] = len(blob)
    lb = (C.c_uint8 * max(len(blob), 1)).from_buffer_copy(blob + b"\0")
    keep += [ops, names, ctypes_, lt, li, ln, lo, lb]
    pred = N.dr_predicate(nops, ops, ncols, names, ctypes_, nl, lt, li, ln, lo, lb)
    return pred, keep
