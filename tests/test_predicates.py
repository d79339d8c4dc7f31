"""Host side of K5 on CPU: metadata/data predicate split, column resolution and the lowering of
expressions to the postfix program, checked by running the program with a small stack machine
(the semantics the device kernel implements) against the oracle's tree evaluation."""
import itertools
import random

import pytest

from delta_amd import predicates as P
from oracle import delta_oracle as O
from tests import filter_corpus as F

SCHEMA = {"part": "integer", "d": "date", "b": "boolean", "s": "string", "big": "long"}
TYPE_NAME = {v: k for k, v in P.TYPE_CODE.items()}


def run_program(prog, pv):
    def cast(c):
        name, t = prog.cols[c]
        v = O.cast_string((pv or {}).get(name), TYPE_NAME[t])
        return v.encode() if isinstance(v, str) else v

    st = []
    for op, arg in prog.ops:
        if op == P.OP_COL:
            st.append(cast(arg))
        elif op == P.OP_LIT:
            st.append(prog.lits[arg][1])
        elif op in (2, 3, 4, 5, 6, 7):
            y, x = st.pop(), st.pop()
            st.append(None if x is None or y is None else
                      {2: x == y, 3: x != y, 4: x < y, 5: x <= y, 6: x > y, 7: x >= y}[op])
        elif op == 8:
            y, x = st.pop(), st.pop()
            st.append((x is None and y is None) or (x is not None and y is not None and x == y))
        elif op == 9:
            lits = st[len(st) - arg:]
            del st[len(st) - arg:]
            x = st.pop()
            if x is None:
                st.append(None)
            elif any(l is not None and l == x for l in lits):
                st.append(True)
            else:
                st.append(None if any(l is None for l in lits) else False)
        elif op in (10, 11):
            x = st.pop()
            st.append((x is None) if op == 10 else (x is not None))
        elif op == 12:
            y, x = st.pop(), st.pop()
            st.append(False if (x is False or y is False) else (None if (x is None or y is None) else True))
        elif op == 13:
            y, x = st.pop(), st.pop()
            st.append(True if (x is True or y is True) else (None if (x is None or y is None) else False))
        elif op == 14:
            x = st.pop()
            st.append(None if x is None else (not x))
    assert len(st) == 1
    return st[0] is True


def test_lowering_matches_oracle_on_corpus():
    pvs = [F._pv(i) for i in range(300)] + [None, {}]
    for preds in F.PREDICATES:
        prog = P.build_program(SCHEMA, preds)
        for pv in pvs:
            want = all(O.eval_predicate(e, pv, SCHEMA) is True for e in preds)
            assert run_program(prog, pv) == want, (preds, pv)


def test_split_metadata_and_data_predicates():
    e = ("and", ("and", ("=", ("col", "P"), ("lit", "integer", 1)), (">", ("col", "x"), ("lit", "integer", 2))),
         ("or", ("=", ("col", "`p`"), ("lit", "integer", 3)), ("isnull", ("col", "q"))))
    meta, data = P.split_metadata_and_data_predicates(e, ["p", "q"])
    assert meta == [("=", ("col", "P"), ("lit", "integer", 1)),
                    ("or", ("=", ("col", "`p`"), ("lit", "integer", 3)), ("isnull", ("col", "q")))]
    assert data == [(">", ("col", "x"), ("lit", "integer", 2))]
    prog = P.build_program({"p": "integer", "q": "string"}, meta)
    assert [c for c, _ in prog.cols] == ["p", "q"]


def test_program_errors():
    with pytest.raises(P.PredicateError):
        P.build_program({"p": "double"}, [("=", ("col", "p"), ("lit", "integer", 1))])
    with pytest.raises(P.PredicateError):
        P.build_program({"p": "integer"}, [("=", ("col", "zz"), ("lit", "integer", 1))])
    with pytest.raises(P.PredicateError):
        P.build_program({"p": "date"}, [("=", ("col", "p"), ("lit", "date", "2020-02-30"))])


def test_date_literals_follow_cast_grammar():
    for s in ["2020-03-01", "2020-3-1", "2020", "2020-03-01 10:00", " 2021-12-31T00"]:
        assert P._date_days(s) == O.cast_string(s, "date")
    for s in ["2020-13-01", "20200101", "2021-02-29", ""]:
        assert P._date_days(s) is None
