"""Shared helpers for the known-answer (golden) fixtures and result comparison."""
from __future__ import annotations

import json
import math
import os
import struct
from collections import Counter
from typing import List, Sequence

from google.protobuf import text_format

from pixie_amd import planpb
from pixie_amd.device import Column

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_kat.json")
STRING, FLOAT64 = 5, 4


def load_kat():
    with open(GOLDEN) as f:
        return json.load(f)


def case_plan(case):
    return text_format.Parse(case["plan"], planpb.Plan())


def case_tables(case):
    if "tables" in case:
        return {name: {"types": t["types"], "flags": None,
                       "batches": [[Column.from_values(ty, vals) for ty, vals in zip(t["types"], b)]
                                   for b in t["batches"]]}
                for name, t in case["tables"].items()}
    inp = case["input"]
    batches = [[Column.from_values(t, vals) for t, vals in zip(inp["types"], b)] for b in inp["batches"]]
    return {"t": {"types": inp["types"], "batches": batches, "flags": inp.get("flags")}}


def ulp_diff(a: float, b: float) -> int:
    if a == b:
        return 0
    if math.isnan(a) and math.isnan(b):
        return 0
    ia = struct.unpack("<q", struct.pack("<d", a))[0]
    ib = struct.unpack("<q", struct.pack("<d", b))[0]
    if ia < 0:
        ia = -(ia & 0x7FFFFFFFFFFFFFFF)
    if ib < 0:
        ib = -(ib & 0x7FFFFFFFFFFFFFFF)
    return abs(ia - ib)


def rows(cols: Sequence) -> List[tuple]:
    lists = [c.to_list() if isinstance(c, Column) else list(c) for c in cols]
    n = len(lists[0]) if lists else 0
    return [tuple(l[i] for l in lists) for i in range(n)]


def _norm(v, tol_ulp):
    if isinstance(v, float):
        if math.isnan(v):
            return "nan"
        return v
    return v


def rows_match(got: List[tuple], want: List[tuple], ordered: bool, tol_ulp: int = 0, rel: float = 0.0) -> bool:
    if len(got) != len(want):
        return False
    if not ordered:
        # sort by the non-float fields, then compare with tolerance
        def key(r):
            return tuple((0, str(x)) if not isinstance(x, float) else (1, "") for x in r)
        got = sorted(got, key=lambda r: tuple(str(x) if not isinstance(x, float) else "" for x in r) + (repr(r),))
        want = sorted(want, key=lambda r: tuple(str(x) if not isinstance(x, float) else "" for x in r) + (repr(r),))
    for g, w in zip(got, want):
        if len(g) != len(w):
            return False
        for a, b in zip(g, w):
            if isinstance(a, float) or isinstance(b, float):
                a, b = float(a), float(b)
                if math.isnan(a) and math.isnan(b):
                    continue
                if ulp_diff(a, b) <= tol_ulp:
                    continue
                if rel and abs(a - b) <= rel * max(abs(a), abs(b)):
                    continue
                return False
            elif a != b:
                return False
    return True


def expected_rows(case, bi):
    b = case["output"]["batches"][bi]
    return rows(b["cols"])


def check_case_output(out, case):
    """Compare executed output batches with a KAT case.  The last `unordered_tail` expected batches
    are one multiset split over that many batches (ExpectRowBatchesData)."""
    want = case["output"]["batches"]
    tail = case.get("unordered_tail", 0)
    assert len(out) == len(want), f"{case['name']}: {len(out)} batches, want {len(want)}"
    for bi, (g, w) in enumerate(zip(out, want)):
        assert (g["eow"], g["eos"]) == (w["eow"], w["eos"]), f"{case['name']} batch {bi} flags"
        assert [c.type for c in g["cols"]] == case["output"]["types"]
    head = len(want) - tail
    for bi in range(head):
        got = rows(out[bi]["cols"])
        assert rows_match(got, expected_rows(case, bi), case["ordered"], case["tol_ulp"]), \
            f"{case['name']} batch {bi}: {got} != {expected_rows(case, bi)}"
    if tail:
        got = [r for bi in range(head, len(want)) for r in rows(out[bi]["cols"])]
        exp = [r for bi in range(head, len(want)) for r in expected_rows(case, bi)]
        assert rows_match(got, exp, False, case["tol_ulp"]), f"{case['name']} tail: {got} != {exp}"
