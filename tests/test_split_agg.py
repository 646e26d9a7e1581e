"""Split aggregation: planpb AggregateOperator with partial_agg /
finalize_results (plan.proto:250-257) as the distributed splitter emits them
(partial_op_mgr.cc:47-83).

- partial_agg && !finalize_results: output = groups + serialized_expressions STRING
  (operators.cc:251-257), every UDA's Serialize() bytes back to back in plan order
  (count u64, sum i64|f64, mean {u64 size, f64 sum}, min/max native; math_ops.h:583-772).
- !partial_agg && finalize_results: input = groups + serialized_expressions; states are
  Deserialize()d and Merge()d per group, then finalized.

The reference's AggNode ignores both flags (agg_node.cc has no partial path), so there is no
executable reference here: parity is anchored on the UDAs' own Serialize/Merge/Finalize
contracts (math_ops.h, udf/test_utils.h:157-162 round trip) and on split == unsplit over the
same rows.  CPU tests pin the oracle (and the state layout against numpy); GPU tests compare the
device halves with the oracle through the C++ host engine."""
import struct

import numpy as np
import pytest

import oracle_client as oc
from pixie_amd import host_engine as H
from pixie_amd import plans as P
from pixie_amd.device import Column, datagen_http_events

INT64, FLOAT64, STRING = 2, 4, 5
# (kind, type) of each split_values() entry, in plan order.
VALUES = [("count", "i"), ("mean", "i"), ("sum", "i"), ("min", "i"), ("max", "i"),
          ("mean", "f"), ("sum", "f"), ("min", "f"), ("max", "f")]
STATE_SIZE = {"count": 8, "mean": 16, "sum": 8, "min": 8, "max": 8}
REC = sum(STATE_SIZE[k] for k, _ in VALUES)


def http_shards(n_shards, rows, addr_keys=2000, batch=4096):
    """Row shards of one synthetic http_events table (counter-based generator: a shard is rows
    [s*rows, (s+1)*rows) of the same table), as 4096-row batches."""
    out = []
    for s in range(n_shards):
        cols = datagen_http_events(20250117, s * rows, rows, threads=4, n_pair_keys=addr_keys)
        out.append([[c.slice(a, min(a + batch, rows)) for c in cols] for a in range(0, rows, batch)])
    return out


def http_table(batches):
    return {"http_events": {"types": P.HTTP_TYPES, "names": P.HTTP_NAMES, "batches": batches}}


def decode_states(raw: bytes):
    """serialized_expressions record -> one state tuple per VALUES entry."""
    assert len(raw) == REC, len(raw)
    out, off = [], 0
    for kind, t in VALUES:
        if kind == "count":
            out.append(struct.unpack_from("<Q", raw, off))
        elif kind == "mean":
            out.append(struct.unpack_from("<Qd", raw, off))
        else:
            out.append(struct.unpack_from("<q" if t == "i" else "<d", raw, off))
        off += STATE_SIZE[kind]
    return out


def batches_rows(batches, ng):
    """{group key tuple: remaining columns as a tuple} over all batches (as bytes for strings)."""
    rows = {}
    for b in batches:
        lists = [c.to_list() for c in b["cols"]]
        for i in range(b["rows"]):
            k = tuple(lists[g][i] for g in range(ng))
            assert k not in rows, ("duplicate group", k)
            rows[k] = tuple(l[i] for l in lists[ng:])
    return rows


def partial_table(results, ng):
    """Concatenate the partial outputs (one sink per shard) as the merge plan's input table."""
    batches = []
    for res in results:
        for b in res:
            if b["rows"]:
                batches.append(b["cols"])
    types = [STRING] * ng + [STRING]
    return {"types": types, "names": [f"g{i}" for i in range(ng)] + ["serialized_expressions"],
            "batches": batches}


def as_bytes(s: str) -> bytes:
    return s.encode(errors="surrogateescape")


def check_final(got, ref, what):
    assert set(got) == set(ref), (what, "group sets differ", len(got), len(ref))
    for k in ref:
        for (kind, t), a, b in zip(VALUES, got[k], ref[k]):
            if t == "f" and kind in ("mean", "sum"):
                assert abs(a - b) <= 1e-6 * max(1.0, abs(b)), (what, k, kind, a, b)
            elif t == "f":
                assert a == b, (what, k, kind, a, b)
            elif kind == "mean":
                assert abs(a - b) <= 1e-6 * abs(b), (what, k, kind, a, b)
            else:
                assert a == b, (what, k, kind, a, b)


# ------------------------------------------------------------------------------------------
# CPU: the oracle's split halves.
# ------------------------------------------------------------------------------------------
def test_oracle_partial_states_match_numpy():
    """The partial half's serialized_expressions hold exactly the UDA states (pinned against a
    numpy group-by of the same rows, not against the oracle's own aggregate)."""
    (shard,) = http_shards(1, 20000)
    res = oc.execute_plan(P.split_source_plan(), http_table(shard))["partial"]
    assert len(res) == 1 and res[0]["eos"]
    got = {k: decode_states(as_bytes(v[0])) for k, v in batches_rows(res, 2).items()}
    # numpy reference of the same filter + group-by
    cols = {n: np.concatenate([b[P.HE[n]].to_list() if P.HTTP_TYPES[P.HE[n]] == STRING else b[P.HE[n]].values
                               for b in shard]) for n in P.SPLIT_SRC_COLS}
    sel = cols["resp_status"] >= 400
    groups = {}
    for i in np.nonzero(sel)[0]:
        groups.setdefault((cols["pod"][i], cols["remote_addr"][i]), []).append(i)
    assert set(got) == set(groups)
    for k, idx in groups.items():
        lat = cols["latency"][idx]
        body = cols["resp_body_size"][idx]
        ms = lat.astype(np.float64) / 1e6
        st = got[k]
        n = len(idx)
        assert st[0] == (n,)
        assert st[1][0] == n and abs(st[1][1] - float(lat.sum())) <= 1e-9 * abs(float(lat.sum()))
        assert st[2] == (int(body.sum()),) and st[3] == (int(lat.min()),) and st[4] == (int(lat.max()),)
        assert st[5][0] == n and abs(st[5][1] - ms.sum()) <= 1e-9 * ms.sum()
        assert abs(st[6][0] - ms.sum()) <= 1e-9 * ms.sum()
        assert st[7] == (ms.min(),) and st[8] == (ms.max(),)


def test_oracle_split_equals_full_aggregate():
    shards = http_shards(3, 12000)
    parts = [oc.execute_plan(P.split_source_plan(), http_table(s))["partial"] for s in shards]
    merged = oc.execute_plan(P.split_merge_plan("partials", [STRING, STRING]), {"partials": partial_table(parts, 2)})
    full = oc.execute_plan(P.split_source_plan(partial_agg=False, sink="output"),
                           http_table([b for s in shards for b in s]))
    check_final(batches_rows(merged["output"], 2), batches_rows(full["output"], 2), "oracle merge vs full")


def test_oracle_split_no_groups_and_empty_input():
    shards = http_shards(2, 5000)
    parts = [oc.execute_plan(P.split_source_plan(groups=()), http_table(s))["partial"] for s in shards]
    assert [b["rows"] for p in parts for b in p] == [1, 1]
    merged = oc.execute_plan(P.split_merge_plan("partials", []), {"partials": partial_table(parts, 0)})
    full = oc.execute_plan(P.split_source_plan(groups=(), partial_agg=False, sink="output"),
                           http_table([b for s in shards for b in s]))
    check_final(batches_rows(merged["output"], 0), batches_rows(full["output"], 0), "no groups")
    # A no-groups partial over no rows serializes the initial states (count 0, mean {0, 0.0},
    # min = numeric max, max = numeric_limits::min()).
    empty = oc.execute_plan(P.split_source_plan(groups=()), http_table([]))["partial"]
    st = decode_states(as_bytes(empty[0]["cols"][0].to_list()[0]))
    assert st[0] == (0,) and st[1] == (0, 0.0) and st[3] == (2 ** 63 - 1,) and st[4] == (-2 ** 63,)
    assert st[7] == (np.finfo(np.float64).max,) and st[8] == (np.finfo(np.float64).tiny,)


def test_oracle_split_rejects_unsplittable_and_bad_records():
    q = [P.agg_expr("quantiles", [P.col(4)], [FLOAT64])]
    with pytest.raises(oc.OracleError) as e:
        oc.execute_plan(P.split_source_plan(values=q), http_table([]))
    assert e.value.code == 10  # UNIMPLEMENTED: QuantilesUDA has no Serialize
    bad = {"types": [STRING, STRING], "names": ["g0", "serialized_expressions"],
           "batches": [[Column.from_values(STRING, [b"a"]), Column.from_values(STRING, [b"\0" * (REC - 1)])]]}
    with pytest.raises(oc.OracleError) as e:
        oc.execute_plan(P.split_merge_plan("partials", [STRING]), {"partials": bad})
    assert e.value.code == 3


def test_engine_lowers_split_halves():
    """No device: the partial half is one fused agg with a STRING state output; the merge half
    reads state words (op 80) at the Serialize() offsets and merges mean as MEAN_MERGE (7)."""
    txt = H.explain(P.split_source_plan(), {"http_events": {"types": P.HTTP_TYPES, "batches": []}})
    agg = [l for l in txt.splitlines() if "GpuAggNode" in l][0]
    assert "fused" in agg and agg.endswith("out=[STRING,STRING,STRING]")
    parts = {"partials": {"types": [STRING, STRING, STRING], "batches": []}}
    lines = H.explain(P.split_merge_plan("partials", [STRING, STRING]), parts).splitlines()
    udas = [l.split() for l in lines if "uda kind=" in l]
    kinds = [u[1] for u in udas]
    assert kinds == ["kind=2", "kind=7", "kind=2", "kind=4", "kind=5", "kind=7", "kind=2", "kind=4", "kind=5"]
    # state word offsets: count@0, mean sum@16 (size@8), sum@24, min@32, max@40, mean sum@56 ...
    offs = [int(u[2].split(":")[-1]) for u in udas]
    assert offs == [0, 16, 24, 32, 40, 56, 64, 72, 80]
    assert all(u[2].split("=")[1].startswith("80:") for u in udas)
    out = [l for l in lines if "GpuAggNode" in l][0]
    assert out.endswith("out=[STRING,STRING,INT64,FLOAT64,INT64,INT64,INT64,FLOAT64,FLOAT64,FLOAT64,FLOAT64]")


def test_engine_rejects_partial_quantiles():
    q = [P.agg_expr("quantiles", [P.col(4)], [FLOAT64])]
    with pytest.raises(H.PxcError) as e:
        H.explain(P.split_source_plan(values=q), {"http_events": {"types": P.HTTP_TYPES, "batches": []}})
    assert e.value.code == 10


# ------------------------------------------------------------------------------------------
# GPU: the device halves through the C++ host engine.
# ------------------------------------------------------------------------------------------
def run_engine(plan, tables):
    eng = H.Engine(0)
    try:
        return eng.execute(plan, tables)
    finally:
        eng.close()


@pytest.mark.gpu
def test_device_partial_states_match_oracle():
    (shard,) = http_shards(1, 60000)
    dev = run_engine(P.split_source_plan(), http_table(shard))["partial"]
    ref = oc.execute_plan(P.split_source_plan(), http_table(shard))["partial"]
    D = {k: decode_states(as_bytes(v[0])) for k, v in batches_rows(dev, 2).items()}
    R = {k: decode_states(as_bytes(v[0])) for k, v in batches_rows(ref, 2).items()}
    assert set(D) == set(R) and len(R) > 1000
    for k in R:
        d, r = D[k], R[k]
        assert d[0] == r[0] and d[2] == r[2] and d[3] == r[3] and d[4] == r[4] and d[7] == r[7] and d[8] == r[8], k
        for i in (1, 5):  # mean {size, sum}
            assert d[i][0] == r[i][0] and abs(d[i][1] - r[i][1]) <= 1e-9 * abs(r[i][1]), (k, i)
        assert abs(d[6][0] - r[6][0]) <= 1e-9 * abs(r[6][0]), k


@pytest.mark.gpu
def test_device_split_equals_full_aggregate():
    shards = http_shards(4, 40000)
    dparts = [run_engine(P.split_source_plan(), http_table(s))["partial"] for s in shards]
    full = oc.execute_plan(P.split_source_plan(partial_agg=False, sink="output"),
                           http_table([b for s in shards for b in s]))
    ref = batches_rows(full["output"], 2)
    # device merge of the device partials
    dm = run_engine(P.split_merge_plan("partials", [STRING, STRING]), {"partials": partial_table(dparts, 2)})
    check_final(batches_rows(dm["output"], 2), ref, "device merge of device partials")
    # device merge of the oracle's partials (the wire format is the same on both sides)
    oparts = [oc.execute_plan(P.split_source_plan(), http_table(s))["partial"] for s in shards]
    dm2 = run_engine(P.split_merge_plan("partials", [STRING, STRING]), {"partials": partial_table(oparts, 2)})
    check_final(batches_rows(dm2["output"], 2), ref, "device merge of oracle partials")
    # oracle merge of the device partials
    om = oc.execute_plan(P.split_merge_plan("partials", [STRING, STRING]), {"partials": partial_table(dparts, 2)})
    check_final(batches_rows(om["output"], 2), ref, "oracle merge of device partials")


@pytest.mark.gpu
def test_device_split_no_groups_and_empty():
    shards = http_shards(2, 8000)
    dparts = [run_engine(P.split_source_plan(groups=()), http_table(s))["partial"] for s in shards]
    assert [b["rows"] for p in dparts for b in p] == [1, 1]
    dm = run_engine(P.split_merge_plan("partials", []), {"partials": partial_table(dparts, 0)})
    full = oc.execute_plan(P.split_source_plan(groups=(), partial_agg=False, sink="output"),
                           http_table([b for s in shards for b in s]))
    check_final(batches_rows(dm["output"], 0), batches_rows(full["output"], 0), "device no groups")
    empty_d = run_engine(P.split_source_plan(groups=()), http_table([]))["partial"]
    empty_o = oc.execute_plan(P.split_source_plan(groups=()), http_table([]))["partial"]
    assert as_bytes(empty_d[0]["cols"][0].to_list()[0]) == as_bytes(empty_o[0]["cols"][0].to_list()[0])
    # grouped partial over no rows: one zero-row batch with the (groups, STRING) relation
    eg = run_engine(P.split_source_plan(), http_table([]))["partial"]
    assert [b["rows"] for b in eg] == [0] and [c.type for c in eg[0]["cols"]] == [STRING, STRING, STRING]


@pytest.mark.gpu
def test_device_merge_rejects_bad_records():
    bad = {"types": [STRING, STRING], "names": ["g0", "serialized_expressions"],
           "batches": [[Column.from_values(STRING, [b"a"]), Column.from_values(STRING, [b"\0" * (REC + 8)])]]}
    with pytest.raises(H.PxcError) as e:
        run_engine(P.split_merge_plan("partials", [STRING]), {"partials": bad})
    assert e.value.code == 3
