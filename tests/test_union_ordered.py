"""Time-ordered Union through the engine (union_node.cc:172-258): the reference's own cases
(src/carnot/exec/union_node_test.cc:107-509, plan kUnionOperatorOrdered of
src/carnot/planpb/test_proto.h:341-353: rows_per_batch 5, output (abc STRING, time_ TIME64NS),
parent 0 maps (0, 1), parent 1 maps (1, 0)) fed as RowBatchData messages to two GRPC sources.
The merged output -- rows, batch boundaries and eow/eos -- depends only on each parent's batch
sequence, not on the interleaving, so the expected batches are the reference test's.  Plus a
randomized merge against a stable sort by (time, parent) and an explain check on CPU."""
import numpy as np
import pytest

from pixie_amd import host_engine as H
from pixie_amd import plans as P
from pixie_amd.device import Column

S, T = P.STRING, P.TIME64NS


def _p0(strs, times, eow=False, eos=False):  # parent 0: (abc STRING, time_ TIME64NS)
    return H.rowbatch_to_proto([Column.from_values(S, strs), Column(T, values=np.array(times, dtype=np.int64))], eow, eos)


def _p1(times, strs, eow=False, eos=False):  # parent 1: (time_ TIME64NS, abc STRING)
    return H.rowbatch_to_proto([Column(T, values=np.array(times, dtype=np.int64)), Column.from_values(S, strs)], eow, eos)


def _plan(rows_per_batch=5):
    return P.dag_plan([(1, P.grpc_source_op([S, T], ["abc", "time_"]), []),
                       (2, P.grpc_source_op([T, S], ["time_", "abc"]), []),
                       (3, P.union_op(["abc", "time_"], [[0, 1], [1, 0]], rows_per_batch), [1, 2]),
                       (4, P.sink_op("out"), [3])])


def _strs(c):
    return [bytes(c.data[c.offsets[i]:c.offsets[i + 1]]).decode() for i in range(len(c.offsets) - 1)]


def _run(p0, p1, rows_per_batch=5):
    e = H.Engine(0)
    try:
        res, _ = e.execute_grpc(_plan(rows_per_batch), {}, {1: p0, 2: p1})
    finally:
        e.close()
    return [(_strs(b["cols"][0]), list(map(int, b["cols"][1].values)), b["eow"], b["eos"]) for b in res["out"]]


def test_ordered_union_explains_on_cpu():
    assert "UnionNode(ordered by time_)" in H.explain(_plan(), {})


CASES = {
    "ordered_disjoint": (
        [_p0("ABCD", [0, 1, 2, 3]), _p0("EFG", [4, 5, 6]), _p0("H", [100], True, True)],
        [_p1([10, 11], "ZY"), _p1([20, 25, 30, 40], "XWVU", True, True)],
        [("ABCDE", [0, 1, 2, 3, 4], False, False), ("FGZYX", [5, 6, 10, 11, 20], False, False),
         ("WVUH", [25, 30, 40, 100], True, True)]),
    "ordered_partial_overlap_string": (
        [_p0("AB", [0, 1]), _p0("EFGHIJKL", [4, 5, 6, 7, 8, 9, 10, 11], True, True)],
        [_p1([1, 2], "bc"), _p1([4, 5], "ef"), _p1([11], "l", True, True)],
        [("ABbcE", [0, 1, 1, 2, 4], False, False), ("eFfGH", [4, 5, 5, 6, 7], False, False),
         ("IJKLl", [8, 9, 10, 11, 11], True, True)]),
    "ordered_full_overlap": (
        [_p0("ABCDE", [0, 1, 2, 3, 4]), _p0("FGHIJ", [5, 6, 7, 8, 9]), _p0("KLMNO", [10, 11, 12, 13, 14], True, True)],
        [_p1([0, 1, 2, 3, 4], "abcde"), _p1([5, 6, 7, 8, 9], "fghij", True, True)],
        [("AaBbC", [0, 0, 1, 1, 2], False, False), ("cDdEe", [2, 3, 3, 4, 4], False, False),
         ("FfGgH", [5, 5, 6, 6, 7], False, False), ("hIiJj", [7, 8, 8, 9, 9], False, False),
         ("KLMNO", [10, 11, 12, 13, 14], True, True)]),
    "no_rows_parent": (
        [_p0("ABCD", [0, 1, 2, 3]), _p0("H", [100], True, True)],
        [_p1([], [], True, True)],
        [("ABCDH", [0, 1, 2, 3, 100], True, True)]),
    "many_empty_rbs": (
        [_p0("AB", [0, 1]), _p0([], []), _p0([], []), _p0("EFGHIJKL", [4, 5, 6, 7, 8, 9, 10, 11], True, True)],
        [_p1([1, 2], "bc"), _p1([], []), _p1([4, 5], "ef"), _p1([11], "l"), _p1([], []), _p1([], [], True, True)],
        [("ABbcE", [0, 1, 1, 2, 4], False, False), ("eFfGH", [4, 5, 5, 6, 7], False, False),
         ("IJKLl", [8, 9, 10, 11, 11], False, False), ("", [], True, True)]),
    "all_multiple_empty_rbs": (
        [_p0([], []), _p0([], []), _p0([], []), _p0([], [], True, True)],
        [_p1([], [], True, True)],
        [("", [], True, True)]),
    "all_single_empty_rbs": (
        [_p0([], [], True, True)],
        [_p1([], [], True, True)],
        [("", [], True, True)]),
    "end_on_empty_rb": (
        [_p0(["hello"], [123]), _p0([], [], True, True)],
        [_p1([], [], True, True)],
        [(["hello"], [123], True, True)]),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_reference_union_cases(case):
    p0, p1, want = CASES[case]
    got = _run(p0, p1)
    assert got == [(list(s), t, eow, eos) for s, t, eow, eos in want]


@pytest.mark.gpu
def test_randomized_merge_matches_stable_sort():
    """Each parent's times ascend (the table store's order); the output is the stable merge by
    (time, parent index), cut into rows_per_batch batches, the last one carrying eow / eos."""
    rng = np.random.default_rng(7)
    per_parent = []
    for p in range(2):
        n = int(rng.integers(3000, 6000))
        t = np.sort(rng.integers(0, 2000, n))
        s = [f"p{p}r{i}" for i in range(n)]
        cuts = np.sort(rng.choice(np.arange(1, n), 12, replace=False))
        bounds = [0, *cuts.tolist(), n]
        msgs = []
        for k, (lo, hi) in enumerate(zip(bounds, bounds[1:])):
            last = k == len(bounds) - 2
            msgs.append(_p0(s[lo:hi], t[lo:hi], last, last) if p == 0 else _p1(t[lo:hi], s[lo:hi], last, last))
            if k % 4 == 1:  # empty batches in the stream are skipped
                msgs.append(_p0([], []) if p == 0 else _p1([], []))
        per_parent.append((t, s, msgs))
    got = _run(per_parent[0][2], per_parent[1][2], rows_per_batch=1000)
    rows = sorted([(int(t), p, i, s) for p in range(2) for i, (t, s) in enumerate(zip(per_parent[p][0], per_parent[p][1]))])
    want_s = [r[3] for r in rows]
    want_t = [r[0] for r in rows]
    flat_s = [x for b in got for x in b[0]]
    flat_t = [x for b in got for x in b[1]]
    assert flat_s == want_s and flat_t == want_t
    sizes = [len(b[1]) for b in got]
    assert all(x == 1000 for x in sizes[:-1]) and sizes[-1] == len(rows) - 1000 * (len(sizes) - 1)
    assert [b[3] for b in got] == [False] * (len(got) - 1) + [True]
