"""Generate tests/golden/reference_kat.json: the reference's own known-answer vectors for the
hot path, as plan + input batches + expected output.

Inputs and expected values are transcribed from the cited reference tests (data only); the
plans are built with pixie_amd.plans in the operator shapes those tests feed their nodes.
Regenerate with:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from google.protobuf import text_format  # noqa: E402

from pixie_amd import plans as P  # noqa: E402
from pixie_amd._lib import BOOLEAN, FLOAT64, INT64, STRING, TIME64NS  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kat.json")
I, F, S, B, T = INT64, FLOAT64, STRING, BOOLEAN, TIME64NS


def case(name, source, ops, in_types, batches, flags, out_types, expected, ordered=False, tol_ulp=0):
    names = [f"c{i}" for i in range(len(in_types))]
    plan = P.linear_plan([P.source_op("t", in_types, names, list(range(len(in_types))))] + ops + [P.sink_op("out")])
    return {
        "name": name, "source": source, "plan": text_format.MessageToString(plan),
        "input": {"types": in_types, "batches": batches, "flags": flags},
        "output": {"types": out_types, "batches": expected},
        "ordered": ordered, "tol_ulp": tol_ulp,
    }


def minsum(a, b, init=None, fid=0):
    if init is None:
        return P.agg_expr("minsum", [P.col(a), P.col(b)], [I, I], fid=fid)
    return P.agg_expr("minsum_w_init", [P.col(a), P.col(b)], [I, I], fid=fid, init_args=[P.const(I, init)])


def batch(cols, eow, eos):
    return {"cols": cols, "eow": eow, "eos": eos}


cases = []
A = "src/carnot/exec/agg_node_test.cc"
b12 = [[[1, 2, 3, 4], [2, 5, 6, 8]], [[5, 6, 3, 4], [1, 5, 3, 8]]]
cases.append(case("agg.no_groups_blocking", A + ":304-329", [P.agg_op([], [minsum(0, 1)])], [I, I], b12,
                  [[False, False], [True, True]], [I], [batch([[23]], True, True)]))
cases.append(case("agg.zero_row_row_batch", A + ":331-356", [P.agg_op([], [minsum(0, 1)])], [I, I],
                  [b12[0], [[], []]], [[False, False], [True, True]], [I], [batch([[10]], True, True)]))
cases.append(case("agg.single_group_blocking", A + ":358-383", [P.agg_op([0], [minsum(0, 1)])], [I, I],
                  [[[1, 1, 2, 2], [2, 3, 3, 1]], [[5, 6, 3, 4], [1, 5, 3, 8]]], [[False, False], [True, True]], [I, I],
                  [batch([[1, 2, 3, 4, 5, 6], [2, 3, 3, 4, 1, 5]], True, True)]))
cases.append(case("agg.multiple_groups_blocking", A + ":385-413", [P.agg_op([0, 1], [minsum(2, 1)])], [I, I, I],
                  [[[1, 5, 1, 2], [2, 1, 3, 1], [2, 5, 3, 1]], [[5, 1, 3, 3], [1, 2, 3, 3], [1, 3, 3, 8]]],
                  [[False, False], [True, True]], [I, I, I],
                  [batch([[1, 1, 2, 5, 3], [2, 3, 1, 1, 3], [4, 3, 1, 2, 6]], True, True)]))
cases.append(case("agg.multiple_groups_with_string_blocking", A + ":415-444", [P.agg_op([0, 1], [minsum(2, 1)])], [S, I, I],
                  [[["abc", "def", "abc", "fgh"], [2, 1, 3, 1], [2, 5, 3, 1]], [["ijk", "abc", "abc", "def"], [1, 2, 3, 3], [1, 3, 3, 8]]],
                  [[False, False], [True, True]], [S, I, I],
                  [batch([["abc", "def", "abc", "fgh", "ijk", "def"], [2, 1, 3, 1, 1, 3], [4, 1, 6, 1, 1, 3]], True, True)]))
cases.append(case("agg.no_groups_windowed", A + ":446-484", [P.agg_op([], [minsum(0, 1)], windowed=True)], [I, I],
                  b12 + b12, [[False, False], [True, False], [False, False], [True, True]], [I],
                  [batch([[23]], True, False), batch([[23]], True, True)]))
sg = [[[1, 1, 2, 2], [2, 3, 3, 1]], [[5, 6, 3, 4], [1, 5, 3, 8]]]
sg_out = [[1, 2, 3, 4, 5, 6], [2, 3, 3, 4, 1, 5]]
cases.append(case("agg.single_group_windowed", A + ":486-526", [P.agg_op([0], [minsum(0, 1)], windowed=True)], [I, I],
                  sg + sg, [[False, False], [True, False], [False, False], [True, True]], [I, I],
                  [batch(sg_out, True, False), batch(sg_out, True, True)]))
cases.append(case("agg.no_aggregate_expressions", A + ":528-549", [P.agg_op([0], [])], [I, I],
                  [[[2, 1, 3, 1], [2, 5, 3, 1]], [[1, 2, 3, 3], [1, 3, 3, 8]]], [[False, False], [True, True]], [I],
                  [batch([[2, 1, 3]], True, True)]))
cases.append(case("agg.no_groups_blocking_init_args", A + ":551-576", [P.agg_op([], [minsum(0, 1, init=10, fid=1)])], [I, I],
                  b12, [[False, False], [True, True]], [I], [batch([[33]], True, True)]))
cases.append(case("agg.single_group_blocking_init_args", A + ":578-603", [P.agg_op([0], [minsum(0, 1, init=10, fid=1)])], [I, I],
                  sg, [[False, False], [True, True]], [I, I], [batch([[1, 2, 3, 4, 5, 6], [12, 13, 13, 14, 11, 15]], True, True)]))

Fi = "src/carnot/exec/filter_node_test.cc"
eq1 = P.func("eq", [P.col(0), P.const(I, 1)], [I, I])
fin = [[[1, 1, 3, 4], [1, 3, 6, 9], ["ABC", "DEF", "HELLO", "WORLD"]], [[1, 2, 3], [1, 4, 6], ["Hello", "world", "now"]]]
cases.append(case("filter.basic", Fi + ":78-110", [P.filter_op(eq1, [0, 1, 2])], [I, I, S], fin,
                  [[False, False], [True, True]], [I, I, S],
                  [batch([[1, 1], [1, 3], ["ABC", "DEF"]], False, False), batch([[1], [1], ["Hello"]], True, True)], ordered=True))
cases.append(case("filter.column_selection", Fi + ":112-139", [P.filter_op(eq1, [1])], [I, I, S], fin,
                  [[False, False], [True, True]], [I], [batch([[1, 3]], False, False), batch([[1]], True, True)], ordered=True))
cases.append(case("filter.zero_row_row_batch", Fi + ":141-181", [P.filter_op(eq1, [0, 1, 2])], [I, I, S],
                  [fin[0], [[], [], []], fin[1]], [[False, False], [False, False], [True, True]], [I, I, S],
                  [batch([[1, 1], [1, 3], ["ABC", "DEF"]], False, False), batch([[], [], []], False, False),
                   batch([[1], [1], ["Hello"]], True, True)], ordered=True))
eqA = P.func("eq", [P.col(0), P.const(S, "A")], [S, S], fid=1)
cases.append(case("filter.string_pred", Fi + ":183-214", [P.filter_op(eqA, [0, 1, 2])], [S, I, I],
                  [[["A", "B", "A", "D"], [1, 3, 6, 9], [2, 4, 7, 10]], [["C", "B", "A"], [1, 4, 6], [2, 5, 7]]],
                  [[False, False], [True, True]], [S, I, I],
                  [batch([["A", "A"], [1, 6], [2, 7]], False, False), batch([["A"], [6], [7]], True, True)], ordered=True))

M = "src/carnot/exec/map_node_test.cc"
add01 = P.func("add", [P.col(0), P.col(1)], [I, I])
cases.append(case("map.basic", M + ":77-100", [P.map_op([add01], ["col1"])], [I, I],
                  [[[1, 2, 3, 4], [1, 3, 6, 9]], [[1, 2, 3], [1, 4, 6]]], [[False, False], [True, True]], [I],
                  [batch([[2, 5, 9, 13]], False, False), batch([[2, 6, 9]], True, True)], ordered=True))
cases.append(case("map.zero_row_row_batch", M + ":102-132", [P.map_op([add01], ["col1"])], [I, I],
                  [[[1, 2, 3, 4], [1, 3, 6, 9]], [[], []], [[1, 2, 3], [1, 4, 6]]],
                  [[False, False], [True, True], [False, False]], [I],
                  [batch([[2, 5, 9, 13]], False, False), batch([[]], True, True), batch([[2, 6, 9]], False, False)],
                  ordered=True))

# ExecGraphExecuteTest over kLinearPlanFragment (exec_graph_test.cc:132-199, test_proto.h:725-834).
lin = [P.map_op([P.func("add", [P.col(0), P.col(2)], [I, F])], ["summed"]),
       P.map_op([P.func("multiply", [P.col(0), P.const(I, 2)], [F, I], fid=1)], ["mult"])]
cases.append(case("exec_graph.linear_plan_fragment", "src/carnot/exec/exec_graph_test.cc:132-199", lin, [I, B, F],
                  [[[1, 2, 3], [True, False, True], [1.4, 6.2, 10.2]], [[4, 5], [False, False], [3.4, 1.2]]], None, [F],
                  [batch([[4.8, 16.4, 26.4]], False, False), batch([[14.8, 12.4]], True, True)], ordered=True))

# CarnotTest over BigTestTable (carnot_test.cc:321-442, exec/test_utils.h:250-258).
C_ = "src/carnot/carnot_test.cc"
col1 = [1, 2, 3, 5, 6, 8, 9, 11]
col2 = [0.5, 1.2, 5.3, 0.1, 5.1, 5.2, 0.1, 7.3]
col3 = [6, 2, 12, 5, 60, 56, 12, 13]
grp = [1, 1, 3, 1, 2, 2, 3, 2]
sgr = ["sum", "mean", "sum", "mean", "sum", "mean", "sum", "mean"]
split = [(0, 3), (3, 5), (5, 8)]
big = [[col1[a:b], col2[a:b], col3[a:b], grp[a:b], sgr[a:b]] for a, b in split]
s2 = 0.0
for v in col2:
    s2 += v
gbn = [P.agg_op([], [P.agg_expr("mean", [P.col(1)], [F]), P.agg_expr("count", [P.col(2)], [I], fid=1),
                     P.agg_expr("min", [P.col(1)], [F], fid=2), P.agg_expr("max", [P.col(2)], [I], fid=3),
                     P.agg_expr("sum", [P.col(2)], [I], fid=4), P.agg_expr("sum", [P.col(2)], [I], fid=5)])]
cases.append(case("carnot.group_by_none_agg_test", C_ + ":321-389", gbn, [T, F, I, I, S], big, None, [F, I, F, I, I, I],
                  [batch([[s2 / 8], [8], [0.1], [60], [166], [166]], True, True)]))
cases.append(case("carnot.group_by_test", C_ + ":391-442", [P.agg_op([3, 4], [P.agg_expr("sum", [P.col(2)], [I])])],
                  [T, F, I, I, S], big, None, [I, S, I],
                  [batch([[1, 1, 3, 2, 2], ["sum", "mean", "sum", "sum", "mean"], [6, 7, 24, 60, 69]], True, True)]))

# UDA known answers (math_ops_test.cc:470-637) as no-groups aggregations; merges are the same
# values spread over two input batches (AggNode updates one UDA over every batch).
MO = "src/carnot/funcs/builtins/math_ops_test.cc"
fv = [1.234, 2.442, 1.04, 5.322, 6.333]


def uda_case(name, line, uname, t, batches_vals, expected, out_t, tol=0):
    ops = [P.agg_op([], [P.agg_expr(uname, [P.col(0)], [t])])]
    cases.append(case("uda." + name, MO + ":" + line, ops, [t], [[v] for v in batches_vals], None, [out_t],
                      [batch([[expected]], True, True)], tol_ulp=tol))


mean_exp = 0.0
for v in fv:
    mean_exp += v / len(fv)
uda_case("basic_float64_mean", "470-479", "mean", F, [fv], mean_exp, F, tol=4)
uda_case("basic_bool_mean", "481-496", "mean", B, [[True, True, False, False, False, False]], 2 / 6, F, tol=4)
uda_case("basic_int64_mean", "498-507", "mean", I, [[3, 6, 10, 5, 2]], 5.2, F, tol=4)
uda_case("merge_mean", "509-522", "mean", I, [[3, 6, 10, 5, 2], [1, 4, 5, 2, 8]], 4.6, F, tol=4)
fs = 0.0
for v in fv:
    fs += v
uda_case("basic_float64_sum", "524-532", "sum", F, [fv], fs, F, tol=4)
uda_case("basic_bool_sum", "534-541", "sum", B, [[False, True, True, False, False]], 2, I)
uda_case("basic_int64_sum", "543-550", "sum", I, [[3, 6, 10, 5, 2]], 26, I)
uda_case("merge_sum", "552-564", "sum", I, [[3, 6, 10, 5, 2], [1, 4, 5, 2, 8]], 46, I)
uda_case("basic_int64_max", "566-570", "max", I, [[3, 5, 2, 7, 1]], 7, I)
uda_case("merge_max", "572-582", "max", I, [[3, 6, 10, 5, 2], [1, 4, 5, 2, 11]], 11, I)
uda_case("basic_int64_min", "584-588", "min", I, [[3, 5, 2, 7, 1]], 1, I)
uda_case("basic_float64_min", "590-598", "min", F, [[-4.64, -4.64123445435, 2.252242424, 1.1, -1.1234566]], -4.64123445435, F)
uda_case("merge_min", "600-610", "min", I, [[3, 6, 10, 5, 2], [1, 4, 5, 2, 11]], 1, I)
uda_case("basic_int64_count", "612-615", "count", I, [[5, 2, 7, 1]], 4, I)
uda_case("merge_count", "617-626", "count", I, [[3, 6, 10, 5, 2], [1, 4, 5, 2]], 9, I)
uda_case("partial_count", "631-634", "count", I, [[3, 6, 10, 5, 2]], 5, I)

# EquijoinNode known answers (equijoin_node_test.cc).  Left table "l" is parent 0, right table
# "r" is parent 1.  The output is independent of how the two inputs interleave (probe batches
# wait for build eos), so each table is simply a batch list.  "unordered_tail": the last N
# expected batches are compared as one multiset (ExpectRowBatchesData, emitted from a hash map).
J = "src/carnot/exec/equijoin_node_test.cc"
join_cases = []


def join_case(name, line, jtype, conds, outs, names, lt, lb, rt, rb, out_types, expected, tail=0):
    plan = P.dag_plan([
        (1, P.source_op("l", lt, [f"l{i}" for i in range(len(lt))], list(range(len(lt)))), []),
        (2, P.source_op("r", rt, [f"r{i}" for i in range(len(rt))], list(range(len(rt)))), []),
        (3, P.join_op(jtype, conds, outs, names=names, rows_per_batch=5), [1, 2]),
        (4, P.sink_op("out"), [3]),
    ])
    join_cases.append({
        "name": "join." + name, "source": J + ":" + line, "plan": text_format.MessageToString(plan),
        "tables": {"l": {"types": lt, "batches": lb}, "r": {"types": rt, "batches": rb}},
        "output": {"types": out_types, "batches": expected}, "ordered": True, "tol_ulp": 0,
        "unordered_tail": tail,
    })


join_case("ordered_inner_join", "73-152", P.JOIN_INNER, [(0, 1)], [(0, 1), (1, 1), (1, 0)],
          ["left_1", "right_1", "time_"],
          [I, F], [[[1, 2, 2], [1.0, 2.0, 2.1]], [[9, 1, 1], [9.0, 1.1, 1.2]]],
          [T, I], [[[10, 20, 30, 31], [1, 2, 3, 3]], [[101, 150, 190], [1, 5, 9]]],
          [F, I, T],
          [batch([[1.0, 1.1, 1.2, 2.0, 2.1], [1, 1, 1, 2, 2], [10, 10, 10, 20, 20]], False, False),
           batch([[1.0, 1.1, 1.2, 9.0], [1, 1, 1, 9], [101, 101, 101, 190]], True, True)])
join_case("ordered_left_join", "154-239", P.JOIN_LEFT_OUTER, [(1, 0)], [(1, 1), (0, 1), (0, 0)],
          ["right_1", "left_1", "time_"],
          [T, I], [[[10, 20, 30, 31], [1, 2, 3, 3]], [[101, 150, 190], [1, 5, 9]]],
          [I, F], [[[1, 2, 2], [1.0, 2.0, 2.1]], [[9, 1, 1, 8], [9.0, 1.1, 1.2, 8.0]]],
          [F, I, T],
          [batch([[1.0, 1.1, 1.2, 2.0, 2.1], [1, 1, 1, 2, 2], [10, 10, 10, 20, 20]], False, False),
           batch([[0.0, 0.0, 1.0, 1.1, 1.2], [3, 3, 1, 1, 1], [30, 31, 101, 101, 101]], False, False),
           batch([[0.0, 9.0], [5, 9], [150, 190]], True, True)])
fo_l = [[[101, 200, 101, 200, 101], [1, 2, 3, 4, 5]], [[200, 200, 200, 300, 300], [6, 8, 10, 12, 14]],
        [[400, 500], [16, 18]]]
fo_r = [[[-10, -20, -30], [110, 120, 101]]]
unmatched = [2, 4, 6, 8, 10, 12, 14, 16, 18]
join_case("unordered_full_outer_join", "241-321", P.JOIN_FULL_OUTER, [(0, 1)], [(0, 1), (1, 1), (1, 0)],
          ["left_1", "right_1", "right_0"], [T, I], fo_l, [I, T], fo_r, [I, T, I],
          [batch([[0, 0, 1, 3, 5], [110, 120, 101, 101, 101], [-10, -20, -30, -30, -30]], False, False),
           batch([unmatched[:5], [0] * 5, [0] * 5], False, False),
           batch([unmatched[5:], [0] * 4, [0] * 4], True, True)], tail=2)
join_case("unordered_no_left_columns", "323-395", P.JOIN_FULL_OUTER, [(0, 1)], [(1, 1), (1, 0)],
          ["right_1", "right_0"], [T, I], fo_l, [I, T], fo_r, [T, I],
          [batch([[110, 120, 101, 101, 101], [-10, -20, -30, -30, -30]], False, False),
           batch([[0] * 5, [0] * 5], False, False),
           batch([[0] * 4, [0] * 4], True, True)], tail=2)
join_case("unordered_no_right_columns", "397-462", P.JOIN_FULL_OUTER, [(0, 1)], [(0, 1)],
          ["left_1"], [T, I], fo_l, [I, T], fo_r, [I],
          [batch([[0, 0, 1, 3, 5]], False, False), batch([unmatched[:5]], False, False),
           batch([unmatched[5:]], True, True)], tail=2)
nm_l = [[[101, 102, 101, 103, 101], [1, 2, 3, 4, 5]]]
join_case("unordered_no_matches", "464-526", P.JOIN_INNER, [(0, 1)], [(0, 1), (1, 1), (1, 0)],
          ["left_1", "right_1", "right_0"], [T, I], nm_l, [I, T], [[[-10, -20, -30], [200, 300, 400]]],
          [I, T, I], [batch([[], [], []], True, True)])
join_case("zero_row_row_batch_right", "528-590", P.JOIN_INNER, [(0, 1)], [(0, 1), (1, 1), (1, 0)],
          ["left_1", "right_1", "right_0"], [T, I], nm_l, [I, T], [[[], []]],
          [I, T, I], [batch([[], [], []], True, True)])
join_case("unordered_many_matches", "592-687", P.JOIN_INNER, [(0, 1)], [(0, 1), (1, 1), (1, 0)],
          ["left_1", "time_", "right_0"],
          [T, I], [[[101, 102, 103, 101, 102], [1, 2, 3, 4, 5]], [[103, 101, 104], [6, 7, 8]]],
          [I, T], [[[10, 20, 30, 40], [101, 101, 102, 102]], [[50, 60, 70, 80, 90], [103, 103, 103, 103, 105]]],
          [I, T, I],
          [batch([[1, 4, 7, 1, 4], [101] * 5, [10, 10, 10, 20, 20]], False, False),
           batch([[7, 2, 5, 2, 5], [101, 102, 102, 102, 102], [20, 30, 30, 40, 40]], False, False),
           batch([[3, 6, 3, 6, 3], [103] * 5, [50, 50, 60, 60, 70]], False, False),
           batch([[6, 3, 6], [103] * 3, [70, 80, 80]], True, True)])

# LimitNode (limit_node_test.cc, kLimitOperator1 / kLimitDropOperator1 = limit 10 over columns
# {0, 1} / {0, 2}, test_proto.h:315-337).  ExecNodeTester feeds every batch with explicit flags.
L = "src/carnot/exec/limit_node_test.cc"
limit_cases = []
c12 = [[1, 2, 3, 4, 5, 6, 1, 2, 3, 4, 5, 6], [1, 3, 6, 9, 12, 15, 1, 3, 6, 9, 12, 15]]
lim = lambda n=10, cols=(0, 1): [P.limit_op(n, list(cols))]  # noqa: E731
limit_cases.append(case("limit.single_batch", L + ":66-83", lim(), [I, I], [c12], [[True, True]], [I, I],
                        [batch([c12[0][:10], c12[1][:10]], True, True)], ordered=True))
limit_cases.append(case("limit.single_empty_batch", L + ":85-101", lim(), [I, I], [[[], []]], [[True, True]], [I, I],
                        [batch([[], []], True, True)], ordered=True))
limit_cases.append(case("limit.limit_zero", L + ":103-123", lim(0), [I, I], [c12], [[False, False]], [I, I],
                        [batch([[], []], True, True)], ordered=True))
limit_cases.append(case("limit.single_batch_exact_boundary", L + ":125-141", lim(), [I, I], [[c12[0][:10], c12[1][:10]]],
                        [[False, False]], [I, I], [batch([c12[0][:10], c12[1][:10]], True, True)], ordered=True))
limit_cases.append(case("limit.limits_records_split", L + ":143-170", lim(), [I, I],
                        [[[1, 2, 3, 4, 5, 6], [1, 3, 6, 9, 12, 15]], [[1, 2, 3, 4, 5, 6], [1, 4, 6, 8, 10, 12]]],
                        [[False, False], [True, True]], [I, I],
                        [batch([[1, 2, 3, 4, 5, 6], [1, 3, 6, 9, 12, 15]], False, False),
                         batch([[1, 2, 3, 4], [1, 4, 6, 8]], True, True)], ordered=True))
limit_cases.append(case("limit.limits_exact_boundary", L + ":172-200", lim(), [I, I],
                        [[[1, 2, 3, 4, 5, 6], [1, 3, 6, 9, 12, 15]], [[1, 2, 3, 4], [1, 4, 6, 8]]],
                        [[False, False], [True, True]], [I, I],
                        [batch([[1, 2, 3, 4, 5, 6], [1, 3, 6, 9, 12, 15]], False, False),
                         batch([[1, 2, 3, 4], [1, 4, 6, 8]], True, True)], ordered=True))
c3 = c12 + [[1, 4, 8, 12, 16, 20, 1, 4, 8, 12, 16, 20]]
limit_cases.append(case("limit.drop_input_columns", L + ":216-237", lim(10, (0, 2)), [I, I, I], [c3], [[True, True]], [I, I],
                        [batch([c3[0][:10], c3[2][:10]], True, True)], ordered=True))
limit_cases.append(case("limit.drop_input_columns_fewer_than_limit", L + ":239-260", lim(10, (0, 2)), [I, I, I],
                        [[c[:8] for c in c3]], [[True, True]], [I, I], [batch([c3[0][:8], c3[2][:8]], True, True)],
                        ordered=True))

doc = {
    "generator": "tests/golden/make_golden.py",
    "cases": cases,
    "limit_cases": limit_cases,
    "join_cases": join_cases,
    # QuantilesUDA known answers (math_sketches_test.cc:30-70); EXPECT_DOUBLE_EQ = 4 ULP.
    "quantiles": [
        {"source": "src/carnot/funcs/builtins/math_sketches_test.cc:30-48", "input": fv,
         "expected": {"p01": 1.04, "p10": 1.04, "p50": 2.442, "p90": 6.333, "p99": 6.333}},
        {"source": "src/carnot/funcs/builtins/math_sketches_test.cc:50-70", "input": [1, 2, 2, 1, 1, 5, 6],
         "expected": {"p01": 1, "p10": 1, "p50": 2, "p90": 5.7999999999999998, "p99": 6}},
    ],
}
with open(OUT, "w") as f:
    json.dump(doc, f, indent=1)
print(f"wrote {len(cases)} cases and {len(join_cases)} join cases to {OUT}")
