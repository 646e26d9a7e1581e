"""Builders for planpb plans: expression helpers and the BASELINE.json queries.

The query shapes are what the PxL compiler emits for the north-star scripts
(src/carnot/planner/compiler/compiler_test.cc:1265-1447 shows the compiled shape:
MemorySource -> Map/Filter -> Agg -> ... -> sink).  Operator-name mapping of PxL infix
operators follows src/carnot/planner/ir/func_ir.cc:27-48 (>= -> greaterThanEqual, / -> divide).
"""
from __future__ import annotations

from typing import List, Sequence

from . import planpb
from ._lib import BOOLEAN, FLOAT64, INT64, STRING, TIME64NS, UINT128
from .device import HTTP_EVENTS_SCHEMA


def col(index: int, node: int = 0):
    e = planpb.ScalarExpression()
    e.column.node = node
    e.column.index = index
    return e


def const(dtype: int, value):
    e = planpb.ScalarExpression()
    c = e.constant
    c.data_type = dtype
    if dtype == INT64:
        c.int64_value = int(value)
    elif dtype == FLOAT64:
        c.float64_value = float(value)
    elif dtype == STRING:
        c.string_value = value
    elif dtype == BOOLEAN:
        c.bool_value = bool(value)
    elif dtype == TIME64NS:
        c.time64_ns_value = int(value)
    elif dtype == UINT128:
        c.uint128_value.low = int(value) & (2**64 - 1)
        c.uint128_value.high = int(value) >> 64
    return e


def func(name: str, args: Sequence, arg_types: Sequence[int] = (), fid: int = 0):
    e = planpb.ScalarExpression()
    f = e.func
    f.name = name
    f.id = fid
    for a in args:
        f.args.add().CopyFrom(a)
    f.args_data_types.extend(arg_types)
    return e


def agg_expr(name: str, args: Sequence, arg_types: Sequence[int] = (), fid: int = 0, init_args: Sequence = ()):
    op = planpb.AggregateOperator()
    v = op.values.add()
    v.name = name
    v.id = fid
    for a in args:
        arg = v.args.add()
        if a.WhichOneof("value") == "column":
            arg.column.CopyFrom(a.column)
        else:
            arg.constant.CopyFrom(a.constant)
    v.args_data_types.extend(arg_types)
    for ia in init_args:
        v.init_args.add().CopyFrom(ia.constant)
    return v


def filter_op(expr, columns: Sequence[int], node: int = 0):
    op = planpb.Operator()
    op.op_type = planpb.Operator.DESCRIPTOR.fields_by_name["op_type"].enum_type.values_by_name["FILTER_OPERATOR"].number
    op.filter_op.expression.CopyFrom(expr)
    for c in columns:
        cc = op.filter_op.columns.add()
        cc.node = node
        cc.index = c
    return op


def map_op(exprs: Sequence, names: Sequence[str]):
    op = planpb.Operator()
    op.op_type = 2000
    for e in exprs:
        op.map_op.expressions.add().CopyFrom(e)
    op.map_op.column_names.extend(names)
    return op


def agg_op(groups: Sequence[int], values: Sequence, group_names: Sequence[str] = (), value_names: Sequence[str] = (),
           windowed: bool = False, node: int = 0, partial_agg: bool = False, finalize_results: bool = False):
    op = planpb.Operator()
    op.op_type = 2100
    for g in groups:
        c = op.agg_op.groups.add()
        c.node = node
        c.index = g
    for v in values:
        op.agg_op.values.add().CopyFrom(v)
    op.agg_op.group_names.extend(group_names or [f"g{i}" for i in range(len(groups))])
    op.agg_op.value_names.extend(value_names or [f"v{i}" for i in range(len(values))])
    op.agg_op.windowed = windowed
    op.agg_op.partial_agg = partial_agg
    op.agg_op.finalize_results = finalize_results
    return op


def source_op(name: str, types: Sequence[int], names: Sequence[str], idxs: Sequence[int],
              start_time: int = None, stop_time: int = None, streaming: bool = False):
    op = planpb.Operator()
    op.op_type = 1000
    m = op.mem_source_op
    m.name = name
    m.column_idxs.extend(idxs)
    m.column_types.extend([types[i] for i in idxs])
    m.column_names.extend([names[i] for i in idxs])
    if start_time is not None:
        m.start_time.value = start_time
    if stop_time is not None:
        m.stop_time.value = stop_time
    if streaming:
        m.streaming = True
    return op


def limit_op(limit: int, columns: Sequence[int], abortable_srcs: Sequence[int] = (), node: int = 0):
    """LimitOperator (plan.proto:269-276), as the PxL compiler inserts one before every result
    sink (add_limit_to_batch_result_sink_rule.cc:40-68)."""
    op = planpb.Operator()
    op.op_type = 2300
    op.limit_op.limit = limit
    for c in columns:
        cc = op.limit_op.columns.add()
        cc.node = node
        cc.index = c
    op.limit_op.abortable_srcs.extend(abortable_srcs)
    return op


def sink_op(name: str, types: Sequence[int] = (), names: Sequence[str] = ()):
    op = planpb.Operator()
    op.op_type = 9000
    op.mem_sink_op.name = name
    op.mem_sink_op.column_types.extend(types)
    op.mem_sink_op.column_names.extend(names)
    return op


JOIN_INNER, JOIN_LEFT_OUTER, JOIN_FULL_OUTER = 0, 1, 3


def join_op(join_type: int, conditions: Sequence, outputs: Sequence, names: Sequence[str] = (), rows_per_batch: int = 0):
    """JoinOperator (plan.proto:301-338): conditions = [(left_col, right_col)], outputs =
    [(parent_index, column_index)] with parent 0 = left, 1 = right."""
    op = planpb.Operator()
    op.op_type = 2500
    j = op.join_op
    j.type = join_type
    for lc, rc in conditions:
        c = j.equality_conditions.add()
        c.left_column_index = lc
        c.right_column_index = rc
    for pi, ci in outputs:
        o = j.output_columns.add()
        o.parent_index = pi
        o.column_index = ci
    j.column_names.extend(names or [f"c{i}" for i in range(len(outputs))])
    j.rows_per_batch = rows_per_batch
    return op


def dag_plan(nodes: Sequence) -> "planpb.Plan":
    """One fragment from [(id, op, [parent ids])] in topological order."""
    plan = planpb.Plan()
    frag = plan.nodes.add()
    frag.id = 1
    children = {nid: [] for nid, _, _ in nodes}
    for nid, _, parents in nodes:
        for p in parents:
            children[p].append(nid)
    for nid, op, parents in nodes:
        dn = frag.dag.nodes.add()
        dn.id = nid
        dn.sorted_parents.extend(parents)
        dn.sorted_children.extend(children[nid])
        pn = frag.nodes.add()
        pn.id = nid
        pn.op.CopyFrom(op)
    plan.dag.nodes.add().id = 1
    return plan


def linear_plan(ops: List) -> "planpb.Plan":
    """One fragment, nodes 1..n chained in order (exec_graph.cc topological execution)."""
    plan = planpb.Plan()
    frag = plan.nodes.add()
    frag.id = 1
    for i, op in enumerate(ops):
        nid = i + 1
        dn = frag.dag.nodes.add()
        dn.id = nid
        if i > 0:
            dn.sorted_parents.append(nid - 1)
        if i + 1 < len(ops):
            dn.sorted_children.append(nid + 1)
        pn = frag.nodes.add()
        pn.id = nid
        pn.op.CopyFrom(op)
    pdn = plan.dag.nodes.add()
    pdn.id = 1
    return plan


HTTP_TYPES = [t for _, t in HTTP_EVENTS_SCHEMA]
HTTP_NAMES = [n for n, _ in HTTP_EVENTS_SCHEMA]
HE = {n: i for i, n in enumerate(HTTP_NAMES)}


def c1_plan(table: str = "http_events"):
    """groupby('service').agg(count=('latency', px.count), mean=('latency', px.mean))."""
    src = source_op(table, HTTP_TYPES, HTTP_NAMES, [HE["service"], HE["latency"]])
    agg = agg_op([0], [agg_expr("count", [col(1)], [INT64]), agg_expr("mean", [col(1)], [INT64], fid=1)],
                 ["service"], ["count", "mean"])
    return linear_plan([src, agg, sink_op("output")])


def c2_plan(table: str = "http_events", with_pluck: bool = True):
    """Filter(resp_status >= 400) -> Map(service, req_path, latency_ms = latency / 1e6)
    -> Agg by (service, req_path): count, mean, quantiles -> Map(pluck p50, p99)."""
    src = source_op(table, HTTP_TYPES, HTTP_NAMES,
                    [HE["service"], HE["req_path"], HE["resp_status"], HE["latency"]])
    flt = filter_op(func("greaterThanEqual", [col(2), const(INT64, 400)], [INT64, INT64]), [0, 1, 2, 3])
    mp = map_op([col(0), col(1), func("divide", [col(3), const(FLOAT64, 1e6)], [INT64, FLOAT64], fid=1)],
                ["service", "req_path", "latency_ms"])
    agg = agg_op([0, 1], [agg_expr("count", [col(2)], [FLOAT64], fid=2),
                          agg_expr("mean", [col(2)], [FLOAT64], fid=3),
                          agg_expr("quantiles", [col(2)], [FLOAT64], fid=4)],
                 ["service", "req_path"], ["count", "mean", "latency_quantiles"])
    ops = [src, flt, mp, agg]
    if with_pluck:
        pl = map_op([col(0), col(1), col(2), col(3),
                     func("pluck_float64", [col(4), const(STRING, "p50")], [STRING, STRING], fid=5),
                     func("pluck_float64", [col(4), const(STRING, "p99")], [STRING, STRING], fid=6)],
                    ["service", "req_path", "count", "mean", "p50", "p99"])
        ops.append(pl)
    ops.append(sink_op("output"))
    return linear_plan(ops)


def compiled_c2_plan(table: str = "http_events", limit: int = 10000):
    """C2 in the shape the PxL compiler emits (compiler_test.cc:1265-1447): the aggregate followed
    by an arithmetic Map (mean in seconds, error count + 1, p99 - p50 from the plucked
    quantiles) and the Limit the compiler puts before the result sink (abortable: the source)."""
    src = source_op(table, HTTP_TYPES, HTTP_NAMES,
                    [HE["service"], HE["req_path"], HE["resp_status"], HE["latency"]])
    flt = filter_op(func("greaterThanEqual", [col(2), const(INT64, 400)], [INT64, INT64]), [0, 1, 2, 3])
    mp = map_op([col(0), col(1), func("divide", [col(3), const(FLOAT64, 1e6)], [INT64, FLOAT64], fid=1)],
                ["service", "req_path", "latency_ms"])
    agg = agg_op([0, 1], [agg_expr("count", [col(2)], [FLOAT64], fid=2),
                          agg_expr("mean", [col(2)], [FLOAT64], fid=3),
                          agg_expr("quantiles", [col(2)], [FLOAT64], fid=4)],
                 ["service", "req_path"], ["count", "mean", "latency_quantiles"])
    p50 = func("pluck_float64", [col(4), const(STRING, "p50")], [STRING, STRING], fid=5)
    p99 = func("pluck_float64", [col(4), const(STRING, "p99")], [STRING, STRING], fid=6)
    post = map_op([col(0), col(1), func("add", [col(2), const(INT64, 1)], [INT64, INT64], fid=7),
                   func("divide", [col(3), const(FLOAT64, 1000.0)], [FLOAT64, FLOAT64], fid=8),
                   func("subtract", [p99, p50], [FLOAT64, FLOAT64], fid=9), p50,
                   func("greaterThan", [func("multiply", [p50, const(FLOAT64, 2.0)], [FLOAT64, FLOAT64], fid=10), col(3)],
                        [FLOAT64, FLOAT64], fid=11),
                   col(4)],
                  ["service", "req_path", "errors_plus_one", "mean_s", "p99_minus_p50", "p50", "skewed", "latency_quantiles"])
    lim = limit_op(limit, list(range(8)), abortable_srcs=[1])
    return linear_plan([src, flt, mp, agg, post, lim, sink_op("output")])


def c3_plan(table: str = "http_events"):
    """Same filter, group by (pod, remote_addr): count, mean(latency), sum(resp_body_size)."""
    src = source_op(table, HTTP_TYPES, HTTP_NAMES,
                    [HE["pod"], HE["remote_addr"], HE["resp_status"], HE["latency"], HE["resp_body_size"]])
    flt = filter_op(func("greaterThanEqual", [col(2), const(INT64, 400)], [INT64, INT64]), [0, 1, 3, 4])
    agg = agg_op([0, 1], [agg_expr("count", [col(2)], [INT64]), agg_expr("mean", [col(2)], [INT64], fid=1),
                          agg_expr("sum", [col(3)], [INT64], fid=2)],
                 ["pod", "remote_addr"], ["count", "mean_latency", "sum_resp_body"])
    return linear_plan([src, flt, agg, sink_op("output")])


def c3_full_plan(table: str = "http_events"):
    """BASELINE configs[2] at its full cardinality: no filter, every row aggregated by
    (pod, remote_addr) -- all 10M distinct pairs of the table -- count, mean(latency),
    sum(resp_body_size)."""
    src = source_op(table, HTTP_TYPES, HTTP_NAMES, [HE["pod"], HE["remote_addr"], HE["latency"], HE["resp_body_size"]])
    agg = agg_op([0, 1], [agg_expr("count", [col(2)], [INT64]), agg_expr("mean", [col(2)], [INT64], fid=1),
                          agg_expr("sum", [col(3)], [INT64], fid=2)],
                 ["pod", "remote_addr"], ["count", "mean_latency", "sum_resp_body"])
    return linear_plan([src, agg, sink_op("output")])


# conn_stats subset and a pod metadata table for C5 ("C5 (next)").
CONN_STATS_SCHEMA = [("time_", TIME64NS), ("upid", UINT128), ("remote_addr", STRING), ("remote_port", INT64),
                     ("bytes_sent", INT64), ("bytes_recv", INT64)]
CONN_TYPES = [t for _, t in CONN_STATS_SCHEMA]
CONN_NAMES = [n for n, _ in CONN_STATS_SCHEMA]
POD_META_SCHEMA = [("upid", UINT128), ("pod", STRING), ("namespace", STRING)]
POD_TYPES = [t for _, t in POD_META_SCHEMA]
POD_NAMES = [n for n, _ in POD_META_SCHEMA]
C5_WINDOW_NS = 10 * 1000 * 1000 * 1000


def c5_plan(conn: str = "conn_stats", pods: str = "pod_metadata", window_ns: int = C5_WINDOW_NS):
    """df.time_ = px.bin(df.time_, 10s); groupby(time_, upid, remote_addr).agg(bytes_sent=sum,
    bytes_recv=sum); merge with pod metadata on upid (inner).  The output's time_ comes from the
    left (aggregate) side, so the aggregate is the probe table (equijoin_node.cc:63-69)."""
    c = {n: i for i, n in enumerate(CONN_NAMES)}
    src = source_op(conn, CONN_TYPES, CONN_NAMES,
                    [c["time_"], c["upid"], c["remote_addr"], c["bytes_sent"], c["bytes_recv"]])
    mp = map_op([func("bin", [col(0), const(INT64, window_ns)], [TIME64NS, INT64]), col(1), col(2), col(3), col(4)],
                ["time_", "upid", "remote_addr", "bytes_sent", "bytes_recv"])
    agg = agg_op([0, 1, 2], [agg_expr("sum", [col(3)], [INT64], fid=1), agg_expr("sum", [col(4)], [INT64], fid=2)],
                 ["time_", "upid", "remote_addr"], ["bytes_sent", "bytes_recv"])
    psrc = source_op(pods, POD_TYPES, POD_NAMES, [0, 1, 2])
    join = join_op(JOIN_INNER, [(1, 0)], [(0, 0), (1, 1), (1, 2), (0, 2), (0, 3), (0, 4)],
                   names=["time_", "pod", "namespace", "remote_addr", "bytes_sent", "bytes_recv"])
    return dag_plan([(1, src, []), (2, mp, [1]), (3, agg, [2]), (4, psrc, []), (5, join, [3, 4]),
                     (6, sink_op("output"), [5])])


# Split aggregation: the PEM-side partial agg and the Kelvin-side
# finalize agg the distributed splitter makes of one blocking agg
# (partial_op_mgr.cc:47-83: CreatePrepareOperator sets partial_agg, CreateMergeOperator keeps
# the pre-split values and sets finalize_results; the partial output relation is the groups +
# serialized_expressions, operators.cc:251-257).
SPLIT_SRC_COLS = ["pod", "remote_addr", "resp_status", "latency", "resp_body_size"]


def split_values():
    """Every splittable UDA signature on the path: count, mean/sum/min/max over INT64 columns and
    over a FLOAT64 map result.  Input columns (after the map): 0 pod, 1 remote_addr, 2 latency,
    3 resp_body_size, 4 latency_ms."""
    return [agg_expr("count", [col(2)], [INT64]), agg_expr("mean", [col(2)], [INT64], fid=1),
            agg_expr("sum", [col(3)], [INT64], fid=2), agg_expr("min", [col(2)], [INT64], fid=3),
            agg_expr("max", [col(2)], [INT64], fid=4), agg_expr("mean", [col(4)], [FLOAT64], fid=5),
            agg_expr("sum", [col(4)], [FLOAT64], fid=6), agg_expr("min", [col(4)], [FLOAT64], fid=7),
            agg_expr("max", [col(4)], [FLOAT64], fid=8)]


def split_source_plan(table: str = "http_events", groups: Sequence[int] = (0, 1), values=None,
                      partial_agg: bool = True, finalize_results: bool = False, sink: str = "partial"):
    """Filter(resp_status >= 400) -> Map(+ latency_ms) -> Agg(groups, values) with the given
    split flags (True/False: the PEM half; False/False or True/True: a full aggregate)."""
    values = split_values() if values is None else values
    src = source_op(table, HTTP_TYPES, HTTP_NAMES, [HE[n] for n in SPLIT_SRC_COLS])
    flt = filter_op(func("greaterThanEqual", [col(2), const(INT64, 400)], [INT64, INT64]), [0, 1, 3, 4])
    mp = map_op([col(0), col(1), col(2), col(3), func("divide", [col(2), const(FLOAT64, 1e6)], [INT64, FLOAT64])],
                ["pod", "remote_addr", "latency", "resp_body_size", "latency_ms"])
    agg = agg_op(list(groups), values, [SPLIT_SRC_COLS[g] for g in groups], [f"v{i}" for i in range(len(values))],
                 partial_agg=partial_agg, finalize_results=finalize_results)
    return linear_plan([src, flt, mp, agg, sink_op(sink)])


def split_merge_plan(partials: str, group_types: Sequence[int], values=None, sink: str = "output"):
    """The finalize half: MemorySource over the partial outputs (groups + serialized_expressions)
    -> Agg(partial_agg=False, finalize_results=True) with the pre-split values."""
    values = split_values() if values is None else values
    ng = len(group_types)
    types = list(group_types) + [STRING]
    names = [f"g{i}" for i in range(ng)] + ["serialized_expressions"]
    src = source_op(partials, types, names, list(range(ng + 1)))
    agg = agg_op(list(range(ng)), values, names[:ng], [f"v{i}" for i in range(len(values))],
                 partial_agg=False, finalize_results=True)
    return linear_plan([src, agg, sink_op(sink)])


def grpc_sink_op(grpc_source_id: int, address: str = "kelvin:59300"):
    """GRPCSinkOperator to another Carnot's GRPCSource (plan.proto:190-216)."""
    op = planpb.Operator()
    op.op_type = 9100
    op.grpc_sink_op.address = address
    op.grpc_sink_op.grpc_source_id = grpc_source_id
    return op


def grpc_source_op(types: Sequence[int], names: Sequence[str]):
    """GRPCSourceOperator (plan.proto:182-187)."""
    op = planpb.Operator()
    op.op_type = 1100
    op.grpc_source_op.column_types.extend(types)
    op.grpc_source_op.column_names.extend(names)
    return op


def union_op(names: Sequence[str], mappings: Sequence[Sequence[int]], rows_per_batch: int = 0):
    """UnionOperator (plan.proto:283-295)."""
    op = planpb.Operator()
    op.op_type = 2400
    op.union_op.column_names.extend(names)
    if rows_per_batch:
        op.union_op.rows_per_batch = rows_per_batch
    for m in mappings:
        op.union_op.column_mappings.add().column_indexes.extend(m)
    return op


def split_pem_fragment(dest_id: int, table: str = "http_events", groups: Sequence[int] = (0, 1), values=None):
    """The PEM fragment of a split C3-style aggregate: ... -> Agg(partial) -> GRPCSink(dest)."""
    plan = split_source_plan(table, groups, values)
    frag = plan.nodes[0]
    sink = [n for n in frag.nodes if n.op.WhichOneof("op") == "mem_sink_op"][0]
    sink.op.CopyFrom(grpc_sink_op(dest_id))
    return plan


def split_kelvin_fragment(source_ids: Sequence[int], group_types: Sequence[int], values=None, sink: str = "output"):
    """The Kelvin fragment: one GRPCSource per PEM -> Union -> Agg(finalize) -> sink."""
    values = split_values() if values is None else values
    ng = len(group_types)
    types = list(group_types) + [STRING]
    names = [f"g{i}" for i in range(ng)] + ["serialized_expressions"]
    nodes = [(sid, grpc_source_op(types, names), []) for sid in source_ids]
    un = union_op(names, [list(range(ng + 1))] * len(source_ids))
    agg = agg_op(list(range(ng)), values, names[:ng], [f"v{i}" for i in range(len(values))],
                 partial_agg=False, finalize_results=True)
    base = max(source_ids) + 1
    nodes += [(base, un, list(source_ids)), (base + 1, agg, [base]), (base + 2, sink_op(sink), [base + 1])]
    return dag_plan(nodes)
