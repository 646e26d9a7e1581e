"""Lower a linear planpb fragment onto the device operators.

MemorySource -> (Filter | Map)* -> Agg(blocking) [-> Map] -> Sink becomes ONE pxg_agg whose
filter program is the conjunction of the filters and whose key / UDA-argument programs are
the Map expressions substituted into the Agg's column references.  This is the graph-level
fusion SURVEY.md §7 recommends at the operator switch (src/carnot/exec/exec_graph.cc:66-80):
a blocking agg only emits at eos (src/carnot/exec/agg_node.cc:169-171), so the intermediate
Filter/Map batches are not observable.  Plans without an Agg run as pxg_filter / pxg_map.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import BOOLEAN, FLOAT64, INT64, OP, STRING
from .compile import ExprCompiler, Prog, UnsupportedError, compile_uda
from .device import Agg, Column, Ctx, Table

QUANTILE_KEYS = ["p01", "p10", "p25", "p50", "p75", "p90", "p99"]


def quantiles_json_column(q7: np.ndarray) -> Column:
    """QuantilesUDA::Finalize strings (src/carnot/funcs/builtins/math_sketches.h:40-54) of G
    groups of 7 doubles, rendered by the engine's rapidjson restatement (pxc_quantiles_json,
    pixie_amd/host/json_double.h) so the Python lowering and the C++ engine emit the same bytes."""
    import ctypes as C
    from . import host_engine
    lib = host_engine.load()
    q = np.ascontiguousarray(np.asarray(q7, dtype=np.float64).reshape(-1, 7))
    out = C.c_void_p()
    n = C.c_int64()
    code = lib.pxc_quantiles_json(q.ctypes.data_as(C.POINTER(C.c_double)), q.shape[0], C.byref(out), C.byref(n))
    if code != 0:
        raise RuntimeError(f"pxc_quantiles_json failed: {lib.pxc_last_error().decode()}")
    try:
        raw = C.string_at(out.value, n.value)
    finally:
        lib.pxc_free(out)
    strs = raw.split(b"\0")[:q.shape[0]]
    return Column.from_values(STRING, strs)


def quantiles_json(q7: Sequence[float]) -> str:
    """One group's QuantilesUDA::Finalize string."""
    return quantiles_json_column(np.asarray(q7, dtype=np.float64).reshape(1, 7)).to_list()[0]


def _ops(plan):
    frag = plan.nodes[0]
    order = [dn.id for dn in frag.dag.nodes]
    by_id = {pn.id: pn.op for pn in frag.nodes}
    return [by_id[i] for i in order]


class LinearQuery:
    def __init__(self, plan, table_types: Sequence[int], expected_groups: int = 0):
        ops = _ops(plan)
        src = ops[0]
        if src.WhichOneof("op") != "mem_source_op":
            raise UnsupportedError("plan must start with a MemorySource")
        idxs = list(src.mem_source_op.column_idxs) or list(range(len(table_types)))
        self.table_types = list(table_types)
        # env[i] = (insns, type, pool) of the current column i, expressed over table columns
        env: List[Tuple[list, int, bytes]] = [([(OP["COL"], table_types[c], c, 0)], table_types[c], b"") for c in idxs]
        self.filter: Optional[Prog] = None
        self.agg_op = None
        self.post_map = None
        self.sink_name = None
        self.map_only: List = []
        i = 1
        while i < len(ops):
            kind = ops[i].WhichOneof("op")
            if kind == "filter_op":
                comp = ExprCompiler([e[1] for e in env], inline=dict(enumerate(env)))
                pred = comp.compile(ops[i].filter_op.expression)
                if pred.result_type != BOOLEAN:
                    raise ValueError("Predicate expression must be a boolean")
                self.filter = pred if self.filter is None else _and(self.filter, pred)
                env = [env[int(c.index)] for c in ops[i].filter_op.columns]
            elif kind == "map_op":
                comp = ExprCompiler([e[1] for e in env], inline=dict(enumerate(env)))
                new_env = []
                for e in ops[i].map_op.expressions:
                    p = comp.compile(e)
                    new_env.append((p.insns_py, p.result_type, p.pool))
                env = new_env
            elif kind == "agg_op":
                self.agg_op = ops[i].agg_op
                break
            elif kind in ("mem_sink_op", "grpc_sink_op"):
                self.sink_name = ops[i].mem_sink_op.name if kind == "mem_sink_op" else ops[i].grpc_sink_op.output_table.table_name
                break
            else:
                raise UnsupportedError(f"operator {kind} not supported by the device lowering")
            i += 1
        self.env = env
        self.out_types = [e[1] for e in env]
        if self.agg_op is not None:
            a = self.agg_op
            comp = ExprCompiler([e[1] for e in env], inline=dict(enumerate(env)))
            self.keys = [Prog(env[int(g.index)][0], env[int(g.index)][1], env[int(g.index)][2]) for g in a.groups]
            self.udas = [compile_uda(v, comp) for v in a.values]
            self.windowed = a.windowed
            self.expected_groups = expected_groups
            self.out_types = [k.result_type for k in self.keys] + [u.out_type for u in self.udas]
            rest = ops[i + 1:]
            if rest and rest[0].WhichOneof("op") == "map_op":
                self.post_map = rest[0].map_op
                rest = rest[1:]
            if rest:
                r = rest[0]
                k = r.WhichOneof("op")
                self.sink_name = r.mem_sink_op.name if k == "mem_sink_op" else r.grpc_sink_op.output_table.table_name

    # -----------------------------------------------------------------------------------
    def make_agg(self, ctx: Ctx) -> Agg:
        return Agg(ctx, self.keys, self.udas, self.filter, expected_groups=self.expected_groups, windowed=self.windowed)

    def run(self, ctx: Ctx, table: Table, agg: Optional[Agg] = None) -> List[Column]:
        if self.agg_op is None:
            return self._run_filter_map(ctx, table)
        own = agg is None
        if own:
            agg = self.make_agg(ctx)
        agg.consume(table)
        agg.finalize()
        cols = agg.result()
        if own:
            agg.close()
        return self.emit(cols)

    def emit(self, cols: List[Column]) -> List[Column]:
        """Agg output (quantiles as 7 doubles) -> the reference's output columns, then the
        post-agg Map (column refs and pluck_float64 of a quantiles column)."""
        nk = len(self.keys)
        out: List[Column] = []
        qraw: Dict[int, np.ndarray] = {}
        for j, c in enumerate(cols):
            if j >= nk and self.udas[j - nk].kind == _lib.UDA_QUANTILES:
                qraw[j] = c.values
                out.append(quantiles_json_column(c.values))
            else:
                out.append(c)
        if self.post_map is None:
            return out
        res = []
        for e in self.post_map.expressions:
            kind = e.WhichOneof("value")
            if kind == "column":
                res.append(out[int(e.column.index)])
            elif kind == "func" and e.func.name == "pluck_float64" and len(e.func.args) == 2 \
                    and e.func.args[0].WhichOneof("value") == "column" and e.func.args[1].WhichOneof("value") == "constant":
                src = int(e.func.args[0].column.index)
                key = e.func.args[1].constant.string_value
                if src in qraw and key in QUANTILE_KEYS:
                    q = qraw[src].reshape(-1, 7)
                    # a NaN / inf quantile truncates the JSON, which pluck_float64 fails to parse: 0.0
                    ok = np.isfinite(q).all(axis=1)
                    res.append(Column(FLOAT64, values=np.ascontiguousarray(np.where(ok, q[:, QUANTILE_KEYS.index(key)], 0.0))))
                else:
                    import json
                    vals = []
                    for s in out[src].to_list():
                        try:
                            d = json.loads(s)
                            v = d.get(key)
                            vals.append(float(v) if isinstance(v, float) else 0.0)
                        except Exception:
                            vals.append(0.0)
                    res.append(Column.from_values(FLOAT64, vals))
            else:
                raise UnsupportedError("post-agg Map supports column references and pluck_float64 only")
        return res

    def _run_filter_map(self, ctx: Ctx, table: Table) -> List[Column]:
        cur = table
        tmp = []
        if self.filter is not None:
            cur = cur.filter(self.filter, list(range(len(self.table_types))))
            tmp.append(cur)
        progs = [Prog(ins, t, pool) for ins, t, pool in self.env]
        out_t = cur.map(progs)
        cols = out_t.fetch_all()
        out_t.close()
        for t in tmp:
            t.close()
        return cols


def _and(a: Prog, b: Prog) -> Prog:
    base = len(a.pool)
    ins_b = [(op, ty, arg + base if (op == OP["CONST"] and ty in (STRING, _lib.UINT128)) else arg, imm)
             for op, ty, arg, imm in b.insns_py]
    return Prog(a.insns_py + ins_b + [(OP["AND"], BOOLEAN, 0, 0)], BOOLEAN, a.pool + b.pool)
