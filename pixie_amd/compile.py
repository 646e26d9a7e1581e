"""Compile planpb scalar / aggregate expressions into libpxg device programs.

This is the device side of udf::Registry (src/carnot/udf/registry.h:101-244): a scalar UDF is
resolved by (name, registry arg types) exactly as ExecState::AddScalarUDF does
(src/carnot/exec/exec_state.h:102-113, src/carnot/plan/scalar_expression.cc:243-252), then
lowered to typed postfix instructions.  Signatures follow the builtin registrations in
src/carnot/funcs/builtins/math_ops.cc:52-250 and math_sketches.cc:25-28; anything else raises
UnsupportedError (UNIMPLEMENTED) — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from . import _lib
from ._lib import BOOLEAN, FLOAT64, INT64, OP, STRING, TIME64NS, UINT128

B, I, U, F, S, T = BOOLEAN, INT64, UINT128, FLOAT64, STRING, TIME64NS


class UnsupportedError(NotImplementedError):
    """px.statuspb.UNIMPLEMENTED: no device implementation for this signature."""


# (name, (argtypes)) -> (result type, left conversion, right conversion, opcode list)
# conversion: None or an opcode applied right after that operand is pushed.
_UDFS: Dict[Tuple[str, Tuple[int, ...]], Tuple[int, Optional[str], Optional[str], List[str]]] = {}


def _reg(name, args, res, ops, lconv=None, rconv=None):
    _UDFS[(name, tuple(args))] = (res, lconv, rconv, ops)


# arithmetic (math_ops.h:33-150, math_ops.cc:57-105)
_reg("add", (I, I), I, ["ADD_I"]); _reg("add", (F, F), F, ["ADD_F"])
_reg("add", (F, I), F, ["ADD_F"], rconv="I2F"); _reg("add", (I, F), F, ["ADD_F"], lconv="I2F")
_reg("add", (T, I), T, ["ADD_I"]); _reg("add", (I, T), T, ["ADD_I"])
_reg("subtract", (I, I), I, ["SUB_I"]); _reg("subtract", (F, F), F, ["SUB_F"])
_reg("subtract", (F, I), F, ["SUB_F"], rconv="I2F"); _reg("subtract", (I, F), F, ["SUB_F"], lconv="I2F")
_reg("subtract", (T, I), T, ["SUB_I"]); _reg("subtract", (T, T), I, ["SUB_I"]); _reg("subtract", (I, T), I, ["SUB_I"])
for a, b in [(I, I), (F, I), (I, F), (F, F)]:  # DivideUDF: double(a) / double(b) (math_ops.h:84-89)
    _reg("divide", (a, b), F, ["DIV_F"], lconv="I2F" if a == I else None, rconv="I2F" if b == I else None)
_reg("multiply", (I, I), I, ["MUL_I"]); _reg("multiply", (F, F), F, ["MUL_F"])
_reg("multiply", (F, I), F, ["MUL_F"], rconv="I2F"); _reg("multiply", (I, F), F, ["MUL_F"], lconv="I2F")
for a, b in [(T, I), (T, T), (I, T), (I, I)]:
    _reg("modulo", (a, b), I, ["MOD_I"])
# logical (math_ops.h:265-315)
_reg("logicalOr", (I, I), B, ["OR"]); _reg("logicalOr", (B, B), B, ["OR"])
_reg("logicalAnd", (I, I), B, ["AND"]); _reg("logicalAnd", (B, B), B, ["AND"])
_reg("logicalNot", (I,), B, ["NOT"]); _reg("logicalNot", (B,), B, ["NOT"])
_reg("negate", (I,), I, ["NEG_I"]); _reg("negate", (F,), F, ["NEG_F"]); _reg("invert", (I,), I, ["INV_I"])
# equality (math_ops.cc:145-175); FLOAT64 == FLOAT64 is ApproxEqualUDF.
for t_ in (I, T, B):
    _reg("equal", (t_, t_), B, ["EQ_I"]); _reg("notEqual", (t_, t_), B, ["NE_I"])
_reg("equal", (S, S), B, ["EQ_S"]); _reg("notEqual", (S, S), B, ["NE_S"])
_reg("equal", (U, U), B, ["EQ_U"]); _reg("notEqual", (U, U), B, ["NE_U"])
_reg("equal", (B, I), B, ["EQ_I"]); _reg("equal", (I, B), B, ["EQ_I"])
_reg("notEqual", (B, I), B, ["NE_I"]); _reg("notEqual", (I, B), B, ["NE_I"])
_reg("equal", (I, F), B, ["EQ_F"], lconv="I2F"); _reg("equal", (F, I), B, ["EQ_F"], rconv="I2F")
_reg("notEqual", (I, F), B, ["NE_F"], lconv="I2F"); _reg("notEqual", (F, I), B, ["NE_F"], rconv="I2F")
_reg("equal", (F, F), B, ["APPROX_EQ_F"]); _reg("notEqual", (F, F), B, ["APPROX_NE_F"])
_reg("approxEqual", (F, F), B, ["APPROX_EQ_F"])
# ordering (math_ops.h:412-510)
for nm, sfx in [("greaterThan", "GT"), ("greaterThanEqual", "GE"), ("lessThan", "LT"), ("lessThanEqual", "LE")]:
    _reg(nm, (I, I), B, [sfx + "_I"]); _reg(nm, (T, T), B, [sfx + "_I"])
    _reg(nm, (F, F), B, [sfx + "_F"]); _reg(nm, (S, S), B, [sfx + "_S"])
# bin (math_ops.h:512-527)
_reg("bin", (I, I), I, ["BIN_I"]); _reg("bin", (T, T), T, ["BIN_I"]); _reg("bin", (I, T), I, ["BIN_I"])
_reg("bin", (T, I), T, ["BIN_I"]); _reg("bin", (F, I), I, ["BIN_I"], lconv="F2I")
_reg("time_to_int64", (T,), I, []); _reg("int64_to_time", (I,), T, [])
# Test-registry UDF of FilterNodeTest (filter_node_test.cc:41-53), registered like the reference
# test registers it ("eq" on INT64 and STRING).
_reg("eq", (I, I), B, ["EQ_I"]); _reg("eq", (S, S), B, ["EQ_S"])

# UDAs: (name, types) -> (kind, arg type, output type)
_UDAS = {}
for t_ in (F, I, B):
    _UDAS[("mean", (t_,))] = (_lib.UDA_MEAN, t_, F)
_UDAS[("sum", (F,))] = (_lib.UDA_SUM, F, F)
_UDAS[("sum", (I,))] = (_lib.UDA_SUM, I, I)
_UDAS[("sum", (B,))] = (_lib.UDA_SUM, B, I)
for t_ in (F, I, T):
    _UDAS[("max", (t_,))] = (_lib.UDA_MAX, t_, t_)
    _UDAS[("min", (t_,))] = (_lib.UDA_MIN, t_, t_)
for t_ in (F, I, T, B, S, U):
    _UDAS[("count", (t_,))] = (_lib.UDA_COUNT, t_, I)
_UDAS[("quantiles", (I,))] = (_lib.UDA_QUANTILES, I, S)
_UDAS[("quantiles", (F,))] = (_lib.UDA_QUANTILES, F, S)
# AggNodeTest's registry-local test UDAs (agg_node_test.cc:44-72, 282-289).
_UDAS[("minsum", (I, I))] = (_lib.UDA_MINSUM, I, I)
_UDAS[("minsum_w_init", (I, I, I))] = (_lib.UDA_MINSUM, I, I)


class Prog:
    """A pxg_program owned by Python (keeps its buffers alive)."""

    def __init__(self, insns: List[Tuple[int, int, int, int]], result_type: int, pool: bytes = b""):
        self.insns_py = insns
        self.result_type = result_type
        self.pool = pool
        self._arr = (_lib.Insn * max(1, len(insns)))(*[_lib.Insn(op, ty, arg, imm) for op, ty, arg, imm in insns])
        self._pool = C.create_string_buffer(pool + b"\0" * 16, len(pool) + 16)
        c = _lib.Program()
        c.n_insns = len(insns)
        c.result_type = result_type
        c.insns = self._arr
        c.pool_len = len(pool)
        c.pool = C.cast(self._pool, C.c_void_p)
        self.c = c

    @property
    def is_column(self) -> bool:
        return len(self.insns_py) == 1 and self.insns_py[0][0] == OP["COL"]


def col(index: int, type_: int) -> Prog:
    return Prog([(OP["COL"], type_, index, 0)], type_)


def _const_insn(v, pool: bytearray):
    dt = v.data_type
    if dt == BOOLEAN:
        return (OP["CONST"], dt, 0, 1 if v.bool_value else 0)
    if dt == INT64:
        return (OP["CONST"], dt, 0, v.int64_value)
    if dt == TIME64NS:
        return (OP["CONST"], dt, 0, v.time64_ns_value)
    if dt == FLOAT64:
        return (OP["CONST"], dt, 0, struct.unpack("<q", struct.pack("<d", v.float64_value))[0])
    if dt == STRING:
        b = v.string_value.encode()
        off = len(pool)
        pool.extend(b)
        while len(pool) % 8:
            pool.append(0)
        return (OP["CONST"], dt, off, len(b))
    if dt == UINT128:
        off = len(pool)
        pool.extend(struct.pack("<QQ", v.uint128_value.low, v.uint128_value.high))
        return (OP["CONST"], dt, off, 16)
    raise UnsupportedError(f"constant type {dt}")


class ExprCompiler:
    """Lowers planpb.ScalarExpression trees; `inline` maps an input column index to an already
    compiled instruction list (Map expressions substituted into downstream operators)."""

    def __init__(self, input_types: Sequence[int], inline: Optional[Dict[int, Tuple[list, int, bytes]]] = None):
        self.input_types = list(input_types)
        self.inline = inline or {}

    def type_of(self, e) -> int:
        _, t, _ = self._emit(e, bytearray())
        return t

    def compile(self, e) -> Prog:
        pool = bytearray()
        insns, t, _ = self._emit(e, pool)
        return Prog(insns, t, bytes(pool))

    def _emit(self, e, pool: bytearray):
        kind = e.WhichOneof("value")
        if kind == "column":
            idx = int(e.column.index)
            if idx in self.inline:
                ins, t, sub_pool = self.inline[idx]
                # relocate the sub-program's pool
                base = len(pool)
                pool.extend(sub_pool)
                out = [(op, ty, arg + base if (op == OP["CONST"] and ty in (STRING, UINT128)) else arg, imm)
                       for op, ty, arg, imm in ins]
                return out, t, None
            if idx >= len(self.input_types):
                raise ValueError(f"column {idx} out of range")
            t = self.input_types[idx]
            return [(OP["COL"], t, idx, 0)], t, None
        if kind == "constant":
            return [_const_insn(e.constant, pool)], e.constant.data_type, None
        if kind == "func":
            f = e.func
            if len(f.init_args):
                raise UnsupportedError(f"scalar UDF {f.name} with init args")
            parts = [self._emit(a, pool) for a in f.args]
            types = tuple(p[1] for p in parts)
            key = (f.name, types)
            if key not in _UDFS:
                raise UnsupportedError(f"no device UDF {f.name}{tuple(_lib.TYPE_NAMES.get(t, t) for t in types)}")
            res, lconv, rconv, ops = _UDFS[key]
            out = []
            for i, (ins, t, _) in enumerate(parts):
                out.extend(ins)
                conv = lconv if i == 0 else rconv
                if conv:
                    out.append((OP[conv], F if conv == "I2F" else I, 0, 0))
            for o in ops:
                out.append((OP[o], res, 0, 0))
            if not ops:  # time_to_int64 / int64_to_time: value unchanged, type relabelled (x + 0)
                out.append((OP["CONST"], I, 0, 0))
                out.append((OP["ADD_I"], res, 0, 0))
            return out, res, None
        raise ValueError("empty scalar expression")


@dataclass
class UdaDef:
    kind: int
    arg_type: int
    out_type: int
    arg: Optional[Prog]
    arg2: Optional[Prog]
    init: Optional[int]
    c: _lib.UdaSpec = field(default=None)

    def build(self):
        s = _lib.UdaSpec()
        s.kind = self.kind
        s.arg_type = self.arg_type
        if self.arg is not None:
            s.arg = self.arg.c
        if self.arg2 is not None:
            s.arg2 = self.arg2.c
        s.has_init = 1 if self.init is not None else 0
        s.init_i64 = self.init or 0
        self.c = s
        return self


def compile_uda(agg_expr, compiler: ExprCompiler) -> UdaDef:
    """Resolve an AggregateExpression (plan.proto:553-570) against the device UDA registry."""
    arg_progs = []
    for a in agg_expr.args:
        se = _planpb_scalar_from_arg(a)
        arg_progs.append(compiler.compile(se))
    init_types = tuple(v.data_type for v in agg_expr.init_args)
    types = init_types + tuple(p.result_type for p in arg_progs)
    key = (agg_expr.name, types)
    if key not in _UDAS:
        raise UnsupportedError(f"no device UDA {agg_expr.name}{tuple(_lib.TYPE_NAMES.get(t, t) for t in types)}")
    kind, at, out = _UDAS[key]
    init = None
    if agg_expr.init_args:
        init = int(agg_expr.init_args[0].int64_value)
    arg = arg_progs[0] if arg_progs else None
    arg2 = arg_progs[1] if len(arg_progs) > 1 else None
    if kind == _lib.UDA_COUNT:
        arg, arg2 = arg, None
    return UdaDef(kind, at, out, arg, arg2, init).build()


def _planpb_scalar_from_arg(a):
    from .planpb import ScalarExpression
    se = ScalarExpression()
    if a.WhichOneof("value") == "column":
        se.column.CopyFrom(a.column)
    else:
        se.constant.CopyFrom(a.constant)
    return se


def uda(kind: int, arg: Optional[Prog] = None, arg2: Optional[Prog] = None, init: Optional[int] = None) -> UdaDef:
    at = arg.result_type if arg is not None else INT64
    out = {_lib.UDA_COUNT: INT64, _lib.UDA_MEAN: FLOAT64, _lib.UDA_QUANTILES: STRING, _lib.UDA_MINSUM: INT64,
           _lib.UDA_SUM: FLOAT64 if at == FLOAT64 else INT64}.get(kind, at)
    if kind == _lib.UDA_COUNT and arg is None:
        at = INT64
    return UdaDef(kind, at, out, arg, arg2, init).build()
