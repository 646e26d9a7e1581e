"""The Python lowering (pixie_amd/compile.py + pipeline.py, used by tests/device_runner.py) and
the C++ engine's lowering (carnot_host.cc, what pxc_execute_plan and the bench run) must emit
the same device programs for the same plan: same fused filter, same group-key programs, same
UDA kinds and argument programs.  Guards the two registries against drifting apart."""
import pytest

from pixie_amd import host_engine as H
from pixie_amd import plans as P
from pixie_amd.pipeline import LinearQuery

HTTP = {"http_events": {"types": P.HTTP_TYPES, "batches": []}}


def _engine_lowering(plan, tables):
    txt = H.explain(plan, tables)
    lines = [l.strip() for l in txt.splitlines()]
    prog = lambda l: [tuple(int(x) for x in i.split(":")) for i in l.split(None, 1)[1].split()]  # noqa: E731
    filt = [prog(l) for l in lines if l.startswith("filter:")]
    keys = [prog(l) for l in lines if l.startswith("key:")]
    udas = []
    for l in lines:
        if l.startswith("uda kind="):
            kind = int(l.split()[1].split("=")[1])
            arg = l.split("arg=", 1)[1]
            udas.append((kind, None if arg == "-" else [tuple(int(x) for x in i.split(":")) for i in arg.split()]))
    return (filt[0] if filt else None), keys, udas


def _remap(p, idxs):
    """Engine programs over a host table reference projected source columns; map them to the
    table's own column indices (what the Python lowering emits)."""
    return [(op, ty, idxs[arg] if op == 1 else arg, imm) for op, ty, arg, imm in p]


PLANS = {
    "c1": P.c1_plan(),
    "c2": P.c2_plan(with_pluck=False),
    "c2_pluck": P.c2_plan(with_pluck=True),
    "c3": P.c3_plan(),
    "split_pem": P.split_source_plan(),
    "split_full": P.split_source_plan(partial_agg=False, finalize_results=False),
}


@pytest.mark.parametrize("name", sorted(PLANS))
def test_python_and_engine_lowerings_agree(name):
    plan = PLANS[name]
    idxs = list(plan.nodes[0].nodes[0].op.mem_source_op.column_idxs)
    filt, keys, udas = _engine_lowering(plan, HTTP)
    q = LinearQuery(plan, P.HTTP_TYPES)
    assert (q.filter is None) == (filt is None)
    if filt is not None:
        assert _remap(filt, idxs) == [tuple(i) for i in q.filter.insns_py]
    assert [_remap(k, idxs) for k in keys] == [[tuple(i) for i in k.insns_py] for k in q.keys]
    assert [k for k, _ in udas] == [u.kind for u in q.udas]
    for (kind, arg), u in zip(udas, q.udas):
        if arg is not None and u.arg is not None:
            assert _remap(arg, idxs) == [tuple(i) for i in u.arg.insns_py], (name, kind)
