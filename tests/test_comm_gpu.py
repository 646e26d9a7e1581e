"""The multi-GPU exchange on the device: pxg_comm (RCCL) + pxg_agg_alltoall, and two real
processes sharing GPU 0 that export -> exchange -> import -> finalize their row shards, checked
against the CPU restatement over the union of the shards (groups and counts
bit-exact, mean 1e-6, quantiles <= 4 ULP for groups <= 8000 values, rank bound above)."""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import oracle_client as oc
import parity
from pixie_amd import plans as P
from pixie_amd.device import Comm, Ctx, Table, datagen_http_events
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu
SEED = 20250117
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


_SELF = textwrap.dedent('''
    import sys
    sys.path.insert(0, {repo!r})
    from pixie_amd import plans as P
    from pixie_amd.device import Comm, Ctx, Table
    from pixie_amd.pipeline import LinearQuery
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events({seed}, 0, 2_000_000, 10_000_000)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    a.consume(t)
    a.finalize()
    local = sorted(map(tuple, zip(*[c.to_list() for c in a.result()])))
    print("comm init", flush=True)
    comm = Comm(ctx, 0, 1, Comm.unique_id())
    print("exchange", flush=True)
    # the bench's step, three times in a row: reset -> consume -> alltoall -> finalize
    for rep in range(3):
        a.reset()
        a.consume(t)
        sent, recv = a.alltoall(comm)
        assert sent == recv and sent > 0
        g = a.finalize()
        # world of one: the gather to rank 0 leaves the result as it is
        assert a.gather(comm, 0) == g
        merged = sorted(map(tuple, zip(*[c.to_list() for c in a.result()])))
        assert len(merged) == len(local), (rep, len(merged), len(local))
    # Keys, counts and means are identical (the per-group sums are double-double, rounded once,
    # so the staging order -- tile completion order -- does not reach them).  The quantiles of
    # groups > ~10,000 values come from the exported centroid lists (sort path) on one side and
    # the selection path on the other: equal up to their centroid sums' rounding.
    assert len(local) == len(merged)
    for x, y in zip(local, merged):
        assert x[:3] == y[:3], (x, y)
        assert x[3] == y[3], (x, y)
        if x[2] <= 10_000:
            assert x[4] == y[4], (x, y)
        else:
            assert all(abs(a - b) <= 1e-12 * abs(a) for a, b in zip(x[4], y[4])), (x, y)
    comm.close()
    print("ok", sent, flush=True)
''')

# RCCL's bootstrap uses a socket; on the single-GPU test box the loopback interface is the one
# every rank can reach.  RCCL calls cannot be interrupted in-process, so they run in children
# under a timeout.
_ENV = dict(NCCL_SOCKET_IFNAME="lo", NCCL_DEBUG="WARN")


def test_alltoall_single_rank_is_identity(tmp_path):
    """World of one: the RCCL exchange sends this rank's whole state to itself; finalize must
    give the local result (keys, counts, quantiles identical; means to the last bits)."""
    script = tmp_path / "self.py"
    script.write_text(_SELF.format(repo=REPO, seed=SEED))
    r = subprocess.run([sys.executable, str(script)], env=dict(os.environ, **_ENV), timeout=120, capture_output=True, text=True)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


_SELF_HC = textwrap.dedent('''
    import os, sys
    os.environ["PXG_HC_MIN_GROUPS"] = "1"
    sys.path.insert(0, {repo!r})
    from pixie_amd import plans as P
    from pixie_amd.device import Comm, Ctx, Table
    from pixie_amd.pipeline import LinearQuery
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events({seed}, 0, 1_000_000, 300_000)
    q = LinearQuery(P.c3_plan(), P.HTTP_TYPES, expected_groups=100_000)
    a = q.make_agg(ctx)
    a.consume(t)
    assert a.info()["hc_mode"] == 1
    a.finalize()
    local = sorted(map(tuple, zip(*[c.to_list() for c in a.result()])))
    comm = Comm(ctx, 0, 1, Comm.unique_id())
    for rep in range(2):
        a.reset()
        a.consume(t)
        assert a.info()["hc_mode"] == 1
        sent, recv = a.alltoall(comm)  # partition groups exported as states, no spill
        assert sent == recv and sent > 0
        g = a.finalize()
        merged = sorted(map(tuple, zip(*[c.to_list() for c in a.result()])))
        assert g == len(local) == len(merged), (rep, g, len(local), len(merged))
        for x, y in zip(local, merged):
            assert x[:3] == y[:3] and x[4] == y[4], (x, y)
            assert abs(x[3] - y[3]) <= 1e-12 * abs(x[3]), (x, y)
    comm.close()
    print("ok", sent, flush=True)
''')


def test_alltoall_single_rank_high_cardinality(tmp_path):
    """World of one over a high-cardinality run (C3 plan, partition records): the exchange sends
    the partition pass's groups as states (ExportHcGroups) and the merged result equals the
    local one (keys, counts, sums exact; means 1e-12)."""
    script = tmp_path / "self_hc.py"
    script.write_text(_SELF_HC.format(repo=REPO, seed=SEED))
    r = subprocess.run([sys.executable, str(script)], env=dict(os.environ, **_ENV), timeout=120, capture_output=True, text=True)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


_RANK = textwrap.dedent('''
    import json, os, sys
    sys.path.insert(0, {repo!r})
    import torch
    import torch.distributed as dist
    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table, Comm
    from pixie_amd.dist import exchange_partials
    from pixie_amd.pipeline import LinearQuery
    rank, world, n, mode, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events({seed}, rank * n, n, 10_000_000)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    a.consume(t)
    via = "gloo"
    if mode == "rccl":
        obj = [Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        try:
            comm = Comm(ctx, rank, world, obj[0])
            sent, recv = a.alltoall(comm)
            via = "rccl"
        except Exception as e:  # RCCL refuses two ranks on one device on some builds
            print("rccl unavailable on a shared GPU:", e, file=sys.stderr)
            sent, recv = exchange_partials(a)
    else:
        sent, recv = exchange_partials(a)
    a.finalize()
    cols = a.result()
    import numpy as np
    arrs = {{}}
    for j, c in enumerate(cols):
        arrs[f"t{{j}}"] = np.array([c.type])
        for f in ("values", "offsets", "data"):
            if getattr(c, f) is not None:
                arrs[f"{{f}}{{j}}"] = np.asarray(getattr(c, f))
    np.savez(out + ".npz", **arrs)
    json.dump({{"via": via, "sent": sent, "recv": recv, "ncols": len(cols)}}, open(out, "w"))
    dist.barrier()
    dist.destroy_process_group()
''')


@pytest.mark.parametrize("mode", ["gloo", "rccl"])
def test_two_processes_share_gpu0_exchange_matches_oracle(tmp_path, mode):
    world, n = 2, 300_000
    script = tmp_path / "rank.py"
    script.write_text(_RANK.format(repo=REPO, seed=SEED))
    env = dict(os.environ, **_ENV, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29500 + (os.getpid() % 1000) + (7 if mode == "rccl" else 0)))
    procs = [subprocess.Popen([sys.executable, str(script), str(r), str(world), str(n), mode, str(tmp_path / f"r{r}.json")], env=env)
             for r in range(world)]
    import time
    deadline = time.time() + 150
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=max(1.0, deadline - time.time())))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("rank process timed out")
    assert codes == [0, 0]
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    from pixie_amd.device import Column
    parts = []
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.json.npz")
        parts.append([Column(int(z[f"t{j}"][0]), **{f: z[f"{f}{j}"] for f in ("values", "offsets", "data") if f"{f}{j}" in z})
                      for j in range(res[r]["ncols"])])
    dev = parity.concat_columns(parts)
    # oracle over the union of both shards
    cols = datagen_http_events(SEED, 0, world * n, n_pair_keys=10_000_000, threads=8)
    plan = P.c2_plan(with_pluck=False)
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}
    ref = oc.execute_plan(plan, tables)["output"][0]["cols"]
    gv = parity.GroupValues([[cols[2], cols[3]]], [cols[5].values >= 400], [cols[6].values / 1e6])
    rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "quantiles"], gv)
    assert rep["ok"], rep  # compare_agg also rejects a group finalized on two ranks (duplicates)
    for x in res:
        assert x["sent"] > 0 and x["recv"] > 0
    print("exchange via", [x["via"] for x in res], "bytes sent / received per rank", [(x["sent"], x["recv"]) for x in res])
    if mode == "rccl" and any(x["via"] != "rccl" for x in res):
        # RCCL refuses two ranks on one device ("invalid usage": duplicate GPU), so on a one-GPU
        # box the ranks exchanged over gloo; the result above is still checked, but the RCCL
        # multi-rank transport itself is not exercised here (world 1 covers pxg_agg_alltoall).
        pytest.skip("RCCL refuses two ranks on one GPU; exchange fell back to gloo (result checked)")
