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
    from datetime import timedelta
    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table, Comm
    from pixie_amd.dist import exchange_partials, gather_device_results, close_host_comms
    from pixie_amd.pipeline import LinearQuery
    rank, world, n, mode, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    plan_name = sys.argv[6] if len(sys.argv) > 6 else "c2"
    if plan_name == "c3":
        os.environ["PXG_HC_MIN_GROUPS"] = "1"  # the high-cardinality path: partition groups exported as states
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world, timeout=timedelta(seconds=90))
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events({seed}, rank * n, n, 300_000 if plan_name == "c3" else 10_000_000)
    plan = P.c3_plan() if plan_name == "c3" else P.c2_plan(with_pluck=False)
    q = LinearQuery(plan, P.HTTP_TYPES, expected_groups=100_000 if plan_name == "c3" else 65536)
    a = q.make_agg(ctx)
    reps = 2 if mode == "gloo" else 1
    for rep in range(reps):  # the bench's step twice: the host communicator and buffers are reused
        a.reset()
        a.consume(t)
        selected = a.rows_selected()
        hc = a.info()["hc_mode"]  # the consume's mode (the exchange resets and imports)
        via = "host-comm"
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
            # pxg_agg_alltoall over a host communicator: ExportPartialDev / XLayoutDevKernel /
            # ImportPartialsV2 with the received headers, bytes over gloo
            sent, recv = exchange_partials(a)
        owned = a.finalize()
        gathered = gather_device_results(a) if via == "host-comm" else None
    cols = a.result() if (via != "host-comm" or rank == 0) else []
    import numpy as np
    arrs = {{}}
    for j, c in enumerate(cols):
        arrs[f"t{{j}}"] = np.array([c.type])
        for f in ("values", "offsets", "data"):
            if getattr(c, f) is not None:
                arrs[f"{{f}}{{j}}"] = np.asarray(getattr(c, f))
    np.savez(out + ".npz", **arrs)
    json.dump({{"via": via, "sent": sent, "recv": recv, "ncols": len(cols), "owned": owned, "gathered": gathered,
               "selected": selected, "hc": hc}}, open(out, "w"))
    dist.barrier()
    close_host_comms()
    dist.destroy_process_group()
''')


def _run_ranks(tmp_path, mode, world, n, plan_name="c2"):
    script = tmp_path / "rank.py"
    script.write_text(_RANK.format(repo=REPO, seed=SEED))
    env = dict(os.environ, **_ENV, MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(29500 + (os.getpid() % 1000) + (7 if mode == "rccl" else 0) + 13 * world + (3 if plan_name == "c3" else 0)))
    procs = [subprocess.Popen([sys.executable, str(script), str(r), str(world), str(n), mode, str(tmp_path / f"r{r}.json"), plan_name],
                              env=env)
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
    assert codes == [0] * world
    return [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]


def _load_cols(tmp_path, r, ncols):
    from pixie_amd.device import Column
    z = np.load(tmp_path / f"r{r}.json.npz")
    return [Column(int(z[f"t{j}"][0]), **{f: z[f"{f}{j}"] for f in ("values", "offsets", "data") if f"{f}{j}" in z})
            for j in range(ncols)]


def _check_against_oracle(dev, world, n):
    cols = datagen_http_events(SEED, 0, world * n, n_pair_keys=10_000_000, threads=8)
    plan = P.c2_plan(with_pluck=False)
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}
    ref = oc.execute_plan(plan, tables)["output"][0]["cols"]
    gv = parity.GroupValues([[cols[2], cols[3]]], [cols[5].values >= 400], [cols[6].values / 1e6])
    rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "quantiles"], gv)
    assert rep["ok"], rep  # compare_agg also rejects a group finalized on two ranks (duplicates)
    sel = int((cols[5].values >= 400).sum())
    return sel


@pytest.mark.parametrize("world", [2, 3])
def test_host_comm_alltoall_and_gather_match_oracle(tmp_path, world):
    """the RCCL path's device code at world > 1.  Ranks sharing GPU 0 run
    pxg_agg_alltoall + pxg_agg_gather over a host communicator (pxg_comm_init_host, bytes over
    gloo): ExportPartialDev's device part layout, the {bytes, header} records, ImportPartialsV2
    with the received headers and GatherRebaseKernel's multi-rank rebase.  Rank 0's gathered
    result is checked against the oracle over the union of the shards."""
    n = 300_000
    res = _run_ranks(tmp_path, "gloo", world, n)
    assert all(x["via"] == "host-comm" for x in res)
    dev = _load_cols(tmp_path, 0, res[0]["ncols"])
    sel = _check_against_oracle(dev, world, n)
    assert res[0]["gathered"] == sum(x["owned"] for x in res) == len(dev[0])
    assert all(x["gathered"] == 0 for x in res[1:])
    assert sum(x["selected"] for x in res) == sel  # rows_selected before the exchange
    assert sum(x["sent"] for x in res) == sum(x["recv"] for x in res)
    for x in res:
        assert x["sent"] > 0 and x["recv"] > 0


def test_host_comm_high_cardinality_matches_oracle(tmp_path):
    """The C3 shape (high-cardinality mode: the partition pass's groups exported as states,
    ExportHcGroups) through pxg_agg_alltoall + pxg_agg_gather at world 2 over the host
    communicator, against the oracle over both shards: keys, counts and sums exact, means 1e-6."""
    world, n = 2, 400_000
    res = _run_ranks(tmp_path, "gloo", world, n, plan_name="c3")
    assert all(x["via"] == "host-comm" and x["hc"] == 1 for x in res)
    dev = _load_cols(tmp_path, 0, res[0]["ncols"])
    cols = datagen_http_events(SEED, 0, world * n, n_pair_keys=300_000, threads=8)
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}
    ref = oc.execute_plan(P.c3_plan(), tables)["output"][0]["cols"]
    rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "exact"])
    assert rep["ok"], rep
    assert res[0]["gathered"] == sum(x["owned"] for x in res) == rep["groups_ref"]


def test_two_processes_share_gpu0_rccl_or_skip(tmp_path):
    world, n = 2, 300_000
    res = _run_ranks(tmp_path, "rccl", world, n)
    if any(x["via"] != "rccl" for x in res):
        # RCCL refuses two ranks on one device ("invalid usage": duplicate GPU), so on a one-GPU
        # box the ranks exchanged over the host communicator instead (covered above).
        pytest.skip("RCCL refuses two ranks on one GPU; exchange fell back to the host communicator")
    parts = [_load_cols(tmp_path, r, res[r]["ncols"]) for r in range(world)]
    _check_against_oracle(parity.concat_columns(parts), world, n)


def _hip():
    import ctypes as C
    import torch  # noqa: F401  (one HIP runtime: torch's, which libpxg shares)
    h = C.CDLL("libamdhip64.so.7")
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipMemcpy.restype = C.c_int
    return h


def _dev_bytes(ptr, n):
    import ctypes as C
    buf = (C.c_uint8 * max(n, 1))()
    assert _hip().hipMemcpy(C.addressof(buf), ptr, n, 2) == 0  # hipMemcpyDeviceToHost
    return bytes(buf)[:n]


@pytest.mark.parametrize("plan_name", ["c2", "c3_hc"])
def test_device_export_layout_matches_host_layout(ctx, plan_name):
    """ExportPartialDev (the device layout pxg_agg_alltoall sends) against ExportPartialV2 (the
    host layout of pxg_agg_export_partial) at n_parts 2, 3 and 8: every part's bytes and header
    identical, sizes equal up to the 8-byte alignment."""
    import torch
    if plan_name == "c3_hc":
        os.environ["PXG_HC_MIN_GROUPS"] = "1"
    try:
        t = Table(ctx, P.HTTP_TYPES)
        t.append_http_events(SEED, 0, 1_000_000, 300_000 if plan_name == "c3_hc" else 10_000_000)
        plan = P.c3_plan() if plan_name == "c3_hc" else P.c2_plan(with_pluck=False)
        q = LinearQuery(plan, P.HTTP_TYPES, expected_groups=100_000 if plan_name == "c3_hc" else 65536)
        a = q.make_agg(ctx)
        for n_parts in (2, 3, 8):
            a.reset()
            a.consume(t)
            if plan_name == "c3_hc":
                assert a.info()["hc_mode"] == 1
            offs, nb = a.export_partial(n_parts)
            buf = torch.zeros(max(sum(_seg(offs, nb)), 8), dtype=torch.uint8, device="cuda")
            a.export_partial(n_parts, buf)
            host = buf.cpu().numpy().tobytes()
            ptr, seg, hdr = a.export_partial_dev(n_parts)
            assert seg == [(b + 7) & ~7 for b in nb], (n_parts, seg, nb)
            dev = _dev_bytes(ptr, sum(seg))
            at = 0
            for p in range(n_parts):
                assert dev[at:at + nb[p]] == host[offs[p]:offs[p] + nb[p]], (plan_name, n_parts, p)
                assert hdr[64 * p:64 * (p + 1)] == host[offs[p]:offs[p] + 64], (plan_name, n_parts, p)
                at += seg[p]
        a.close()
        t.close()
    finally:
        os.environ.pop("PXG_HC_MIN_GROUPS", None)


def _seg(offs, nb):
    from pixie_amd.dist import segments
    return segments(offs, nb)


_FAIL_RANK = textwrap.dedent('''
    import json, os, sys
    sys.path.insert(0, {repo!r})
    import torch
    import torch.distributed as dist
    from datetime import timedelta
    from pixie_amd import plans as P
    from pixie_amd._lib import PxgError
    from pixie_amd.device import Ctx, Table
    from pixie_amd.dist import exchange_partials, close_host_comms
    from pixie_amd.pipeline import LinearQuery
    rank, world, kind, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events({seed}, rank * 200_000, 200_000, 10_000_000)
    a = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536).make_agg(ctx)
    a.consume(t)
    if rank == world - 1:
        os.environ["PXG_TEST_EXPORT_FAIL"] = kind
    res = {{"rank": rank}}
    try:
        exchange_partials(a)
        res["error"] = None
    except PxgError as e:
        res["error"] = str(e)
    os.environ.pop("PXG_TEST_EXPORT_FAIL", None)
    # the communicator is still usable afterwards: a clean exchange of the same state
    a.reset()
    a.consume(t)
    sent, recv = exchange_partials(a)
    res["after"] = [sent, recv]
    json.dump(res, open(out, "w"))
    dist.barrier()
    close_host_comms()
    dist.destroy_process_group()
''')


@pytest.mark.parametrize("kind", ["host", "device"])
def test_failed_export_fails_every_rank_without_a_hang(tmp_path, kind):
    """a rank whose export fails -- on the host before anything is issued,
    or in the device layout (finalize checks / send-buffer bound) -- announces -1 bytes in the
    {bytes, header} exchange; then no rank posts the part exchange and every rank returns an
    error (the peers name the failed rank) instead of waiting.  The same communicator then runs
    a clean exchange."""
    world = 3
    script = tmp_path / "fail_rank.py"
    script.write_text(_FAIL_RANK.format(repo=REPO, seed=SEED))
    env = dict(os.environ, **_ENV, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(31000 + (os.getpid() % 1000) + (5 if kind == "device" else 0)))
    procs = [subprocess.Popen([sys.executable, str(script), str(r), str(world), kind, str(tmp_path / f"f{r}.json")], env=env)
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
            pytest.fail("a rank hung after an export failure")
    assert codes == [0] * world
    res = [json.load(open(tmp_path / f"f{r}.json")) for r in range(world)]
    assert all(x["error"] for x in res), res
    for x in res[:-1]:
        assert f"rank {world - 1} failed its export" in x["error"], x
    assert all(x["after"][0] > 0 and x["after"][1] > 0 for x in res)
