"""CPU (gloo, world_size 2 and 3) coverage of the multi-rank exchange in pixie_amd/dist.py:
the export -> all-to-all(v) -> reset -> import protocol, with a host stand-in for the device
agg that serialises (key, value) records the way pxg_agg_export_partial lays out parts
(8-byte aligned segments, back to back).  The device export/import kernels themselves are
covered by tests/test_partial.py on the GPU."""
import os
import socket
import struct
import zlib

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pixie_amd.dist import exchange_partials, segments


class HostAgg:
    """Groups keyed by string, each with a list of int values; part = crc32(key) % n."""
    device = "cpu"

    def __init__(self, rows):
        self.groups = {}
        for k, v in rows:
            self.groups.setdefault(k, []).append(v)

    def _parts(self, n):
        parts = [b""] * n
        for k in sorted(self.groups):
            kb = k.encode()
            vs = self.groups[k]
            rec = struct.pack("<II", len(kb), len(vs)) + kb + struct.pack(f"<{len(vs)}q", *vs)
            parts[zlib.crc32(kb) % n] += rec
        return parts

    def export_partial(self, n, dst=None):
        parts = self._parts(n)
        offs, nb, at = [], [], 0
        for p in parts:
            offs.append(at)
            nb.append(len(p))
            at += (len(p) + 7) & ~7
        if dst is not None:
            for o, p in zip(offs, parts):
                if p:
                    dst[o:o + len(p)] = torch.frombuffer(bytearray(p), dtype=torch.uint8)
        return offs, nb

    def reset(self):
        self.groups = {}

    def import_partial(self, src):
        b = bytes(src.numpy().tobytes())
        at = 0
        while at + 8 <= len(b):
            kl, nv = struct.unpack_from("<II", b, at)
            if kl == 0 and nv == 0:
                break   # alignment padding
            at += 8
            k = b[at:at + kl].decode()
            at += kl
            vs = list(struct.unpack_from(f"<{nv}q", b, at))
            at += 8 * nv
            self.groups.setdefault(k, []).extend(vs)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = [(f"svc-{(rank * 7 + i) % 23}", rank * 1000 + i) for i in range(200 + 37 * rank)]
        agg = HostAgg(rows)
        sent, recvd = exchange_partials(agg)
        owned = {k: sorted(v) for k, v in agg.groups.items()}
        assert all(zlib.crc32(k.encode()) % world == rank for k in owned)
        q.put((rank, owned, sent, recvd))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_partitions_every_group_to_one_owner(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    merged = {}
    for _, owned, _, _ in res:
        assert not (set(owned) & set(merged))
        merged.update(owned)
    want = {}
    for rank in range(world):
        for i in range(200 + 37 * rank):
            want.setdefault(f"svc-{(rank * 7 + i) % 23}", []).append(rank * 1000 + i)
    assert merged == {k: sorted(v) for k, v in want.items()}
    assert sum(r[2] for r in res) == sum(r[3] for r in res)


def test_segments_are_aligned_and_cover_parts():
    offs, nb = [0, 16, 40], [13, 20, 5]
    assert segments(offs, nb) == [16, 24, 8]


def _transport_worker(rank, world, port, q):
    """Two batches like pxg_agg_alltoall's: {8-byte count, 64-byte header} per peer, then parts
    of per-peer sizes; every transfer to a peer matched in issue order (tags)."""
    from pixie_amd.dist import GlooTransport
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = GlooTransport()
        size = lambda s, d: 0 if (s + d) % 3 == 2 else 1 + 37 * s + 11 * d  # some pairs send nothing
        bufs = []
        ops = []
        for p in range(world):
            if p == rank:
                continue  # libpxg never passes self transfers
            cnt = bytearray(struct.pack("<q", size(rank, p)))
            hdr = bytearray(bytes([rank * 16 + p]) * 64)
            rc, rh = bytearray(8), bytearray(64)
            bufs += [cnt, hdr, rc, rh]
            ops += [(p, True, memoryview(cnt)), (p, False, memoryview(rc)), (p, True, memoryview(hdr)), (p, False, memoryview(rh))]
        tr(ops)
        got = {}
        for i, p in enumerate(x for x in range(world) if x != rank):
            rc, rh = bufs[4 * i + 2], bufs[4 * i + 3]
            got[p] = struct.unpack("<q", bytes(rc))[0]
            assert bytes(rh) == bytes([p * 16 + rank]) * 64
        parts, ops = {}, []
        for p in range(world):
            if p == rank:
                continue
            n = size(rank, p)
            if n:
                out = bytearray((rank * 31 + p + i) & 0xFF for i in range(n))
                parts[("s", p)] = out
                ops.append((p, True, memoryview(out)))
            if got[p]:
                inb = bytearray(got[p])
                parts[("r", p)] = inb
                ops.append((p, False, memoryview(inb)))
        tr(ops)
        for p in range(world):
            if p != rank and got[p]:
                want = bytes((p * 31 + rank + i) & 0xFF for i in range(size(p, rank)))
                assert bytes(parts[("r", p)]) == want, (rank, p)
        q.put((rank, tr.batches))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_transport_matches_transfers_in_order(world):
    """The host communicator's byte mover (pixie_amd.dist.GlooTransport, behind
    pxg_comm_init_host) on gloo: per-peer transfers meet in issue order, zero-size pairs are
    skipped symmetrically, every byte arrives."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transport_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert sorted(r[1] for r in res) == [2] * world
