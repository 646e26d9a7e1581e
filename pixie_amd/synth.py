"""Seeded synthetic conn_stats and pod metadata tables for C5.  Host-side numpy;
every value is a pure function of (seed, row) so shards of one table are independent.

conn_stats: time_ spans `span_s` seconds from t0 (ten-second bins -> span_s / 10 windows),
upid one of `n_pods` 128-bit ids, remote_addr one of `n_addrs` dotted quads, remote_port,
bytes_sent / bytes_recv uniform [0, 2^20).  pod_metadata: one row per upid for the first
`covered` fraction of the pods (so an inner join drops the rest) plus `extra` upids that never
appear in conn_stats."""
from __future__ import annotations

from typing import Dict, List

import numpy as np

from ._lib import INT64, STRING, TIME64NS, UINT128
from .device import Column

T0_NS = 1_700_000_000 * 10**9


def upids(n: int) -> np.ndarray:
    i = np.arange(n, dtype=np.uint64)
    lo = (i * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(0x5851F42D4C957F2D)
    hi = np.full(n, 0x0000_1000_0000_0000, dtype=np.uint64) | i
    return np.stack([lo, hi], axis=1)


def _strings(vals: List[str], idx: np.ndarray) -> Column:
    enc = [v.encode() for v in vals]
    lens = np.array([len(b) for b in enc], dtype=np.int64)[idx]
    offs = np.zeros(len(idx) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    blob = np.frombuffer(b"".join(enc), dtype=np.uint8)
    starts = np.concatenate([[0], np.cumsum([len(b) for b in enc])])[idx]
    # gather bytes: position p within row r comes from blob[starts[r] + p - offs[r]]
    row = np.repeat(np.arange(len(idx)), lens)
    pos = np.arange(int(offs[-1])) - offs[:-1][row] + starts[row]
    data = np.concatenate([blob[pos], np.zeros(16, np.uint8)]) if len(pos) else np.zeros(16, np.uint8)
    return Column(STRING, offsets=offs.astype(np.int32), data=data)


def addrs(n: int) -> List[str]:
    return [f"10.{(i >> 16) & 255}.{(i >> 8) & 255}.{i & 255}" for i in range(n)]


def conn_stats(seed: int, row_begin: int, nrows: int, n_pods: int = 2000, n_addrs: int = 5000,
               span_s: int = 300) -> List[Column]:
    rng = np.random.default_rng([seed, row_begin])
    t = T0_NS + rng.integers(0, span_s * 10**9, nrows, dtype=np.int64)
    pod = rng.integers(0, n_pods, nrows)
    addr = rng.integers(0, n_addrs, nrows)
    return [Column(TIME64NS, values=np.sort(t)),
            Column(UINT128, values=np.ascontiguousarray(upids(n_pods)[pod])),
            _strings(addrs(n_addrs), addr),
            Column(INT64, values=rng.integers(1024, 65536, nrows, dtype=np.int64)),
            Column(INT64, values=rng.integers(0, 1 << 20, nrows, dtype=np.int64)),
            Column(INT64, values=rng.integers(0, 1 << 20, nrows, dtype=np.int64))]


def pod_metadata(n_pods: int = 2000, covered: float = 0.9, extra: int = 200) -> List[Column]:
    keep = np.arange(int(n_pods * covered))
    ids = np.concatenate([upids(n_pods)[keep], upids(n_pods + extra)[n_pods:]])
    n = len(ids)
    names = [f"pl/pod-{i:05d}-{(i * 2654435761) % 100000:05x}" for i in range(n)]
    ns = ["pl", "kube-system", "default", "px-sock-shop", "online-boutique"]
    return [Column(UINT128, values=np.ascontiguousarray(ids)), _strings(names, np.arange(n)),
            _strings(ns, np.arange(n) % len(ns))]


def batched(cols: List[Column], rows_per_batch: int) -> List[List[Column]]:
    n = len(cols[0])
    return [[c.slice(a, min(a + rows_per_batch, n)) for c in cols] for a in range(0, n, rows_per_batch)]


def c5_tables(seed: int, nrows: int, rows_per_batch: int = 4096, **kw) -> Dict[str, dict]:
    from .plans import CONN_NAMES, CONN_TYPES, POD_NAMES, POD_TYPES
    n_pods = kw.get("n_pods", 2000)
    cs = conn_stats(seed, 0, nrows, n_pods=n_pods, n_addrs=kw.get("n_addrs", 5000), span_s=kw.get("span_s", 300))
    pm = pod_metadata(n_pods)
    return {"conn_stats": {"types": CONN_TYPES, "names": CONN_NAMES, "batches": batched(cs, rows_per_batch)},
            "pod_metadata": {"types": POD_TYPES, "names": POD_NAMES, "batches": batched(pm, 1024)}}
