"""TEST INFRASTRUCTURE ONLY: a CPU stand-in for one rank of bench.py's N > 1 step, so that the
launcher (`bench.py --gpus N` starting its own ranks), the gloo rendezvous on 127.0.0.1, the
barrier-bracketed timed loop, the max over ranks, the rank-0 gather and the generator-truth parity
block can be exercised on a machine without a GPU (tests/test_bench_launch.py).  bench.py loads it
only under the hidden --standin flag, and then marks its JSON line "STAND-IN".

The step mirrors the device protocol with host arithmetic:
  * the rank's shard [rank * n, (rank + 1) * n) of the synthetic http_events table (the libpxg
    host generator, bit-identical to the device one);
  * Filter(resp_status >= 400) -> latency / 1e6 keyed by (service, req_path);
  * exchange of the selected (group, value) rows to owner = group % world (all_to_all_single);
  * per owned group count, mean and the restated t-digest quantiles (oracle/, every group here
    has <= 8000 values, so the digest is order-independent);
  * the owners' result columns gathered on rank 0 (pixie_amd.dist.gather_results).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

import oracle_client as oc
import parity
from pixie_amd import plans as P
from pixie_amd.device import Column, datagen_http_events
from pixie_amd.dist import gather_results


class StandinRank:
    def __init__(self, args, rank, world, seed, n_pair_keys):
        self.rank, self.world = rank, world
        self.n = args.rows_per_gpu or 50_000
        cols = datagen_http_events(seed, rank * self.n, self.n, n_pair_keys=n_pair_keys, threads=2)
        self.svc, self.paths = parity.http_events_key_tables()
        svc_id = {s: i for i, s in enumerate(self.svc)}
        path_id = {}
        for i, p in enumerate(self.paths):
            path_id.setdefault(p, i)
        sv, pa = cols[P.HE["service"]], cols[P.HE["req_path"]]
        sraw, praw = sv.data.tobytes(), pa.data.tobytes()
        so, po = sv.offsets, pa.offsets
        gid = np.array([svc_id[sraw[so[i]:so[i + 1]]] * 1024 + path_id[praw[po[i]:po[i + 1]]] for i in range(self.n)], np.int64)
        sel = cols[P.HE["resp_status"]].values >= 400
        self.gid = gid[sel]
        self.val = cols[P.HE["latency"]].values[sel] / 1e6
        self.alg_bytes = 16 * self.n + sum(len(c.data) - 16 + 4 * len(c) for c in (sv, pa))
        self.exch = {"bytes_sent": 0, "bytes_recv": 0, "via": "torch.distributed all_to_all_single (gloo, stand-in)",
                     "gather": "torch.distributed gather_object"}
        self.parts = None

    def step(self):
        owner = self.gid % self.world
        order = np.argsort(owner, kind="stable")
        g, v = self.gid[order], self.val[order]
        send = np.bincount(owner, minlength=self.world).astype(np.int64)
        recv = torch.empty(self.world, dtype=torch.int64)
        dist.all_to_all_single(recv, torch.from_numpy(send))
        rs = recv.tolist()
        rg = torch.empty(sum(rs), dtype=torch.int64)
        rv = torch.empty(sum(rs), dtype=torch.float64)
        dist.all_to_all_single(rg, torch.from_numpy(g), output_split_sizes=rs, input_split_sizes=send.tolist())
        dist.all_to_all_single(rv, torch.from_numpy(v), output_split_sizes=rs, input_split_sizes=send.tolist())
        rg, rv = rg.numpy(), rv.numpy()
        o = np.argsort(rg, kind="stable")
        rg, rv = rg[o], rv[o]
        keys, starts, counts = np.unique(rg, return_index=True, return_counts=True)
        lib = oc.load()
        q = np.zeros((len(keys), 7))
        for i, (a, c) in enumerate(zip(starts, counts)):
            x = np.ascontiguousarray(rv[a:a + c])
            lib.oracle_tdigest_quantiles(x.ctypes.data_as(C.POINTER(C.c_double)), len(x), q[i].ctypes.data_as(C.POINTER(C.c_double)))
        means = np.add.reduceat(rv, starts) / counts if len(keys) else np.zeros(0)
        cols = [Column.from_values(P.STRING, [self.svc[k // 1024] for k in keys]),
                Column.from_values(P.STRING, [self.paths[k % 1024] for k in keys]),
                Column(P.INT64, values=counts.astype(np.int64)), Column(P.FLOAT64, values=means), Column(P.FLOAT64, values=q)]
        self.parts = gather_results(cols)
        self.exch["bytes_sent"], self.exch["bytes_recv"] = int(16 * len(g)), int(16 * len(rg))
        return sum(len(p[0]) for p in self.parts) if self.parts else 0

    def sync(self):
        pass

    def profile(self):
        return {}

    def start_timing(self):
        pass

    def consume_ms(self):
        return 0, 0.0, 0.0

    def selected(self):
        return int(len(self.gid))

    def result(self):
        return parity.concat_columns(self.parts)

    def close(self):
        pass
