"""Wall time of the boundary-chain builders (pxg_digest_chains) for a few group-size mixes."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pixie_amd import _lib  # noqa: E402
from pixie_amd.device import Ctx  # noqa: E402

ctx = Ctx(0)
lib = _lib.load()
cap = 2048


def run(ws, wave, reps=5):
    w = torch.tensor(ws, dtype=torch.int64, device="cuda")
    starts = torch.zeros(len(ws) * cap, dtype=torch.int32, device="cuda")
    nc = torch.zeros(len(ws), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        _lib.check(lib.pxg_digest_chains(ctx.h, C.c_void_p(w.data_ptr()), len(ws), wave, C.c_void_p(starts.data_ptr()), cap,
                                         C.c_void_p(nc.data_ptr())))
        best = min(best, time.perf_counter() - t)
    return best * 1e3


rng = np.random.default_rng(1)
for name, ws in [("1 x W=4096", [4096]), ("1 x W=720000", [720000]), ("64 x W in [1201,4096]", list(rng.integers(1201, 4097, 64))),
                 ("4000 x W in [1201,4096]", list(rng.integers(1201, 4097, 4000))),
                 ("14600 x W (2/3 exit)", list(rng.integers(1201, 4097, 4000)) + [100] * 10600)]:
    ws = [int(x) for x in ws]
    print(f"{name:28s} seq {run(ws, 0):8.3f} ms   wave {run(ws, 1):8.3f} ms", flush=True)

# instrumented single chains
for W in [1500, 4096, 20000, 720000]:
    w = torch.tensor([W], dtype=torch.int64, device="cuda")
    starts = torch.zeros(cap, dtype=torch.int32, device="cuda")
    nc = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.check(lib.pxg_digest_chains(ctx.h, C.c_void_p(w.data_ptr()), 1, 2, C.c_void_p(starts.data_ptr()), cap, C.c_void_p(nc.data_ptr())))
    st = starts.cpu().numpy()[cap - 8:].view(np.uint64)
    print(f"W={W}: nc={int(nc[0])} eval_cycles={st[0]} resolve_cycles={st[1]} rounds={st[2]} exact_rounds={st[3]} "
          f"-> {st[0]/max(st[2],1):.0f} + {st[1]/max(st[2],1):.0f} cycles/round", flush=True)
