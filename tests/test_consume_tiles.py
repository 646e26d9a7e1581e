"""The fast consume kernel's 32768-row tiles (chosen in production only when a launch has >= 8
rounds of resident workgroups, i.e. ~1B rows) against the CPU restatement at a size the oracle
finishes quickly: a child process forces the tile size (PXG_CONSUME_TILE is read once per
process) and runs the C2 plan over device-generated rows; the parent compares with the oracle
using the bench's parity bars (groups and counts bit-exact, mean 1e-6, quantiles <= 4 ULP /
rank bound)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_client as oc
import parity
from pixie_amd import plans as P
from pixie_amd.device import Column, datagen_http_events

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 20250117

_CHILD = r'''
import sys
sys.path.insert(0, {repo!r})
import numpy as np
from pixie_amd import plans as P
from pixie_amd.device import Ctx, Table
from pixie_amd.pipeline import LinearQuery
n, out = int(sys.argv[1]), sys.argv[2]
ctx = Ctx(0)
t = Table(ctx, P.HTTP_TYPES)
t.append_http_events({seed}, 0, n, 10_000_000)
q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
cols = q.run(ctx, t)
arrs = {{}}
for j, c in enumerate(cols):
    arrs[f"t{{j}}"] = np.array([c.type])
    for f in ("values", "offsets", "data"):
        if getattr(c, f) is not None:
            arrs[f"{{f}}{{j}}"] = np.asarray(getattr(c, f))
np.savez(out, **arrs)
'''


@pytest.mark.parametrize("tile", ["32768"])
def test_forced_tile_size_matches_oracle(tmp_path, tile):
    n = 3_000_000
    script = tmp_path / "child.py"
    script.write_text(_CHILD.format(repo=REPO, seed=SEED))
    out = tmp_path / "res.npz"
    r = subprocess.run([sys.executable, str(script), str(n), str(out)], env=dict(os.environ, PXG_CONSUME_TILE=tile),
                       timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    z = np.load(out)
    ncols = sum(1 for k in z.files if k.startswith("t"))
    dev = [Column(int(z[f"t{j}"][0]), **{f: z[f"{f}{j}"] for f in ("values", "offsets", "data") if f"{f}{j}" in z})
           for j in range(ncols)]
    cols = datagen_http_events(SEED, 0, n, n_pair_keys=10_000_000, threads=8)
    plan = P.c2_plan(with_pluck=False)
    ref = oc.execute_plan(plan, {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}})["output"][0]["cols"]
    gv = parity.GroupValues([[cols[2], cols[3]]], [cols[5].values >= 400], [cols[6].values / 1e6])
    rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "quantiles"], gv)
    assert rep["ok"], rep
