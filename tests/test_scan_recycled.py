"""Look-back scan status words in device memory recycled from another process.

The single-pass u32 scan (pxg_scan.hip ScanLookbackU32Kernel) tags each tile's status word with
an epoch.  Epochs count from 1 in every process, so device memory that another process of this
library freed can come back holding words whose epoch is live in this one.  Process A generates
tables with one seed and exits; process B then generates tables of the same sizes with another
seed (the same sequence of scans, so the same epochs, over the memory A just freed) and its
string offsets and rows must equal the host generator's."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

from golden.make_datagen_hash import digests
from pixie_amd.device import datagen_http_events

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS, TABLES = 6_000_000, 3

_GEN = textwrap.dedent('''
    import json, sys
    sys.path.insert(0, {repo!r})
    sys.path.insert(0, {tests!r})
    import numpy as np
    from golden.make_datagen_hash import digests
    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table
    seed, out = int(sys.argv[1]), sys.argv[2]
    ctx = Ctx(0)
    res = []
    for i in range({tables}):
        t = Table(ctx, P.HTTP_TYPES)
        t.append_http_events(seed, i * {rows}, {rows}, 10_000_000)
        cols = t.fetch_all()
        mono = all(bool(np.all(np.diff(np.asarray(c.offsets, dtype=np.int64)) >= 0)) for c in cols if c.offsets is not None)
        res.append({{"monotone": mono, "digests": digests(cols) if i == 0 else None}})
        t.close()
    json.dump(res, open(out, "w"))
    ctx.close()
''')


def _run(tmp_path, seed, name):
    script = tmp_path / "gen.py"
    script.write_text(_GEN.format(repo=REPO, tests=os.path.join(REPO, "tests"), rows=ROWS, tables=TABLES))
    out = tmp_path / name
    subprocess.run([sys.executable, str(script), str(seed), str(out)], check=True, timeout=240)
    return json.load(open(out))


def test_scans_ignore_status_words_left_by_another_process(tmp_path):
    _run(tmp_path, 1, "a.json")
    b = _run(tmp_path, 20250117, "b.json")
    assert all(x["monotone"] for x in b), b
    host = datagen_http_events(20250117, 0, ROWS, n_pair_keys=10_000_000, threads=8)
    assert b[0]["digests"] == json.loads(json.dumps(digests(host)))
