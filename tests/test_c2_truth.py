"""The generator ground truth used for parity at the 1B-row north_star size
(oracle/http_events_truth.cc, tests/parity.py::check_c2_against_truth) against the host generator's
materialised table grouped by exact key bytes (CPU)."""
import numpy as np

import parity
from pixie_amd import plans as P
from pixie_amd.device import datagen_http_events

SEED = 20250117


def _by_key(cols):
    svc, path = cols[P.HE["service"]], cols[P.HE["req_path"]]
    sel = cols[P.HE["resp_status"]].values >= 400
    lat = cols[P.HE["latency"]].values
    out = {}
    so, sd, po, pd = svc.offsets, svc.data.tobytes(), path.offsets, path.data.tobytes()
    for r in np.flatnonzero(sel):
        k = (sd[so[r]:so[r + 1]], pd[po[r]:po[r + 1]])
        out.setdefault(k, []).append(lat[r] / 1e6)
    return out


def test_truth_matches_materialised_generator_rows():
    row0, n = 123_456_789, 200_000
    ref = _by_key(datagen_http_events(SEED, row0, n, threads=4))
    svc, paths = parity.http_events_key_tables()
    canon = {}
    for i, p in enumerate(paths):
        canon.setdefault(p, i)
    flags = np.zeros(64 * 1024, np.uint8)
    want = list(ref)[:50]
    for s, p in want:
        flags[svc.index(s) * 1024 + canon[p]] = 1
    counts, sums, voff, vals = parity.c2_truth(SEED, row0, n, flags, threads=4)
    assert int(counts.sum()) == sum(len(v) for v in ref.values())
    assert int((counts > 0).sum()) == len(ref)
    for (s, p), v in ref.items():
        g = svc.index(s) * 1024 + canon[p]
        assert counts[g] == len(v)
        assert sums[g] == int(round(sum(x * 1e6 for x in v)))
    for s, p in want:  # collected values: the group's values in row order, bit-exact
        g = svc.index(s) * 1024 + canon[p]
        np.testing.assert_array_equal(vals[voff[g]:voff[g] + counts[g]], np.array(ref[(s, p)]))


def test_duplicate_path_strings_are_one_group():
    """Two generator path indices can spell the same string; the truth merges them."""
    _, paths = parity.http_events_key_tables()
    assert len(set(paths)) < len(paths)  # the synthetic table does have such paths
