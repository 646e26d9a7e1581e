"""Parity at the north_star configuration (BASELINE.json north_star: 1B-row filter +
group-by(service, req_path) with count/mean/quantiles on ONE GPU), the shape the bench's n1 leg
times: 32768-row consume tiles, selection with 4096 bins for groups of up to ~6.9M values.
Checked against the generator's ground truth (tests/parity.py::check_c2_against_truth): keys and
counts bit-exact, means 1e-6, quantiles of the 20 largest groups within the rank bound of the
oracle t-digest fed row order, 200 seeded <= 8000-value groups within 4 ULP of it.
Reference semantics: agg_node.cc:303-349, math_sketches.h:36-54."""
import pytest

import parity
from pixie_amd import plans as P
from pixie_amd.device import Table
from pixie_amd.host_engine import plan_agg

pytestmark = pytest.mark.gpu
SEED = 20250117


@pytest.mark.parametrize("n", [1_000_000_000])
def test_c2_at_1b_rows_matches_generator_truth(ctx, n):
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(SEED, 0, n, 10_000_000)
    a = plan_agg(ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)
    try:
        a.reset()
        a.consume(t)
        g = a.finalize()
        assert a.info()["big_sort_groups"] == 0  # every big group served by selection
        rep = parity.check_c2_against_truth(a.result(), SEED, 0, n, threads=16)
    finally:
        a.close()
        t.close()
    print(rep)
    assert "groups_ref" in rep, rep
    assert g == rep["groups_ref"]
    assert rep["selected_rows_dev"] == rep["selected_rows_ref"]
    assert rep["ok"], rep
    assert rep["quantiles"]["largest_group"] > 5_000_000


@pytest.mark.parametrize("n", [3 * (1 << 24) + 4100])
def test_c2_across_full_chunks_matches_generator_truth(ctx, n):
    """Three full 2^24-row chunks and a partial one: the streamed consume's windows cross chunk
    boundaries inside a workgroup's run (its offsets run ahead of its payloads there)."""
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(SEED, 0, n, 10_000_000)
    a = plan_agg(ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)
    try:
        a.reset()
        a.consume(t)
        g = a.finalize()
        rep = parity.check_c2_against_truth(a.result(), SEED, 0, n, threads=16)
    finally:
        a.close()
        t.close()
    assert "groups_ref" in rep, rep
    assert g == rep["groups_ref"]
    assert rep["selected_rows_dev"] == rep["selected_rows_ref"]
    assert rep["ok"], rep
