"""True min / max on the exchange (VERDICT r04 "digest merge"; math_sketches.h:38 Merge ->
tdigest merge(&other)).  A rank that holds more than 8 * delta values of a group ships the
centroid list of its single-pass digest (pxg_partial.hip XWriteGroupsKernel).  Past ~405K values
(delta = 1000: W * integratedQ(1) > 1) the list's first centroid holds several values, so its
mean is not the rank's true minimum (the greedy pass closes the last centroid on the maximum).

These tests show that shipping the true extremes cannot change a result:
  * the 7 quantiles read the digest's min_ / max_ only when the first / last centroid holds at
    least 2% of the weight (QuantileProcessed, oracle/tdigest.h), and no centroid a merge starts
    from is that heavy once W > 50;
  * so the merged quantiles with the ranks' true extremes carried into the owner's digest
    (oracle_tdigest_batch_quantiles_mm) equal, bit for bit, those with the extremes taken from
    the centroid means (the restated MergeProcessed), for per-rank groups of 420K-900K values;
  * the device merge (pxg_digest_merge, DigestMergeKernel) agrees with both and with the rank
    bound of the exact quantiles of all values.
A tiny digest (W <= 50) where the extremes do matter is included so the comparison is known to
be sensitive."""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_client as oc

QS = [0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99]
PART_SHIFT = 48


def _rank(sorted_vals, x):
    n = len(sorted_vals)
    return (np.searchsorted(sorted_vals, x, "left") + np.searchsorted(sorted_vals, x, "right")) / 2 / n


def _rank_samples(seed):
    rng = np.random.default_rng(seed)
    return [rng.lognormal(1.0, 1.1, n) for n in (420_000, 650_000, 900_000)]


def test_first_centroid_holds_several_values_past_405k():
    s = np.random.default_rng(7).lognormal(1.0, 1.1, 900_000)
    m, w = oc.tdigest_centroids(s)
    assert w[0] > 1 and m[0] > s.min()  # the first centroid's mean is not the minimum any more
    assert m[-1] <= s.max()  # (the greedy pass closes the last centroid on the largest value alone)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_carried_extremes_leave_the_quantiles_unchanged(seed):
    samples = _rank_samples(seed)
    parts = [("centroids", oc.tdigest_centroids(s)) for s in samples]
    ext = [(float(s.min()), float(s.max())) for s in samples]
    plain = oc.tdigest_batch_quantiles(parts)
    carried = oc.tdigest_batch_quantiles(parts, extremes=ext)
    assert np.array_equal(np.asarray(plain).view(np.uint64), np.asarray(carried).view(np.uint64))
    allv = np.sort(np.concatenate(samples))
    for q, v in zip(QS, carried):
        assert abs(_rank(allv, v) - q) <= 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / len(allv), (q, v)


def test_mixed_raw_and_lists_unchanged():
    rng = np.random.default_rng(11)
    big = [rng.normal(50, 9, n) for n in (500_000, 450_000)]
    raw = rng.normal(50, 9, 7000)
    parts = [("centroids", oc.tdigest_centroids(big[0])), ("raw", raw), ("centroids", oc.tdigest_centroids(big[1]))]
    ext = [(float(big[0].min()), float(big[0].max())), None, (float(big[1].min()), float(big[1].max()))]
    a = oc.tdigest_batch_quantiles(parts)
    b = oc.tdigest_batch_quantiles(parts, extremes=ext)
    assert np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))


def test_tiny_digest_does_read_the_extremes():
    """W = 4 in three centroids: p01 interpolates from min_ (the comparison above is sensitive)."""
    parts = [("centroids", (np.array([1.0, 5.0, 9.0]), np.array([2.0, 1.0, 1.0])))]
    a = oc.tdigest_batch_quantiles(parts)
    b = oc.tdigest_batch_quantiles(parts, extremes=[(0.0, 9.0)])
    assert a[0] != b[0]


@pytest.mark.gpu
def test_device_merge_of_large_rank_lists(ctx):
    import torch
    from pixie_amd import _lib
    samples = _rank_samples(5)
    parts = [oc.tdigest_centroids(s) for s in samples]
    vals = np.concatenate([np.asarray(m, np.float64).view(np.uint64) for m, _ in parts])
    wts = np.concatenate([(np.uint64(p << PART_SHIFT) | np.asarray(w, np.float64).astype(np.uint64)).astype(np.uint64)
                          for p, (_, w) in enumerate(parts)])
    v = torch.from_numpy(vals.view(np.int64)).cuda()
    w = torch.from_numpy(wts.view(np.int64)).cuda()
    out = torch.zeros(7, dtype=torch.float64, device="cuda")
    _lib.check(_lib.load().pxg_digest_merge(ctx.h, C.c_void_p(v.data_ptr()), C.c_void_p(w.data_ptr()), len(v), 4,
                                            C.c_void_p(out.data_ptr())))
    dev = out.cpu().numpy()
    ext = [(float(s.min()), float(s.max())) for s in samples]
    ref = oc.tdigest_batch_quantiles([("centroids", p) for p in parts], extremes=ext)
    allv = np.sort(np.concatenate(samples))
    for q, d, r in zip(QS, dev, ref):
        assert abs(d - r) <= 1e-12 * max(1.0, abs(r)), (q, d, r)
        assert abs(_rank(allv, d) - q) <= 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / len(allv), (q, d)
