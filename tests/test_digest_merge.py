"""The owner side of the multi-GPU exchange: the merged t-digest of one group built from the
contributions of several ranks (raw values of ranks that held <= 8 * delta of them, the single-
pass centroid list of the others), DigestMergeKernel through pxg_digest_merge, against the
restated tdigest batch add (oracle/tdigest.h merge_batch; math_sketches.h:38 merges digests).

Bars: the device restates the same arithmetic in the same order, so results agree to 1e-12
relative (device sin / asin may round differently from glibc in the last bit, which can move a
centroid boundary); and every quantile is inside the rank bound of the exact quantile of all the
values (parity above 8000 values is a rank bound)."""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_client as oc
from pixie_amd import _lib

pytestmark = pytest.mark.gpu
QS = [0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99]
PART_SHIFT = 48


def _device_merge(ctx, parts, arg_type=4):
    """parts: [("raw", values) | ("centroids", (means, weights))] in part order."""
    import torch
    vals, wts = [], []
    for p, (kind, payload) in enumerate(parts):
        if kind == "raw":
            v = np.asarray(payload)
            bits = v.astype(np.int64).view(np.uint64) if arg_type == 2 else v.astype(np.float64).view(np.uint64)
            vals.append(bits)
            wts.append(np.full(len(v), np.uint64(p << PART_SHIFT), np.uint64))
        else:
            m, w = payload
            vals.append(np.asarray(m, np.float64).view(np.uint64))
            wts.append((np.uint64(p << PART_SHIFT) | np.asarray(w, np.float64).astype(np.uint64)).astype(np.uint64))
    v = torch.from_numpy(np.concatenate(vals).view(np.int64)).cuda()
    w = torch.from_numpy(np.concatenate(wts).view(np.int64)).cuda()
    out = torch.zeros(7, dtype=torch.float64, device="cuda")
    _lib.check(_lib.load().pxg_digest_merge(ctx.h, C.c_void_p(v.data_ptr()), C.c_void_p(w.data_ptr()), len(v), arg_type,
                                            C.c_void_p(out.data_ptr())))
    return out.cpu().numpy().tolist()


def _rank(sorted_vals, x):
    n = len(sorted_vals)
    return (np.searchsorted(sorted_vals, x, "left") + np.searchsorted(sorted_vals, x, "right")) / 2 / n


def _check(ctx, parts, allvals, arg_type=4):
    dev = _device_merge(ctx, parts, arg_type)
    ref = oc.tdigest_batch_quantiles([(k, (np.asarray(p, np.float64) if k == "raw" else p)) for k, p in parts])
    allv = np.sort(np.asarray(allvals, np.float64)[~np.isnan(np.asarray(allvals, np.float64))])
    for q, d, r in zip(QS, dev, ref):
        assert abs(d - r) <= 1e-12 * max(1.0, abs(r)), (q, d, r)
        bound = 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / len(allv)
        assert abs(_rank(allv, d) - q) <= bound + 1e-3, (q, d)  # the digest itself vs the exact quantile
    return dev


def test_centroid_lists_only(ctx):
    rng = np.random.default_rng(1)
    samples = [rng.lognormal(1.0, 1.0, n) for n in (20_000, 50_000, 9_000)]
    parts = [("centroids", oc.tdigest_centroids(s)) for s in samples]
    _check(ctx, parts, np.concatenate(samples))


def test_raw_and_centroids_with_nan(ctx):
    rng = np.random.default_rng(2)
    big = [rng.lognormal(0.5, 0.8, n) for n in (30_000, 12_000)]
    raw1 = rng.lognormal(0.5, 0.8, 5000)
    raw2 = rng.lognormal(0.5, 0.8, 8000)
    raw2[::997] = np.nan
    parts = [("centroids", oc.tdigest_centroids(big[0])), ("raw", raw1), ("centroids", oc.tdigest_centroids(big[1])), ("raw", raw2)]
    _check(ctx, parts, np.concatenate(big + [raw1, raw2]))


def test_single_list_is_not_reprocessed(ctx):
    """One processed list of <= 2 * delta centroids and nothing else: the batch add does not
    process it again, so the quantiles are the list's own."""
    rng = np.random.default_rng(3)
    s = rng.normal(10, 3, 100_000)
    m, w = oc.tdigest_centroids(s)
    assert len(m) <= 2000
    dev = _check(ctx, [("centroids", (m, w))], s)
    own = oc.tdigest_batch_quantiles([("centroids", (m, w))])
    assert dev == pytest.approx(own, rel=1e-15, abs=0)


def test_integer_raw_values_and_ties(ctx):
    """INT64 arguments ride raw as integers; duplicated values across parts (ties)."""
    rng = np.random.default_rng(4)
    ints = [rng.integers(0, 500, n) for n in (7000, 6000, 8000)]
    big = rng.integers(0, 500, 40_000)
    parts = [("raw", ints[0]), ("centroids", oc.tdigest_centroids(big.astype(np.float64))), ("raw", ints[1]), ("raw", ints[2])]
    dev = _device_merge(ctx, parts, arg_type=2)
    ref = oc.tdigest_batch_quantiles([("raw", ints[0].astype(np.float64)), parts[1], ("raw", ints[1].astype(np.float64)),
                                      ("raw", ints[2].astype(np.float64))])
    allv = np.sort(np.concatenate(ints + [big]).astype(np.float64))
    for q, d, r in zip(QS, dev, ref):
        # ties: equal means from different parts may meet the greedy pass in another order
        bound = 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / len(allv)
        assert abs(_rank(allv, d) - _rank(allv, r)) <= bound, (q, d, r)


def test_many_parts(ctx):
    rng = np.random.default_rng(5)
    parts, allv = [], []
    for p in range(24):
        n = int(rng.integers(2000, 60_000))
        x = rng.lognormal(2.0, 1.2, n)
        allv.append(x)
        parts.append(("raw", x) if n <= 8000 else ("centroids", oc.tdigest_centroids(x)))
    _check(ctx, parts, np.concatenate(allv))
