"""The host generator against the committed per-column hashes of its first 1M rows
(tests/golden/datagen_hash.json, written by tests/golden/make_datagen_hash.py)."""
import json
import os

from golden.make_datagen_hash import digests
from pixie_amd.device import datagen_http_events

HERE = os.path.dirname(os.path.abspath(__file__))


def test_host_generator_matches_committed_hashes():
    g = json.load(open(os.path.join(HERE, "golden", "datagen_hash.json")))
    cols = datagen_http_events(g["seed"], 0, g["rows"], n_pair_keys=g["n_pair_keys"], threads=8)
    assert digests(cols) == g["sha256"]
