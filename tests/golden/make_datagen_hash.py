"""Writes tests/golden/datagen_hash.json: SHA-256 per column of the first 1M synthetic
http_events rows (seed 20250117), so the host generator (and, through test_datagen_device.py,
the device generator) is pinned to the committed spec."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from pixie_amd.device import HTTP_EVENTS_SCHEMA, datagen_http_events  # noqa: E402


def column_digest(c) -> str:
    h = hashlib.sha256()
    if c.type == 5:
        h.update(c.offsets.tobytes())
        h.update(c.data[:int(c.offsets[-1])].tobytes())
    else:
        h.update(c.values.tobytes())
    return h.hexdigest()


def digests(cols):
    return {name: column_digest(c) for (name, _), c in zip(HTTP_EVENTS_SCHEMA, cols)}


if __name__ == "__main__":
    cols = datagen_http_events(20250117, 0, 1_000_000, n_pair_keys=10_000_000, threads=8)
    out = {"seed": 20250117, "rows": 1_000_000, "n_pair_keys": 10_000_000, "sha256": digests(cols)}
    with open(os.path.join(HERE, "datagen_hash.json"), "w") as f:
        json.dump(out, f, indent=1)
