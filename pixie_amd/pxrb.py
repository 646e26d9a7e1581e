"""PXRB: the result serialisation shared by the C++ host engine (pixie_amd/host) and the
test oracle: per sink, its RowBatches with eow/eos flags and Arrow-layout columns."""
from __future__ import annotations

import struct

import numpy as np

BOOLEAN, INT64, UINT128, FLOAT64, STRING, TIME64NS = 1, 2, 3, 4, 5, 6


def parse_pxrb(buf: bytes):
    """PXRB -> {sink name: [ {'rows': n, 'eow': b, 'eos': b, 'cols': [Column...]} ]}."""
    from pixie_amd.device import Column
    off = 0

    def take(fmt):
        nonlocal off
        v = struct.unpack_from(fmt, buf, off)
        off += struct.calcsize(fmt)
        return v

    magic, ntables = take("<II")
    assert magic == 0x42525850
    out = {}
    for _ in range(ntables):
        (nl,) = take("<I")
        name = buf[off:off + nl].decode()
        off += nl
        (nb,) = take("<I")
        batches = []
        for _ in range(nb):
            nrows, eow, eos, _pad, ncols = take("<qBBHI")
            cols = []
            for _ in range(ncols):
                (t,) = take("<i")
                if t == STRING:
                    offs = np.frombuffer(buf, dtype=np.int32, count=nrows + 1, offset=off).copy()
                    off += 4 * (nrows + 1)
                    nbytes = int(offs[-1])
                    data = np.frombuffer(buf, dtype=np.uint8, count=nbytes, offset=off).copy()
                    off += nbytes
                    cols.append(Column(STRING, offsets=offs, data=np.concatenate([data, np.zeros(16, np.uint8)])))
                elif t == UINT128:
                    v = np.frombuffer(buf, dtype=np.uint64, count=2 * nrows, offset=off).copy().reshape(nrows, 2)
                    off += 16 * nrows
                    cols.append(Column(UINT128, values=v))
                elif t == BOOLEAN:
                    v = np.frombuffer(buf, dtype=np.uint8, count=nrows, offset=off).copy()
                    off += nrows
                    cols.append(Column(BOOLEAN, values=v))
                else:
                    dt = np.float64 if t == FLOAT64 else np.int64
                    v = np.frombuffer(buf, dtype=dt, count=nrows, offset=off).copy()
                    off += 8 * nrows
                    cols.append(Column(t, values=v))
            batches.append({"rows": nrows, "eow": bool(eow), "eos": bool(eos), "cols": cols})
        out[name] = batches
    return out
