#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from rocprofv3 `--pmc` CSV passes.

Usage: pmc_summary.py --kernel AggConsumeKernel --rows N --fetch DIR --write DIR --out JSON

FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit one TCC pass,
MI355X_MICROARCH.md §rocprofv3 PMC slots).  Both are in KiB.  On gfx950 FETCH_SIZE reports
half the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM), so the read side is
doubled: hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, averaged over the kernel's
launches.  The result is written as the JSON bench.py reads into roofline.traffic.
"""
import argparse
import csv
import glob
import json
import os
import re


def counter_values(d, kernel, counter):
    vals = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if re.search(kernel, row.get("Kernel_Name", "")) and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} under {d}")
    return vals


def counter_avg(d, kernel, counter):
    vals = counter_values(d, kernel, counter)
    return sum(vals) / len(vals), len(vals)


def counter_per_step(d, kernel, counter, steps):
    """Sum over every matching launch / steps: a step may launch the kernel more than once
    (the consume's probe-record prefix launch + the rest of the range)."""
    vals = counter_values(d, kernel, counter)
    return sum(vals) / steps, len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default=r"AggConsume(Fast)?Kernel", help="regex on the kernel name")
    ap.add_argument("--name", default="agg_consume")
    ap.add_argument("--rows", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=0,
                    help="consume steps in the run: report bytes per step (every matching launch of a step summed: the "
                         "probe-record prefix launch + the main launch) instead of per launch")
    a = ap.parse_args()
    if a.steps > 0:
        fetch_kib, nf = counter_per_step(a.fetch, a.kernel, "FETCH_SIZE", a.steps)
        write_kib, nw = counter_per_step(a.write, a.kernel, "WRITE_SIZE", a.steps)
    else:
        fetch_kib, nf = counter_avg(a.fetch, a.kernel, "FETCH_SIZE")
        write_kib, nw = counter_avg(a.write, a.kernel, "WRITE_SIZE")
    res = {
        "kernel": a.name,
        "kernel_symbol": a.kernel,
        "rows_per_gpu": a.rows,
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib": write_kib,
        "launches": [nf, nw],
        "per": f"consume step ({a.steps} steps)" if a.steps > 0 else "launch",
        "hbm_read_bytes_per_launch": 2 * fetch_kib * 1024,
        "hbm_write_bytes_per_launch": write_kib * 1024,
        "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
        "correction": "gfx950: FETCH_SIZE doubled (MI355X_MICROARCH.md §HBM); KiB -> bytes",
    }
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
