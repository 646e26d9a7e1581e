"""carnot_csv: the `carnot_executable` harness (src/carnot/carnot_executable.cc:109-300) over the
device engine.  A CSV with a type row and a name row is cut into RowBatches of --rowbatch_size,
run through a binary planpb.Plan as table `csv_table`, and the first output table is written as
CSV without a header (ints as integers, FLOAT64 "%.2f", BOOLEAN true/false, STRING raw).  The
expected file is the oracle's result over the same values parsed the reference's way (std::stoi
for INT64/TIME64NS, std::stof -> float32 for FLOAT64, `== "true"` for BOOLEAN), formatted the same
way.  Row order of an aggregate is the hash map's, so lines compare as multisets."""
import os
import subprocess

import numpy as np
import pytest

import oracle_client as oc
from pixie_amd import plans as P
from pixie_amd.device import Column

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "pixie_amd", "lib", "carnot_csv")
B, I, F, S, T = P.BOOLEAN, P.INT64, P.FLOAT64, P.STRING, P.TIME64NS
TYPE_NAMES = {B: "boolean", I: "int64", F: "float64", S: "string", T: "time64ns", P.UINT128: "uint128"}


def _quote(v):
    return '"' + v.replace('"', '""') + '"' if ("," in v or '"' in v) else v


def _write_csv(path, types, names, cols):
    with open(path, "w") as f:
        f.write(",".join(TYPE_NAMES[t] for t in types) + "\n")
        f.write(",".join(names) + "\n")
        n = len(cols[0])
        for r in range(n):
            f.write(",".join(_quote(c[r]) for c in cols) + "\n")


def _fmt(col, r):
    if col.type == F:
        return "%.2f" % col.values[r]
    if col.type == B:
        return "true" if col.values[r] else "false"
    if col.type == S:
        return bytes(col.data[col.offsets[r]:col.offsets[r + 1]]).decode()
    if col.type == P.UINT128:
        return f"{int(col.values[r, 1])}:{int(col.values[r, 0])}"
    return str(int(col.values[r]))


def _expected_lines(plan, types, names, text_cols):
    parsed = []
    for t, c in zip(types, text_cols):
        if t in (I, T):
            parsed.append(Column(t, values=np.array([int(x) for x in c], dtype=np.int64)))
        elif t == F:
            parsed.append(Column(t, values=np.array([float(x) for x in c], dtype=np.float32).astype(np.float64)))
        elif t == B:
            parsed.append(Column(t, values=np.array([x == "true" for x in c], dtype=np.uint8)))
        else:
            parsed.append(Column.from_values(S, c))
    out = oc.execute_plan(plan, {"csv_table": {"types": types, "names": names, "batches": [parsed]}})
    first = next(iter(out.values()))
    lines = []
    for b in first:
        for r in range(b["rows"]):
            lines.append(",".join(_fmt(c, r) for c in b["cols"]))
    return lines


def _run(tmp_path, plan, types, names, text_cols, rb=100):
    csv = tmp_path / "in.csv"
    pb = tmp_path / "plan.pb"
    out = tmp_path / "out.csv"
    _write_csv(csv, types, names, text_cols)
    pb.write_bytes(plan.SerializeToString())
    r = subprocess.run([EXE, f"--input_file={csv}", f"--output_file={out}", f"--plan_file={pb}", f"--rowbatch_size={rb}"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    return out.read_text().splitlines(), r.stderr


def _close_lines(got, want, float_cols):
    """Keys / counts / strings identical; a "%.2f" mean may sit on a rounding edge where the
    device's and the oracle's sums differ in the last bits, so those fields agree within 0.01."""
    assert len(got) == len(want)
    key = lambda line: [f for i, f in enumerate(line.split(",")) if i not in float_cols]
    g = sorted(got, key=key)
    w = sorted(want, key=key)
    for a, b in zip(g, w):
        fa, fb = a.split(","), b.split(",")
        for i, (x, y) in enumerate(zip(fa, fb)):
            if i in float_cols:
                assert abs(float(x) - float(y)) <= 0.0100001, (a, b)
            else:
                assert x == y, (a, b)


def _dataset(n, seed=5):
    rng = np.random.default_rng(seed)
    svc = [f"svc-{x}" for x in rng.integers(0, 37, n)]
    lat = [str(int(x)) for x in rng.integers(-2_000_000_000, 2_000_000_000, n)]
    tm = [str(int(x)) for x in rng.integers(0, 2_147_483_647, n)]
    ok = ["true" if x else ("false" if y else "TRUE") for x, y in zip(rng.random(n) < 0.6, rng.random(n) < 0.5)]
    ratio = [repr(float(x)) for x in rng.normal(0, 1000, n)]
    path = [f'/a,"{x}"' if x % 7 == 0 else f"/p{x}" for x in rng.integers(0, 50, n)]  # written quoted
    return [T, S, S, I, B, F], ["time_", "service", "req_path", "latency", "ok", "ratio"], [tm, svc, path, lat, ok, ratio]


def test_harness_rejects_uint128_and_bad_usage(tmp_path):
    """Host-side checks that run before any device work (CPU)."""
    if not os.path.exists(EXE):
        pytest.skip("carnot_csv not built")
    (tmp_path / "u.csv").write_text("int64,uint128\na,b\n1,2\n")
    (tmp_path / "p.pb").write_bytes(b"")
    r = subprocess.run([EXE, f"--input_file={tmp_path / 'u.csv'}", f"--output_file={tmp_path / 'o.csv'}",
                        f"--plan_file={tmp_path / 'p.pb'}"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "uint128" in r.stderr
    (tmp_path / "t.csv").write_text("int32\na\n1\n")
    r = subprocess.run([EXE, f"--input_file={tmp_path / 't.csv'}", f"--output_file={tmp_path / 'o.csv'}",
                        f"--plan_file={tmp_path / 'p.pb'}"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Could not recognize type" in r.stderr
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2


@pytest.mark.gpu
@pytest.mark.parametrize("n,rb", [(1, 100), (2_345, 100), (120_000, 1024)])
def test_c1_groupby_count_mean(tmp_path, n, rb):
    """C1 over the CSV table: groupby(service).agg(count, mean(latency))."""
    types, names, cols = _dataset(n)
    plan = P.linear_plan([P.source_op("csv_table", types, names, [1, 3]),
                          P.agg_op([0], [P.agg_expr("count", [P.col(1)], [I]), P.agg_expr("mean", [P.col(1)], [I], fid=1)],
                                   ["service"], ["count", "mean"]),
                          P.sink_op("output")])
    got, err = _run(tmp_path, plan, types, names, cols, rb)
    want = _expected_lines(plan, types, names, cols)
    _close_lines(got, want, {2})
    assert '"exec_s"' in err


@pytest.mark.gpu
def test_filter_map_bool_float_string_output(tmp_path):
    """Filter(ok) -> Map(req_path, ratio * 2, latency, time_, ok): every output type, quoted CSV
    fields, std::stof rounding and "TRUE" read as false."""
    types, names, cols = _dataset(5_000, seed=9)
    plan = P.linear_plan([P.source_op("csv_table", types, names, [0, 2, 3, 4, 5]),
                          P.filter_op(P.col(3), [0, 1, 2, 3, 4]),
                          P.map_op([P.col(1), P.func("multiply", [P.col(4), P.const(F, 2.0)], [F, F]), P.col(2), P.col(0), P.col(3)],
                                   ["req_path", "r2", "latency", "time_", "ok"]),
                          P.sink_op("output")])
    got, _ = _run(tmp_path, plan, types, names, cols, 333)
    want = _expected_lines(plan, types, names, cols)
    assert got == want  # no aggregate: row order is the input order, every field exact
