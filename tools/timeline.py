"""Print the kernel timeline after the last agg_consume kernel of a rocprofv3 kernel trace."""
import csv
import sys

path = sys.argv[1]
rows = []
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pxg::", "")[:30]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", r.get("Stream_Id", ""))))
rows.sort()
idx = [i for i, r in enumerate(rows) if "AggConsumeFast" in r[2]]
i0 = idx[-2] if len(idx) > 1 else idx[-1]
i1 = idx[-1]
t0 = rows[i0][1]
for s, e, n, q in rows[i0:i1 + 1]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}us q{q} {n}")
