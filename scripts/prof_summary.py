"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel launch-duration distribution (us)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
d = defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].split("(")[0][:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if len(v) < 20:
        continue
    v2 = sorted(v)
    print(f"{k:48s} n={len(v):5d} min={v2[0]:7.2f} med={v2[len(v) // 2]:7.2f} p90={v2[9 * len(v) // 10]:7.2f} "
          f"share={100 * sum(v) / tot:5.1f}%")
