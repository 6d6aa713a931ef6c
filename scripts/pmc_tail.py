"""Per-kernel means of rocprofv3 counters (and kernel-trace durations) over each kernel's LAST n dispatches, so that
a run's warm-up dispatches do not dilute a steady-state reading.

    python scripts/pmc_tail.py <n> <counter or trace dirs...>
"""
import csv
import glob
import sys
from collections import defaultdict

n = int(sys.argv[1])
acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"].split("(")[0][:60], r["Counter_Name"], int(r.get("Dispatch_Id") or 0))
            per[key] += float(r["Counter_Value"])
        for (kern, cn, disp), v in sorted(per.items(), key=lambda kv: kv[0][2]):
            acc[kern][cn].append(v)
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            acc[r["Kernel_Name"].split("(")[0][:60]]["duration_us"].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for kern, cs in acc.items():
    print(kern)
    for cn, vs in sorted(cs.items()):
        t = vs[-n:]
        print(f"   {cn:28s} last {len(t):3d} of {len(vs):4d}: mean={sum(t) / len(t):.6g}")
