"""Per-kernel mean of every PMC counter over dispatches in rocprofv3 counter_collection CSVs.

    python scripts/pmc_summary.py gpurun_out/pmc/dec1 [more dirs...]
"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0][:60], r["Counter_Name"])
            per[(k, r.get("Dispatch_Id", r.get("Correlation_Id", "")))] += float(r["Counter_Value"])
        for ((kern, cn), _), v in per.items():
            acc[kern][cn].append(v)
for kern, cs in acc.items():
    print(kern)
    for cn, vs in sorted(cs.items()):
        print(f"   {cn:28s} n={len(vs):4d} mean={sum(vs) / len(vs):.6g}")
