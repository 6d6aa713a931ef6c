"""Per-step timeline from a rocprofv3 kernel trace (run_kernel_trace.csv) of a train run: a step runs from one decoder
sweep's start to the next one's. Prints the median step length, the kernels of the median step (start / end relative
to its sweep's start, queue, name) and the per-step time of each kernel family over the steady-state steps.

    python scripts/step_timeline.py gpurun_out/x/run_kernel_trace.csv [--sweep k_dec] [--skip 20]
"""
import argparse
import csv
import statistics as st
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--sweep", default="k_dec", help="substring of the sweep kernel's name (k_dec2 / k_dec5 / k_dec_fp8)")
ap.add_argument("--skip", type=int, default=20, help="steps to skip at the start (capture, eager steps)")
args = ap.parse_args()
rows = list(csv.DictReader(open(args.trace)))
ks = []
for r in rows:
    name = r.get("Kernel_Name") or r.get("Name") or ""
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    ks.append((s, e, q, name))
ks.sort()
sweep_starts = [s for s, e, q, n in ks if args.sweep in n and "finalize" not in n]
steps = [(a, b) for a, b in zip(sweep_starts, sweep_starts[1:])]
steps = steps[args.skip:]
# drop the probe / eager tail: keep steps within 3x the median length
lens = [(b - a) / 1e3 for a, b in steps]
med = st.median(lens)
steady = [(a, b) for (a, b), L in zip(steps, lens) if L < 3 * med]
lens = [(b - a) / 1e3 for a, b in steady]
print(f"steps {len(steady)}  median {st.median(lens):.1f} us  mean {st.mean(lens):.1f}  min {min(lens):.1f}  "
      f"max {max(lens):.1f}")
# the median step's kernels
mi = min(range(len(steady)), key=lambda i: abs(lens[i] - st.median(lens)))
a, b = steady[mi]
print(f"median step ({lens[mi]:.1f} us):")
for s, e, q, n in ks:
    if a <= s < b:
        print(f"  {(s - a) / 1e3:9.2f} {(e - a) / 1e3:9.2f} q{q} {n[:70]}")
fam = defaultdict(float)
for a, b in steady:
    for s, e, q, n in ks:
        if a <= s < b:
            fam[n.split("(")[0][:60]] += (e - s) / 1e3
print("per step (us):")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
    print(f"  {v / len(steady):9.1f}  {k}")
