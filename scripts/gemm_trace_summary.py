"""Per-shape kernel times of scripts/bench_gemm.py from a rocprofv3 kernel trace: the library's launches (hvae::,
the probe's hold kernel dropped) and torch.mm's (every other GEMM kernel) of each shape, in launch order.

    python scripts/gemm_trace_summary.py <run_kernel_trace.csv> [--reps 50] [--warmup 10]
"""
import argparse
import csv
import json

NAMES = ["fwd_heads", "fwd_proj_a", "fwd_proj_b", "bwd_dWb", "bwd_dp1", "bwd_dWa", "bwd_dz", "bwd_dWh", "bwd_dh"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    segs, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        if "k_probe_hold" in n:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "hvae::" in n:
            kind = "hvae"
        elif "Cijk" in n or "gemm" in n.lower():
            kind = "torch"
        else:
            continue
        if kind == "hvae" and (cur is None or cur["state"] == "torch"):
            cur = {"hvae": [], "torch": [], "state": "hvae", "kernel": n.split("(")[0]}
            segs.append(cur)
        if cur is None:
            continue
        if kind == "torch":
            cur["state"] = "torch"
        cur[kind].append(d)
    for name, s in zip(NAMES, segs):
        h = s["hvae"][a.warmup:]
        t = s["torch"][a.warmup:]  # torch.mm: one kernel per call on these shapes (a trailing one is the next shape's)
        print(json.dumps({"shape": name, "hvae_us": round(sum(h) / max(len(h), 1), 2), "hvae_launches": len(h),
                          "torch_us": round(sum(t[:a.reps]) / max(len(t[:a.reps]), 1), 2), "kernel": s["kernel"]}))


if __name__ == "__main__":
    main()
