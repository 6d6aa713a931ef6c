"""Stamp an SQ / GRBM counter pass of the d = 768 sweeps (scripts/gpu_r03_pmc_sq.sh) with the kernel-source digest
and derive the fractions DESIGN.md quotes.

    python scripts/pmc_sq_stamp.py <out.json> name=<counter dir> [...]

mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); wait fractions over SQ_WAVE_CYCLES;
LDS bank conflicts over SQ_LDS_IDX_ACTIVE.
"""
import csv
import glob
import json
import subprocess
import sys
from collections import defaultdict
from pathlib import Path


def means(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0], r["Counter_Name"], r.get("Dispatch_Id", r.get("Correlation_Id")))
            per[k] += float(r["Counter_Value"])
        for (kern, cn, _), v in per.items():
            acc[kern][cn].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"dispatches": len(next(iter(cs.values())))}
            for k, cs in acc.items()}


def main():
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "recommendation-system_amd"))
    from hvae.provenance import kernel_source_digest
    head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
    out = {"source": "rocprofv3 --pmc (one pass: 8 SQ + GRBM_GUI_ACTIVE), scripts/bench_decoder.py --nb 4096 "
                     "--N 1000000 --D 768", "src_sha": kernel_source_digest(), "measured_at_commit": head}
    for spec in sys.argv[2:]:
        name, d = spec.split("=")
        for kern, c in means(d).items():
            gui = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
            out[name] = {"kernel": kern, **{k: round(v, 1) for k, v in c.items()},
                         "mfma_busy": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * gui), 4) if gui else None,
                         "wait_any_frac": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
                         "wait_inst_any_frac": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4),
                         "lds_conflict_frac": round(c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1.0), 4)}
    Path(sys.argv[1]).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
