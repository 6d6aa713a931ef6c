"""Turn FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_<workload>.json (HBM bytes per launch).

    python scripts/pmc_to_traffic.py <workload> <fetch_dir> <write_dir> kernel_regex=name [...] [src_sha=<hex>]

src_sha: the kernel-source digest of the tree the passes ran on (bench.py prints it; default: this tree's).

FETCH_SIZE and WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
coalesced streaming reads, global_load and LDS-DMA alike (MI355X_MICROARCH.md, HBM), so it is doubled;
WRITE_SIZE is exact for 16-B stores. Both count Infinity-Cache hits as well (memory-side requests).
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def per_kernel(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            key = r.get("Dispatch_Id", r.get("Correlation_Id"))
            per[key] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
        for k, v in per.items():
            vals[names[k]].append(v)
    return vals


def main():
    wl, fdir, wdir = sys.argv[1:4]
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "recommendation-system_amd"))
    from hvae.provenance import kernel_source_digest
    import subprocess
    head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes); FETCH_SIZE x2 (gfx950)",
           # bench.py reports this file's traffic only while the kernel sources hash to src_sha
           "src_sha": kernel_source_digest(), "measured_at_commit": head or None}
    for spec in sys.argv[4:]:
        rx, name = spec.split("=")
        if rx == "src_sha":
            out["src_sha"] = name
            continue
        fv = [v for k, vs in fetch.items() if re.search(rx, k) for v in vs]
        wv = [v for k, vs in write.items() if re.search(rx, k) for v in vs]
        if not fv or not wv:
            continue
        rd = 2 * 1024 * sum(fv) / len(fv)
        wr = 1024 * sum(wv) / len(wv)
        out[name] = {"kernel_regex": rx, "read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
                     "hbm_bytes_per_launch": round(rd + wr), "dispatches": [len(fv), len(wv)]}
    Path(f"profiles/pmc_{wl}.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
