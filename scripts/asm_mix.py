"""Instruction mix of one kernel's innermost loop (the blocks LLVM marks "in Loop") in a device .s file.

    hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only csrc/x.hip -o x.s
    python scripts/asm_mix.py x.s <mangled-name-substring> [--all]

Prints per-block line / MFMA counts and the opcode histogram summed over the loop blocks (--all: whole kernel).
"""
import collections
import re
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    whole = "--all" in sys.argv
    lines = open(path).read().splitlines()
    i = next(k for k, ln in enumerate(lines) if sub in ln and ln.split(";")[0].rstrip().endswith(":")
             and not ln.startswith((".", "\t")))
    j = i
    while not lines[j].startswith(".Lfunc_end"):
        j += 1
    body = lines[i:j]
    idx = [k for k, ln in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", ln)] + [len(body)]
    tot = collections.Counter()
    for n in range(len(idx) - 1):
        seg = body[idx[n]:idx[n + 1]]
        if not whole and "Loop" not in body[idx[n]]:
            continue
        c = collections.Counter(ln.strip().split()[0] for ln in seg
                                if ln.strip() and not ln.strip().startswith((".", ";")))
        nm = sum(v for k, v in c.items() if k.startswith("v_mfma"))
        print(f"{body[idx[n]][:70]:70s} {len(seg):5d} lines  mfma {nm}")
        tot += c
    print()
    for k, v in tot.most_common(80):
        print(f"{v:5d} {k}")


if __name__ == "__main__":
    main()
