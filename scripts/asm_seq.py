"""Print the issue order of MFMA (M), LDS-DMA (D), barrier (|) and exp (e) instructions of one kernel in a
device assembly file (hipcc --cuda-device-only -S), and its register counts.

    python scripts/asm_seq.py <file.s> <mangled-kernel-name-prefix>
"""
import sys


def main():
    path, prefix = sys.argv[1], sys.argv[2]
    s = open(path).read().split("\n")
    i = next(k for k, line in enumerate(s) if line.startswith(prefix) and line.split(";")[0].rstrip().endswith(":"))
    name = s[i].split(";")[0].rstrip()[:-1]
    j = i
    while not s[j].startswith(".Lfunc_end"):
        j += 1
    seq = []
    for line in s[i:j]:
        t = line.strip().split()
        if not t:
            continue
        if "mfma" in t[0]:
            seq.append("M")
        elif t[0].startswith("buffer_load") and "lds" in line:
            seq.append("D")
        elif t[0] == "s_barrier":
            seq.append("|")
        elif t[0].startswith("v_exp"):
            seq.append("e")
    print("".join(seq))
    for line in s:
        if line.startswith(f"\t.set {name}.num_") and ("gpr" in line):
            print(line.strip())


if __name__ == "__main__":
    main()
