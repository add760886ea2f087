"""Instruction histogram of one kernel in a hipcc -S listing, per basic block.

usage: isa_hist.py listing.s kernel_substring [--blocks]
Prints the mnemonic histogram of the kernel and of its largest basic blocks
(the accumulation loop body of k_msm_accum_seg is the largest by far).
"""
import re
import sys
from collections import Counter


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and name in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, label = [], [], "entry"
    for l in lines[start + 1:end]:
        s = l.strip()
        if re.match(r"^\.LBB\S*:", s):
            blocks.append((label, cur))
            label, cur = s[:-1], []
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        cur.append(s.split()[0])
    blocks.append((label, cur))
    tot = Counter(m for _, b in blocks for m in b)
    print("kernel", lines[start][:90], "instructions", sum(tot.values()))
    for lab, b in sorted(blocks, key=lambda x: -len(x[1]))[:4]:
        c = Counter(b)
        v = sum(n for m, n in c.items() if m.startswith("v_"))
        print(f"\nblock {lab}: {len(b)} instr, {v} VALU")
        for m, n in c.most_common(25):
            print(f"  {m:28s} {n}")


if __name__ == "__main__":
    main()
