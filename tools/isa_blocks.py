"""Basic-block table (instructions, VALU, v_mad_u64_u32, branch targets) of one
kernel in a hipcc -S listing.  usage: isa_blocks.py listing.s kernel_substring"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sys.argv[2] in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
lab, n, valu, mads, br = "entry", 0, 0, 0, []


def emit():
    print(f"{lab:12s} n={n:5d} valu={valu:5d} mads={mads:5d} br={' '.join(br)}")


for l in lines[start + 1:end]:
    s = l.strip()
    m = re.match(r"^(\.LBB\S*):", s)
    if m:
        emit()
        lab, n, valu, mads, br = m.group(1), 0, 0, 0, []
        continue
    if not s or s.startswith((";", ".", "//")):
        continue
    op = s.split()[0]
    n += 1
    valu += op.startswith("v_")
    mads += op == "v_mad_u64_u32"
    if op.startswith("s_cbranch") or op == "s_branch":
        br.append(op.replace("s_cbranch_", "") + ":" + s.split()[-1])
emit()
