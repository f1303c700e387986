"""Compressed instruction sequence of a kernel's MFMA-heaviest basic block:
    python tools/isa_seq.py file.s mangled_name_substring
M mfma, r ds_read, w ds_write, L vector-memory load, v VALU, [..] waitcnt, |B| barrier."""
import re
import sys

s = open(sys.argv[1]).read()
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", s, re.M) if sys.argv[2] in m.group(1)]
for name in names:
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    blocks, cur = [], []
    for l in s[i:j].splitlines():
        if re.match(r"^\.LBB", l):
            blocks.append(cur)
            cur = [l]
        else:
            cur.append(l)
    blocks.append(cur)
    best = max(blocks, key=lambda b: sum("mfma" in x for x in b))
    seq = []
    for l in best:
        t = l.strip().split()
        if not t:
            continue
        op = t[0]
        if "mfma" in op:
            seq.append("M")
        elif op.startswith("ds_read"):
            seq.append("r")
        elif op.startswith("ds_write"):
            seq.append("w")
        elif op.startswith("s_waitcnt"):
            seq.append("[" + l.strip()[10:] + "]")
        elif op.startswith(("buffer_load", "global_load")):
            seq.append("L")
        elif op.startswith("s_barrier"):
            seq.append("|B|")
        elif op.startswith("v_"):
            seq.append("v")
        elif "scratch" in op:
            seq.append("S")
    print(name, len(best), "instructions,", sum(c == "M" for c in seq), "MFMA")
    print("".join(seq))
