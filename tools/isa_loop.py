"""Instruction histogram of each loop (backward-branch target block range) of one kernel in a
hipcc -save-temps .s file.

    python tools/isa_loop.py file.s name-substring
"""
import re
import sys
from collections import Counter


def main(path, pat):
    s = open(path).read()
    m = next(m for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M) if pat in m.group(1))
    end = s.find(".Lfunc_end", m.end())
    lines = [l.strip() for l in s[m.end():end].split("\n")]
    labels = {l[:-1].split()[0].rstrip(":"): i for i, l in enumerate(lines) if re.match(r"^\.LBB\S+:", l)}
    loops = []
    for i, l in enumerate(lines):
        mm = re.match(r"^s_c?branch\S*\s+(\.LBB\S+)", l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
            loops.append((labels[mm.group(1)], i))
    print(m.group(1))
    for a, b in loops:
        c = Counter()
        for l in lines[a:b + 1]:
            if not l or l.startswith(";") or l.endswith(":"):
                continue
            op = l.split()[0]
            cls = ("mfma" if "mfma" in op else "ds_read" if op.startswith("ds_read") else "ds_write" if op.startswith("ds_write")
                   else "glds" if "lds_dword" in op else "vmem" if op.startswith(("global_", "buffer_")) else
                   "waitcnt" if op.startswith("s_waitcnt") else "salu" if op.startswith("s_") else
                   "v_exp" if op.startswith("v_exp") else "valu" if op.startswith("v_") else op)
            c[cls] += 1
        print(f"  loop lines {a}-{b}: " + ", ".join(f"{k}={v}" for k, v in c.most_common()))
    ops = Counter(l.split()[0] for a, b in loops[-1:] for l in lines[a:b + 1] if l and not l.startswith(";") and not l.endswith(":") and l.startswith("v_"))
    print("  last loop VALU ops:", ", ".join(f"{k}={v}" for k, v in ops.most_common(30)))


if __name__ == "__main__":
    main(*sys.argv[1:])
