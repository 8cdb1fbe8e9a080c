"""Print every s_waitcnt containing vmcnt in one kernel of a .s file with a few lines of context
(to spot ring-draining vmcnt(0) inside a tile loop).

    python tools/isa_waits.py file.s name-substring
"""
import re
import sys


def main(path, pat):
    s = open(path).read()
    m = next(m for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M) if pat in m.group(1))
    end = s.find(".Lfunc_end", m.end())
    lines = [l.strip() for l in s[m.end():end].split("\n")]
    for i, l in enumerate(lines):
        if "vmcnt" in l:
            ctx = [x for x in lines[max(0, i - 4):i + 3] if x and not x.startswith(";;")]
            print(f"{i}: " + " | ".join(x[:48] for x in ctx))


if __name__ == "__main__":
    main(*sys.argv[1:])
