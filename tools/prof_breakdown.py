"""Per-kernel time of the LAST micro-step in a rocprofv3 --kernel-trace database (bench.py --microsteps K).

usage: python tools/prof_breakdown.py <run_results.db> [top]"""
import collections
import re
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
con = sqlite3.connect(db)
rows = list(con.execute("select name, start, end from kernels order by start"))
first = [i for i, r in enumerate(rows) if "flow_noise" in r[0]]
seg = rows[first[-1]:] if first else rows
cnt, tim = collections.Counter(), collections.Counter()
for n, s, e in seg:
    k = re.sub(r"^void ", "", n[:160]).replace("(anonymous namespace)::", "")
    cnt[k] += 1
    tim[k] += e - s
tot = sum(tim.values())
print(f"last micro-step: {len(seg)} launches, {tot / 1e6:.2f} ms kernel time")
for k, v in sorted(tim.items(), key=lambda x: -x[1])[:top]:
    print(f"{v / 1e6:9.2f} ms {100 * v / tot:5.1f}% {cnt[k]:5d}  {k[:110]}")
