"""Summarise rocprofv3 PMC rocpd databases: per kernel, each counter summed over dispatches."""
import glob
import sqlite3
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
for f in sorted(glob.glob(sys.argv[1] + "/p*_results.db")):
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    kcol = "kernel_name" if "kernel_name" in cols else [x for x in cols if "name" in x][0]
    for k, n, v in c.execute(f"select {kcol}, counter_name, sum(value) from counters_collection group by {kcol}, counter_name"):
        tot[k][n] += v
for k, d in tot.items():
    if "attn" not in k and "gemm" not in k:
        continue
    print(k[:90])
    for n in sorted(d):
        print(f"   {n:32s} {d[n]:.4e}")
