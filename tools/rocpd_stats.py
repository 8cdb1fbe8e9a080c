"""rocprofv3 rocpd database -> kernel stats CSV (the --stats kernel_stats.csv columns).

    python tools/rocpd_stats.py gpurun_out/<dir>/run_results.db > profiles/<round>_kernel_stats.csv
"""
import sqlite3
import statistics
import sys
from collections import defaultdict


def main(path):
    c = sqlite3.connect(path)
    d = defaultdict(list)
    for name, dur in c.execute("select name, duration from kernels"):
        d[name].append(dur)
    tot = sum(sum(v) for v in d.values())
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"')
    for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        sd = statistics.pstdev(v) if len(v) > 1 else 0.0
        print(f'"{name}",{len(v)},{s},{s / len(v):.3f},{100.0 * s / tot:.2f},{min(v)},{max(v)},{sd:.3f}')


if __name__ == "__main__":
    main(sys.argv[1])
