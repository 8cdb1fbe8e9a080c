"""gpurun_out/traffic/*_counter_collection.csv -> profiles/<tag>_traffic.json (per-launch HBM bytes).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of 16-B/lane
streaming reads (global_load / LDS-DMA), so it is doubled; WRITE_SIZE is exact for 16-B stores.
Both counters are in KiB."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob("gpurun_out/traffic/*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        mt = re.search(r"::(\w+?)_k\b", r["Kernel_Name"])  # attn_bwd_dkdv_k<64>(...) -> attn_bwd_dkdv
        name = mt.group(1) if mt else r["Kernel_Name"][:60]
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]) * 1024)
out = {}
for k, d in vals.items():
    n = len(d["FETCH_SIZE"])
    fetch = 2 * sum(d["FETCH_SIZE"]) / n
    write = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
    out[k] = {"launches": n, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
              "traffic_bytes_per_launch": fetch + write,
              "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on bench.py --steps 1; "
                        "FETCH_SIZE x2 (gfx950 16-B/lane read correction)"}
json.dump(out, open(f"profiles/{tag}_traffic.json", "w"), indent=1)
print(json.dumps(out, indent=1))
