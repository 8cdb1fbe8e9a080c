"""Step-level MFMA utilisation from tools/pmc_step.sh output (rocprofv3 --pmc CSV + kernel trace).

Per kernel family and over the whole micro-step:
  MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs)
  clock      = (GRBM_GUI_ACTIVE / 8) / kernel duration              (shader GHz while it ran)
  vs 2.4 GHz = SQ_VALU_MFMA_BUSY_CYCLES / 1024 / (duration x 2.4 GHz): the matrix pipes' share of
               the peak-clock cycles, i.e. the MFMA fraction of the 2.5 PF/s dense bf16 peak that
               the executed MFMAs (recompute included) occupy.
"""
import csv
import glob
import re
import sys
from collections import defaultdict

d = sys.argv[1]
cnt = defaultdict(lambda: defaultdict(float))  # dispatch id -> counter -> value
name = {}
for f in glob.glob(d + "/**/p1_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        i = r["Dispatch_Id"]
        cnt[i][r["Counter_Name"]] += float(r["Counter_Value"])
        name[i] = r["Kernel_Name"]
dur = {}
for f in glob.glob(d + "/**/p1_kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])


def family(n):
    n = n.replace("(anonymous namespace)::", "")
    if "at::native" in n:
        return "ATen"
    n = re.sub(r"^void ", "", re.sub(r"\(.*", "", n))
    return re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", n)


fam = defaultdict(lambda: [0.0, 0.0, 0.0, 0])  # busy, gui, ns, launches
for i, c in cnt.items():
    if i not in dur:
        continue
    a = fam[family(name[i])]
    a[0] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    a[1] += c.get("GRBM_GUI_ACTIVE", 0.0)
    a[2] += dur[i]
    a[3] += 1
tot = [sum(v[k] for v in fam.values()) for k in range(4)]
print(f"{'kernel family':32s} {'launches':>8s} {'ms':>9s} {'MFMA busy':>9s} {'GHz':>6s} {'vs 2.4GHz':>9s}")
for k, (b, g, ns, n) in sorted(fam.items(), key=lambda kv: -kv[1][2]) + [("TOTAL (one micro-step)", tot)]:
    if ns <= 0 or g <= 0:
        continue
    print(f"{k[:32]:32s} {int(n):8d} {ns / 1e6:9.2f} {b / 1024 / (g / 8):9.3f} {g / 8 / ns:6.3f} "
          f"{b / 1024 / (ns * 2.4):9.3f}")
