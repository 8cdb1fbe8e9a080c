"""Summarise rocprofv3 --pmc CSV output (per kernel, counters summed over dispatches)."""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        tot[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in tot.items():
    mf = d.get("SQ_INSTS_MFMA", 0)
    if not mf:
        continue
    W = d["SQ_WAVE_CYCLES"]
    cyc = d["GRBM_GUI_ACTIVE"] / 8
    print(k[:80])
    print("   VALU/MFMA %.2f  SALU/MFMA %.2f  LDS/MFMA %.2f" % (d["SQ_INSTS_VALU"] / mf, d["SQ_INSTS_SALU"] / mf,
                                                           d["SQ_INSTS_LDS"] / mf))
    print("   wave: active %.2f wait_any %.2f wait_inst %.2f (lds %.2f)" % (
        d["SQ_ACTIVE_INST_ANY"] / W, d["SQ_WAIT_ANY"] / W, d["SQ_WAIT_INST_ANY"] / W, d["SQ_WAIT_INST_LDS"] / W))
    print("   per SIMD: mfma util %.3f  valu issue %.3f  salu issue %.3f  waves/SIMD %.2f  lds util %.3f" % (
        d["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc, d["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / cyc,
        d["SQ_ACTIVE_INST_SCA"] * 4 / 1024 / cyc, W * 4 / 1024 / cyc, d["SQ_LDS_IDX_ACTIVE"] / 256 / cyc))
    if d.get("SQ_LDS_IDX_ACTIVE"):
        print("   lds bank conflict / active %.3f   trans VALU / VALU %.3f" % (
            d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_LDS_IDX_ACTIVE"], d.get("SQ_INSTS_VALU_TRANS_F", 0) / max(d["SQ_INSTS_VALU"], 1)))
