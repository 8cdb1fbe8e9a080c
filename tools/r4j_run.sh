# fused backward: chain-group dequeue A/B (local hand-off; group 0 = all chains of a queue, 1..3) + HBM traffic
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
FUSED_VARIANTS="1,5,9,13" timeout -k 10 300 python -u tools/attn_bench.py --bwd-only --windows none --iters 3 > gpurun_out/r4j_ab.log 2>&1 || exit 1
grep "fused" gpurun_out/r4j_ab.log
for G in 0 1 3; do
  for C in FETCH_SIZE WRITE_SIZE; do
    OWLK_BWD_FUSED_GROUP=$G FRAMES=1536 timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex attn_bwd_fused -f csv -d gpurun_out/r4j_pmc_${G}_$C -o p -- python3 tools/attn_fwd_only.py bwd > gpurun_out/r4j_pmc_${G}_$C.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import csv, glob
for G in (0, 1, 3):
    out = {}
    for C in ("FETCH_SIZE", "WRITE_SIZE"):
        tot = 0.0
        for f in glob.glob(f"gpurun_out/r4j_pmc_{G}_{C}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == C and "attn_bwd_fused" in r["Kernel_Name"]:
                    tot += float(r["Counter_Value"]) * 1024
        out[C] = tot
    print(f"group {G}: fetch x2 {2 * out['FETCH_SIZE'] / 1e9:.2f} GB, write {out['WRITE_SIZE'] / 1e9:.2f} GB per launch")
PY
