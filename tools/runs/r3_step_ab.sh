# Step-level interleaved A/B on one box: round-3 attention tile changes off (OWLK_DQ_NT=2 OWLK_FWD_KT128=0
# OWLK_FWD_NQ3=0 OWLK_BWD_QT2_MIN=1000000000) vs the defaults.  usage: bash tools/runs/r3_step_ab.sh [config]
set -e
cd "$GRAFT_REPO_ROOT"
CFG=${1:-configs/dit_v4.yml}
T=$(basename $CFG .yml)
for r in 1 2; do
  OWLK_DQ_NT=2 OWLK_FWD_KT128=0 OWLK_FWD_NQ3=0 OWLK_BWD_QT2_MIN=1000000000 timeout -k 10 400 python -u bench.py --config $CFG \
    --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/stepab_${T}_off_$r.log 2>&1
  timeout -k 10 400 python -u bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --no-traffic \
    > gpurun_out/stepab_${T}_on_$r.log 2>&1
done
