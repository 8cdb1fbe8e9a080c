# MFMA busy cycles and shader clock of every kernel in one dit_v4 micro-step (one --pmc pass,
# kernel trace for the durations).  Usage (on the box): bash tools/pmc_step.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-pmcstep}
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -f csv \
  -d $R/gpurun_out/$TAG -o p1 -- python3 $R/bench.py --microsteps 1 > $R/gpurun_out/${TAG}.log 2>&1
python3 $R/tools/pmc_step_summary.py $R/gpurun_out/$TAG > $R/gpurun_out/${TAG}_summary.txt 2>&1
