# fused backward: per-item overhead (dequeue / prologue / epilogue) beside the step phases, global and window 16 / 4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_pf.so FUSED_VARIANTS="5" timeout -k 10 300 python -u tools/attn_bench.py --bwd-only --windows 16,4,none --iters 2 > gpurun_out/r4af_prof.log 2>&1 || exit 1
grep "window\|fused" gpurun_out/r4af_prof.log

