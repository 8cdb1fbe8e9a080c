# r6k: lean per-step scalar work (per-item thresholds, incremental pointers): bitwise check, timing, profile
# statement: bitwise check against the 8-wave kernel, timing, phase profile
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/fused4_check.py --time > gpurun_out/r6k_check.log 2>&1 || exit 1
OWLK_LIB=$PWD/owl-audio-exps_amd/owl_wms/_lib/libowlk_prof.so FUSED_VARIANTS=129 timeout -k 10 200 python -u tools/attn_bench.py --bwd-only --windows none,16 --iters 2 > gpurun_out/r6k_prof.log 2>&1
