# r6p: steady-run statement (one asm loop over the uniform FULL tiles): bitwise check, fused tests, A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
timeout -k 10 200 python -u tools/fused4_check.py > gpurun_out/r6p_chk.log 2>&1 || exit 1
tail -1 gpurun_out/r6p_chk.log
timeout -k 10 600 python -u -m pytest tests/test_attn_fused_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6p_tests.log 2>&1 || exit 1
tail -1 gpurun_out/r6p_tests.log
cp owl-audio-exps_amd/owl_wms/_lib/libowlk.so owl-audio-exps_amd/owl_wms/_lib/libowlk_run.so
FUSED_VARIANTS=129 bash tools/ab_libs.sh "base run" 2 --bwd-only --windows none,16,4 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done | tee gpurun_out/r6p_ab.txt
