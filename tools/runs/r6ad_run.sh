# r6ad: K^T fragment image (one ds_read_b128 per dQ k-step) in the one-wave-per-SIMD backward: bitwise
# check vs the 8-wave kernel, fused tests, A/B against HEAD (base)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
timeout -k 10 200 python -u tools/fused4_check.py > gpurun_out/r6ad_chk.log 2>&1 || { tail -5 gpurun_out/r6ad_chk.log; exit 1; }
tail -1 gpurun_out/r6ad_chk.log
timeout -k 10 600 python -u -m pytest tests/test_attn_fused_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ad_tests.log 2>&1 || { tail -20 gpurun_out/r6ad_tests.log; exit 1; }
tail -1 gpurun_out/r6ad_tests.log
cp owl-audio-exps_amd/owl_wms/_lib/libowlk.so owl-audio-exps_amd/owl_wms/_lib/libowlk_kf.so
FUSED_VARIANTS=129 bash tools/ab_libs.sh "base kf" 2 --bwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-60; done | tee gpurun_out/r6ad_ab.txt
