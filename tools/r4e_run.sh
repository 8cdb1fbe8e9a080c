set -o pipefail
cd $GRAFT_REPO_ROOT
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_q32b.so timeout -k 10 300 python -u -m pytest tests/test_attn_fused_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4e_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/ab_libs.sh "q32 q32b" 2 --bwd-only --windows none --iters 3 || exit 1
grep -h "fused\|split\|dkdv\|dq" gpurun_out/libs_*.log | head -40
