set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_attn_fused_gpu.py tests/test_model_gpu.py tests/test_kernels_gpu.py -q -k "fused or sampler or mmdit or frames_few or unaligned_wide" --timeout 120 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1; rc=$?; echo "tests rc=$rc"
[ $rc -le 1 ] || exit 1
bash tools/ab_libs.sh "e0 e3 e7 q32" 1 --bwd-only --windows none --iters 3 || exit 1
FRAMES=1536 WHICH=bwd PROG=attn_fwd_only.py OWLK_BWD_FUSED=2 bash tools/pmc_attn.sh || exit 1
python3 tools/pmc_read.py gpurun_out/pmc_bwd > gpurun_out/r4d_pmc_fused.txt 2>&1; echo "pmc rc=$?"
