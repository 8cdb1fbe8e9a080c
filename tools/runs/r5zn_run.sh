# r5zn: single-pass backward with the dQ products on all 8 waves (OWLK_FUSED_DQ16=1, 16x16x32 quarter
# tiles; PF 2) against production (d0): fused parity tests on d16, then interleaved timing x3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_d16.so timeout -k 10 400 python -u -m pytest tests/test_attn_fused_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5zn_tests.log 2>&1; tail -3 gpurun_out/r5zn_tests.log
bash tools/ab_libs.sh "d0 d16" 3 --bwd-only --windows none,16,4 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "fused" $f | cut -c1-40; done | tee gpurun_out/r5zn_ab.txt
rm -f gpurun_out/libs_*.log
