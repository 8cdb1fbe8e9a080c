# r5zb: asm transposed reads in the attention forward / D = 128 backward (no vmcnt(0) ring drain at
# the first ds_read_b64_tr_b16 of each tile): kernel GPU tests on the new build, then v0 (HEAD) vs v1
# interleaved: D = 64 forward (global, window 16) and D = 128 forward + dK/dV + dQ
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/libs_*.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5zb_tests.log 2>&1 && tail -2 gpurun_out/r5zb_tests.log || exit 1
bash tools/ab_libs.sh "v0 v1" 3 --fwd-only --windows none,16 --iters 3 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "  fwd " $f | cut -c1-40; done | tee gpurun_out/r5zb_ab.txt
rm -f gpurun_out/libs_*.log
bash tools/ab_libs.sh "v0 v1" 2 --dim 128 --heads 20 --windows none --iters 2 || exit 1
for f in gpurun_out/libs_*.log; do echo "== $f"; grep -h "  fwd \|dkdv\|  dq " $f | cut -c1-40; done | tee -a gpurun_out/r5zb_ab.txt
