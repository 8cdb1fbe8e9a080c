# r5zd: window-16 attention forward with 32- / 48-query waves (OWLK_FWD_NQ2W = 2 / 3: 128- / 192-query
# workgroups, 152 VGPRs -> three workgroups per CU at 32) against the 64-query production form; parity
# of the forward at both (GPU tests with the env set), interleaved x3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for nq in 2 3; do OWLK_FWD_NQ2W=$nq timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "fwd or attn" --timeout 120 --timeout-method thread > gpurun_out/r5zd_tests_$nq.log 2>&1 && tail -1 gpurun_out/r5zd_tests_$nq.log || exit 1; done
for i in 1 2 3; do for nq in 0 2 3; do
  echo "== nq2w $nq $i"; OWLK_FWD_NQ2W=$nq timeout -k 10 200 python -u tools/attn_bench.py --fwd-only --windows 16,4 --iters 5 2>&1 | grep "  fwd " | cut -c1-40 || exit 1
done; done | tee gpurun_out/r5zd_ab.txt
