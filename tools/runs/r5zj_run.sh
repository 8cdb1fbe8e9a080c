# r5zj: attention forward prologue -- Q rows loaded unconditionally and the ring's first tiles issued
# before Q is scaled (v1, OWLK_FWD_EARLY_RING) vs HEAD (v0: guarded Q loads, hipcc waits for the first
# rows before issuing the rest and the ring): forward GPU tests (v1), then interleaved x3 timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_attn_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5zj_tests.log 2>&1 && tail -1 gpurun_out/r5zj_tests.log || exit 1
for i in 1 2 3; do for v in v0 v1; do
  echo "== $v d64 $i"; OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/attn_bench.py --fwd-only --windows none,16,4 --iters 5 2>&1 | grep "  fwd " | cut -c1-40 || exit 1
  echo "== $v d128 $i"; OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/attn_bench.py --fwd-only --dim 128 --heads 20 --windows none,16 --iters 3 2>&1 | grep "  fwd " | cut -c1-40 || exit 1
done; done | tee gpurun_out/r5zj_ab.txt
