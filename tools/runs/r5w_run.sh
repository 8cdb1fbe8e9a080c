# r5w: short-K small-tile fp32 GEMMs as one round of 256^2 split-K with a workspace (k2) against k1
# (cond gradient only) and k0 (before both): GEMM / block / model GPU tests of k2, timing, step bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
OWLK_LIB=$L/libowlk_k2.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "gemm or cond or block or model or muon or train" --timeout 200 --timeout-method thread \
  > gpurun_out/r5w_tests.log 2>&1 || { tail -30 gpurun_out/r5w_tests.log; exit 1; }
tail -1 gpurun_out/r5w_tests.log
for i in 1 2; do for v in k0 k1 k2; do
  echo "== $v $i"; OWLK_LIB=$L/libowlk_$v.so timeout -k 10 200 python -u tools/gemm_epi_bench.py 2>&1 | grep "modulation\|cond grad\|mod wgrad" || exit 1
done; done | tee gpurun_out/r5w_ab.txt
for i in 1 2; do for v in k0 k2; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-traffic \
    > gpurun_out/r5w_bench_${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5w_bench_${v}_$i.log; exit 1; }
  echo "$v $i $(grep -o '"value": [0-9.]*' gpurun_out/r5w_bench_${v}_$i.log)"
done; done | tee -a gpurun_out/r5w_ab.txt
