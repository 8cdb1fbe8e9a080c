# r5i: GEMM epilogues -- bit-exact outputs of g1 (paired rounding) and g3 (from registers, plain
# stores) against g0; interleaved timing of g0 g1 g3 and of the main loops alone (n0 / n2: no
# epilogue, A.B^T vs B.A^T operand order)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/r5i
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for v in g0 g1 g3; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py --save /tmp/r5i/$v.pt --iters 3 \
    > gpurun_out/r5i_save_$v.log 2>&1 || { tail -20 gpurun_out/r5i_save_$v.log; exit 1; }
done
{ python tools/gemm_epi_bench.py --compare /tmp/r5i/g0.pt /tmp/r5i/g1.pt; python tools/gemm_epi_bench.py --compare /tmp/r5i/g0.pt /tmp/r5i/g3.pt; } | tee gpurun_out/r5i_epi_compare.txt
for i in 1 2; do for v in g0 g1 g3 n0 n2; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u tools/gemm_epi_bench.py > gpurun_out/r5i_gemm_${v}_$i.log 2>&1 || exit 1
done; done
for f in gpurun_out/r5i_gemm_*.log; do echo "== $f"; grep "TF/s" $f; done | tee gpurun_out/r5i_gemm_ab.txt
