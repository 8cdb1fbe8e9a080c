set -e
cd "$GRAFT_REPO_ROOT"
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for i in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/ne_base_$i.log 2>&1
  OWLK_LIB=$L/libowlk_noepi.so timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/ne_noepi_$i.log 2>&1
done
