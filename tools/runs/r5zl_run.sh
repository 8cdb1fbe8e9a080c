# r5zl: final round-5 library on the other bench configs: mmdit_v2 and dit_v4 with 4 packed documents
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --config configs/mmdit_v2.yml --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r5zl_bench_mmdit_v2.log 2>&1 && tail -1 gpurun_out/r5zl_bench_mmdit_v2.log | cut -c1-200 &&
timeout -k 10 600 python -u bench.py --docs 4 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r5zl_bench_docs4.log 2>&1 && tail -1 gpurun_out/r5zl_bench_docs4.log | cut -c1-200
