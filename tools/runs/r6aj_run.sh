# r6aj: docs-4 bench with packed documents back on the 8-wave backward (W4 default excludes them)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --docs 4 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r6aj_bench_docs4.log 2>&1 || exit 1
tail -1 gpurun_out/r6aj_bench_docs4.log | cut -c1-200
OWLK_BWD_FUSED_W4=1 timeout -k 10 500 python -u bench.py --docs 4 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r6aj_bench_docs4_w4.log 2>&1 || exit 1
tail -1 gpurun_out/r6aj_bench_docs4_w4.log | cut -c1-200
