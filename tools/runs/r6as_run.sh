# r6as: other configs with the round-6 fusions: dit_v4_5B (AdaLN+gate fused on / off), mmdit_v2, docs-4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adaln or gate" > gpurun_out/r6as_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --config configs/dit_v4_5B.yml --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r6as_bench_5B.log 2>&1 || exit 1
OWLK_ADALN_GATE=0 timeout -k 10 500 python -u bench.py --config configs/dit_v4_5B.yml --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r6as_bench_5B_nogatefuse.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --config configs/mmdit_v2.yml --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r6as_bench_mmdit_v2.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --docs 4 --no-cpu-baseline --no-traffic > gpurun_out/r6as_bench_docs4.log 2>&1
