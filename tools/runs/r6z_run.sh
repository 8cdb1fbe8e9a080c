# r6z: one-wave-per-SIMD forward: bitwise vs attn_fwd16_k + oracle tests, then timing (fwd, windows none/16)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attn_fwd4_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r6z_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r6z_tests.log
[ $rc -eq 0 ] || exit 1
OWLK_FWD4=0 timeout -k 10 200 python -u tools/attn_bench.py --fwd-only --windows none,16 --iters 3 > gpurun_out/r6z_fwd16.log 2>&1 || exit 1
OWLK_FWD4=1 timeout -k 10 200 python -u tools/attn_bench.py --fwd-only --windows none,16 --iters 3 > gpurun_out/r6z_fwd4.log 2>&1 || exit 1
grep -h "fwd " gpurun_out/r6z_fwd16.log gpurun_out/r6z_fwd4.log | cut -c1-70
