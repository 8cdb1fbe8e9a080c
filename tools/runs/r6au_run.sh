# r6au: in-step A/B of the round-6 fusions (all on; QK-RoPE GEMM epilogue off; delta epilogue off; AdaLN+gate off)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-traffic > gpurun_out/r6au_all_$i.log 2>&1 || exit 1
  OWLK_GEMM_ROPE=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-traffic > gpurun_out/r6au_norope_$i.log 2>&1 || exit 1
  OWLK_GEMM_DELTA=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-traffic > gpurun_out/r6au_nodelta_$i.log 2>&1 || exit 1
  OWLK_ADALN_GATE=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-traffic > gpurun_out/r6au_nogate_$i.log 2>&1 || exit 1
done
