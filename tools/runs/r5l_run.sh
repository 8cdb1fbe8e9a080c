# r5l: whole-step A/B of the library built with the AMDGPU register-pressure trackers + max-ILP
# scheduling strategy (s4) against the default build (s0): bench.py 2 timed steps, interleaved x2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/owl-audio-exps_amd/owl_wms/_lib
for i in 1 2; do for v in s0 s4; do
  OWLK_LIB=$L/libowlk_$v.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-traffic \
    > gpurun_out/r5l_bench_${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5l_bench_${v}_$i.log; exit 1; }
  echo "$v $i $(grep -o '"value": [0-9.]*' gpurun_out/r5l_bench_${v}_$i.log)"
done; done | tee gpurun_out/r5l_ab.txt
