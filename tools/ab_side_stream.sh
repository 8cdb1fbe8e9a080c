set -e
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  OWLK_BWD_SIDE_STREAM=0 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-profile > gpurun_out/abside_off_$i.log 2>&1
  timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-profile > gpurun_out/abside_on_$i.log 2>&1
done
