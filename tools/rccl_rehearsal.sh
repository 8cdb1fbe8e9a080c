# Multi-rank rehearsal of bench.py's RCCL path (GradReducer all-reduce, Muon all-gather, barrier /
# max-over-ranks timing) with 2 ranks sharing the box's one GPU, at a short sequence. RCCL refuses
# two ranks on one device, so the collectives run over gloo (on the same CUDA tensors).
set -e
cd "$GRAFT_REPO_ROOT"
export OWL_BENCH_SHARE_GPU=1
timeout -k 10 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --frames 128 --no-cpu-baseline --no-profile \
  > gpurun_out/rccl2.log 2>&1
