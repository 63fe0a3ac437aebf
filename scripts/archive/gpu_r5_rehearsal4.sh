#!/usr/bin/env bash
# Four-rank rehearsal of the multi-GPU bench path on the one GPU (bench.py --rehearsal: gloo, every
# rank on cuda:0; the driver's own N = 2 / 4 / 8 runs use one GPU per rank over RCCL).
# Usage: gpurun --timeout 600 -- bash scripts/gpu_r5_rehearsal4.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_reh4}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29519 bench.py --gpus 4 --rehearsal --no-cpu-baseline > $O/bench_rehearsal4.log 2>&1 || { tail -8 $O/bench_rehearsal4.log; exit 1; }
tail -1 $O/bench_rehearsal4.log | cut -c1-400
