#!/usr/bin/env bash
# Round-5 closing evidence at HEAD: GPU suite, smoke, bench line with the CPU leg, rocprofv3 passes
# (scripts/gpu_r5_final.sh), a two-rank rehearsal of the multi-GPU bench path on the one GPU (gloo,
# both ranks on cuda:0), the other tasks' bench lines, and the training traces.
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_final3.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5z}; O=gpurun_out/$T; export TMPDIR=/tmp
bash scripts/gpu_r5_final.sh $T || exit $?
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --rehearsal --no-cpu-baseline > $O/bench_rehearsal2.log 2>&1 || { tail -5 $O/bench_rehearsal2.log; exit 1; }
tail -1 $O/bench_rehearsal2.log | cut -c1-300
for t in standup v4 manager; do
  timeout -k 10 200 python bench.py --task $t --no-cpu-baseline > $O/bench_$t.log 2>&1 || { tail -3 $O/bench_$t.log; exit 1; }
  tail -1 $O/bench_$t.log | cut -c1-160
done
timeout -k 10 200 python bench.py --envs-per-gpu 8192 --no-cpu-baseline > $O/bench_8k.log 2>&1 && tail -1 $O/bench_8k.log | cut -c1-160
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0 || exit 1
bash scripts/gpu_train_profile.sh ${T}_v2 4096 zbot-6b-walking-v2
