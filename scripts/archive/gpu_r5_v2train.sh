#!/usr/bin/env bash
# Walking v2 training throughput at 4096 envs (its PPO cfg, [128, 128, 128] nets): the register-resident
# row kernels against the LDS ones (ZBP_ROWS=lds), each a kernel trace (scripts/gpu_train_profile.sh);
# then the bench lines of the other tasks (stand-up C5, v4, manager) for the README table.
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r5_v2train.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_v2train}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
bash scripts/gpu_train_profile.sh ${T}_reg 4096 zbot-6b-walking-v2 || exit 1
ZBP_ROWS=lds bash scripts/gpu_train_profile.sh ${T}_lds 4096 zbot-6b-walking-v2 || exit 1
for t in standup v4 manager; do
  timeout -k 10 200 python bench.py --task $t --no-cpu-baseline > $O/bench_$t.log 2>&1 || { tail -3 $O/bench_$t.log; exit 1; }
  tail -1 $O/bench_$t.log | cut -c1-160
done
