#!/usr/bin/env bash
# C4 on one GPU: zbot-6b-walking-v2 PPO for 2000 iterations (4096 envs), log every 20 iterations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python scripts/train.py --task zbot-6b-walking-v2 --num_envs 4096 --max_iterations 2000 \
  --log-every 20 --log_dir /tmp/zb_train_v2 > gpurun_out/train_v2_full.log 2>&1 || exit $?
tail -2 gpurun_out/train_v2_full.log
