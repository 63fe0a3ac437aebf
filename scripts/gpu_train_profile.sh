#!/usr/bin/env bash
# PPO training iteration profile: 8 iterations of zbot-6b-walking-v2 at 4096 envs
# (PPORunnerCfgV2) under rocprofv3 --kernel-trace --stats; per-iteration collect / learn times from
# the train log. Usage: gpurun -- bash scripts/gpu_train_profile.sh <tag> [num_envs] [task]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; TAG=${1:-train}; N=${2:-4096}; TASK=${3:-zbot-6b-walking-v2}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 scripts/train.py --task $TASK \
  --num_envs $N --max_iterations 8 --seed 42 --log_root $O/logs > $O/train.log 2>&1
rc=$?; tail -3 $O/train.log; exit $rc
