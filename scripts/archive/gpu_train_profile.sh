#!/usr/bin/env bash
# PPO training iteration timing + profile: 12 iterations of a task (default
# zbot-6b-walking-v2 at 4096 envs, its PPO cfg) plain (collect / learn times from the train log),
# then 6 iterations under rocprofv3 --kernel-trace --stats (csv). A 4th argument 0 selects the torch
# update path (ZBOT_PPO_FUSED=0) for the A/B.
# Usage: gpurun -- bash scripts/gpu_train_profile.sh <tag> [num_envs] [task] [fused]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; TAG=${1:-train}; N=${2:-4096}; TASK=${3:-zbot-6b-walking-v2}
export ZBOT_PPO_FUSED=${4:-1}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/train.py --task $TASK --num_envs $N --max_iterations 12 --seed 42 \
  --log_root $O/logs > $O/train.log 2>&1 || { tail -5 $O/train.log; exit 1; }
tail -2 $O/train.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 scripts/train.py \
  --task $TASK --num_envs $N --max_iterations 6 --seed 42 --log_root $O/logs_prof > $O/train_prof.log 2>&1
rc=$?; tail -1 $O/train_prof.log | cut -c1-300; exit $rc
