#!/usr/bin/env bash
# PPO kernels (libzbot_ppo.so): the fused-update GPU tests, then a C5 training profile (kernel trace
# + stats, scripts/gpu_train_profile.sh) and the 4096-env walking one.
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r5_ppo.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_ppo}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py -m gpu -v -s \
  --timeout 300 --timeout-method thread > $O/test_ppo.log 2>&1
rc=$?; grep -E "passed|failed|Error|fused vs|GAE" $O/test_ppo.log | tail -12
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0 || exit 1
bash scripts/gpu_train_profile.sh ${T}_v2 4096 zbot-6b-walking-v2
