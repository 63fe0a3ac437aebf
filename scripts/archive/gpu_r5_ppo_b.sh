#!/usr/bin/env bash
# PPO kernels after a change: the fused PPO GPU tests, then the C5 PMC passes (scripts/gpu_r5_ppo_pmc.sh).
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_ppo_b.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_ppo_b}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py tests/test_gpu_rollout_wiring.py \
  tests/test_gpu_configs.py -m gpu -v -s -k "ppo or fused or rollout or checkpoint" --timeout 300 --timeout-method thread \
  > $O/test_ppo.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/test_ppo.log | tail -12
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r5_ppo_pmc.sh ${T}_pmc
