#!/usr/bin/env bash
# The fused PPO tests, C5 and v2-4096 training kernel traces, then the staged v2 recipe from step0 with
# seeds 1 and 2 (seed 42: profiles/r5_recipe).
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_check2.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_check2}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py tests/test_gpu_rollout_wiring.py -m gpu -q \
  --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -15 $O/test.log; exit 1; }
tail -1 $O/test.log
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0 || exit 1
bash scripts/gpu_train_profile.sh ${T}_v2 4096 zbot-6b-walking-v2 || exit 1
for sd in 1 2; do EXTRA="--seed $sd" bash scripts/gpu_r5_recipe.sh ${T}_recipe_s$sd || exit 1; done
