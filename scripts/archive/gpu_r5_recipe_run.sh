#!/usr/bin/env bash
# The fused PPO tests, then the staged v2 recipe from step0 (scripts/gpu_r5_recipe.sh).
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_recipe_run.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_recipe}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_ppo_fused.py -m gpu -q --timeout 150 --timeout-method thread \
  > $O/test_ppo.log 2>&1 || { tail -15 $O/test_ppo.log; exit 1; }
tail -1 $O/test_ppo.log
bash scripts/gpu_r5_recipe.sh $T
