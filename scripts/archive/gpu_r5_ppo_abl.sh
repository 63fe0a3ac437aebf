#!/usr/bin/env bash
# The fused PPO tests + C5 PMC passes (scripts/gpu_r5_ppo_b.sh), then one ablation part
# (scripts/gpu_r5_ablate.sh, PART from the environment).
# Usage: gpurun --timeout 1200 -- 'PART=rimface bash scripts/gpu_r5_ppo_abl.sh <tag>'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r5_ppo_b.sh ${1:-r5_ppo_abl} || exit $?
bash scripts/gpu_r5_ablate.sh
