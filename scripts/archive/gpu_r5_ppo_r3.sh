#!/usr/bin/env bash
# The fused PPO tests + a C5 training kernel trace, then the r3seeds ablation part.
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_ppo_r3.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_ppo_r3}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py -m gpu -q --timeout 150 \
  --timeout-method thread > $O/test_ppo.log 2>&1 || { tail -15 $O/test_ppo.log; exit 1; }
tail -1 $O/test_ppo.log
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0 || exit 1
PART=r3seeds bash scripts/gpu_r5_ablate.sh
