#!/usr/bin/env bash
# Fused PPO update on the GPU: its tests first, then the PPO GPU tests, then a training profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/${1:-r4_ppo}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_ppo.py -m gpu -v -s --timeout 200 \
  --timeout-method thread > $O/test_ppo.log 2>&1
rc=$?; grep -E "passed|failed|Error|fused vs" $O/test_ppo.log | tail -12
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_train_profile.sh ${1:-r4_ppo}_train
