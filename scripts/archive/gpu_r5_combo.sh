#!/usr/bin/env bash
# One call, three steps: the fused PPO tests + a C5 training kernel trace (scripts/gpu_train_profile.sh),
# the zb_step_kernel bench A/Bs (scripts/gpu_r5_bench_ab.sh), one ablation part (PART, scripts/gpu_r5_ablate.sh).
# Usage: gpurun --timeout 1200 -- 'PART=selfref bash scripts/gpu_r5_combo.sh <tag>'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_combo}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py -m gpu -q --timeout 150 \
  --timeout-method thread > $O/test_ppo.log 2>&1 || { tail -15 $O/test_ppo.log; exit 1; }
tail -1 $O/test_ppo.log
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0 || exit 1
bash scripts/gpu_r5_bench_ab.sh ${T}_bench || exit 1
[ -n "${PART:-}" ] && bash scripts/gpu_r5_ablate.sh
