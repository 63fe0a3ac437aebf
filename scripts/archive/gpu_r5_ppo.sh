#!/usr/bin/env bash
# PPO kernels (libzbot_ppo.so): the fused-update / rollout / C5 PPO GPU tests (+ the TGS full-state
# tests), smoke and the default bench line, then C5 training profiles (kernel trace + stats,
# scripts/gpu_train_profile.sh) with the register-resident row kernels and, for the A/B, the LDS ones
# (ZBP_ROWS=lds), and the 4096-env walking one.
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_ppo.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_ppo}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py \
  tests/test_gpu_rollout_wiring.py tests/test_gpu_configs.py tests/test_gpu_fullstate.py tests/test_ppo.py -m gpu -v -s \
  -k "ppo or fused or rollout or checkpoint or tgs or graph" --timeout 300 --timeout-method thread > $O/test_ppo.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/test_ppo.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0 || exit 1
ZBP_ROWS=lds timeout -k 10 300 python3 scripts/train.py --task zbot-6b-standup-v0 --num_envs 32768 --max_iterations 12 \
  --seed 42 --log_root $O/logs_lds > $O/train_c5_lds.log 2>&1 || { tail -5 $O/train_c5_lds.log; exit 1; }
tail -2 $O/train_c5_lds.log | cut -c1-400
bash scripts/gpu_train_profile.sh ${T}_v2 4096 zbot-6b-walking-v2
