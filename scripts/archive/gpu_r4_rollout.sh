#!/usr/bin/env bash
# Round-4: the fused rollout step (zbp_act / zbp_env_post) — its GPU tests, the PPO / train-play GPU
# tests, then the training iteration profile at 4096 envs with the fused rollout and without it
# (ZBOT_ROLLOUT_FUSED=0), and the C5 stand-up training rate.
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r4_rollout.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r4i}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_ppo.py tests/test_gpu_train_play.py -m gpu -v \
  --timeout 300 --timeout-method thread > $O/test_rollout.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/test_rollout.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_train_profile.sh ${T}_train 4096 zbot-6b-walking-v2 1 || exit 1
ZBOT_ROLLOUT_FUSED=0 timeout -k 10 300 python3 scripts/train.py --task zbot-6b-walking-v2 --num_envs 4096 --max_iterations 12 \
  --seed 42 --log_root $O/logs_nofuse > $O/train_nofuse.log 2>&1 || { tail -5 $O/train_nofuse.log; exit 1; }
tail -1 $O/train_nofuse.log | cut -c1-300
timeout -k 10 300 python3 scripts/train.py --task zbot-6b-standup-v0 --num_envs 32768 --max_iterations 12 \
  --seed 42 --log_root $O/logs_c5 > $O/train_c5.log 2>&1 || { tail -5 $O/train_c5.log; exit 1; }
tail -1 $O/train_c5.log | cut -c1-300
