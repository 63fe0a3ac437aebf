#!/usr/bin/env bash
# k_act_reg with the actor and the critic in separate workgroups: the PPO GPU tests, then the rollout
# policy step at 4096 envs (walking v2) with the register-resident forward forced (ZBP_ACT=reg)
# against the default (LDS kernel below 16 384 rows), and at C5 (32 768 envs, register path).
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r5_act.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_act}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py tests/test_gpu_rollout_wiring.py \
  tests/test_gpu_train_play.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/test_ppo.log 2>&1 || { echo "ppo tests failed"; tail -30 $O/test_ppo.log; exit 1; }
tail -1 $O/test_ppo.log
bash scripts/gpu_train_profile.sh ${T}_v2 4096 zbot-6b-walking-v2 || exit 1
ZBP_ACT=reg bash scripts/gpu_train_profile.sh ${T}_v2reg 4096 zbot-6b-walking-v2 || exit 1
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0 || exit 1
echo done
