#!/usr/bin/env bash
# Evidence pass, part 2: phase stamps (walking v2 / manager), rocprof summaries (r1h), v2 PPO 2000 iterations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/stamps.py > gpurun_out/stamps_v2.log 2>&1 || exit $?
TASK=zbot-6b-walking-m-v0 timeout -k 10 200 python scripts/stamps.py > gpurun_out/stamps_mgr.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps_v2.log gpurun_out/stamps_mgr.log
TAG=r1h PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_v2.log 2>&1 || exit $?
TAG=r1h_mgr BENCH_ARGS="--task manager" PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_mgr.log 2>&1 || exit $?
timeout -k 10 600 python scripts/train.py --task zbot-6b-walking-v2 --num_envs 4096 --max_iterations 2000 \
  --log-every 20 --log_dir /tmp/zb_train_v2 > gpurun_out/train_v2_full.log 2>&1 || exit $?
tail -3 gpurun_out/train_v2_full.log
