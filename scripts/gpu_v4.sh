#!/usr/bin/env bash
# walking v4 on the GPU: bench, kernel trace, short PPO run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --task v4 --steps 300 --warmup 30 --cpu-baseline-seconds 10 > gpurun_out/bench_v4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v4.log
TAG=r1g_v4 BENCH_ARGS="--task v4" PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_v4.log 2>&1 || exit $?
timeout -k 10 600 python scripts/train.py --task zbot-6b-walking-v4 --num_envs 4096 --max_iterations 40 --log-every 10 > gpurun_out/train_v4.log 2>&1 || exit $?
tail -2 gpurun_out/train_v4.log
