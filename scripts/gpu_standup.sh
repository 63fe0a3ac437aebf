#!/usr/bin/env bash
# stand-up task on the GPU: bench (C5), kernel profile, short PPO run; walking bench for regression
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/bench_walk.log 2>&1 || exit $?
tail -1 gpurun_out/bench_walk.log
timeout -k 10 300 python bench.py --task standup --steps 200 --warmup 20 --cpu-baseline-seconds 10 > gpurun_out/bench_su.log 2>&1 || exit $?
tail -1 gpurun_out/bench_su.log
rm -rf gpurun_out/prof_su
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_su -o run -- python3 bench.py --task standup --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/prof_su.log 2>&1 || exit $?
timeout -k 10 600 python scripts/train.py --task zbot-6b-standup-v0 --num_envs 4096 --max_iterations 40 --log-every 10 > gpurun_out/train_su.log 2>&1 || exit $?
tail -3 gpurun_out/train_su.log
