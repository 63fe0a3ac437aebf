#!/usr/bin/env bash
# manager-based flat env on the GPU: parity tests, bench, kernel trace, short PPO run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/test_manager.log 2>&1 || { tail -40 gpurun_out/test_manager.log; exit 1; }
tail -2 gpurun_out/test_manager.log
timeout -k 10 300 python bench.py --task manager --steps 300 --warmup 30 --cpu-baseline-seconds 10 > gpurun_out/bench_manager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_manager.log
TAG=r1h_mgr BENCH_ARGS="--task manager" PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_mgr.log 2>&1 || exit $?
timeout -k 10 600 python scripts/train.py --task zbot-6b-walking-m-v0 --num_envs 4096 --max_iterations 40 --log-every 10 > gpurun_out/train_mgr.log 2>&1 || exit $?
tail -2 gpurun_out/train_mgr.log
