#!/usr/bin/env bash
# Round-1 evidence pass: all GPU tests, v2 / manager benches, rocprof passes (v2 + manager),
# C4 on one GPU (v2 PPO, 2000 iterations, 4096 envs). Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/test_gpu_all.log 2>&1; rc=$?
tail -15 gpurun_out/test_gpu_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 > gpurun_out/bench_v2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v2.log
timeout -k 10 300 python bench.py --task manager --steps 1000 --warmup 100 > gpurun_out/bench_manager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_manager.log
TAG=r1h PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_v2.log 2>&1 || exit $?
TAG=r1h_mgr BENCH_ARGS="--task manager" PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_mgr.log 2>&1 || exit $?
timeout -k 10 600 python scripts/train.py --task zbot-6b-walking-v2 --num_envs 4096 --max_iterations 2000 \
  --log-every 20 --log_dir /tmp/zb_train_v2 > gpurun_out/train_v2_full.log 2>&1 || exit $?
tail -2 gpurun_out/train_v2_full.log
timeout -k 10 300 python scripts/stamps.py > gpurun_out/stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps.log
