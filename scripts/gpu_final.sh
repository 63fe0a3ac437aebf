#!/usr/bin/env bash
# Evidence pass (TAG r1k): GPU tests, bench lines (all tasks, 65536 envs), rocprof summaries r1k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/test_gpu_all.log 2>&1 || { tail -30 gpurun_out/test_gpu_all.log; exit 1; }
tail -2 gpurun_out/test_gpu_all.log
timeout -k 10 300 python bench.py > gpurun_out/bench_v2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v2.log
for t in manager v4 standup; do
  timeout -k 10 300 python bench.py --task $t > gpurun_out/bench_$t.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$t.log
done
timeout -k 10 300 python bench.py --envs-per-gpu 8192 --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/bench_v2_8192.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v2_8192.log
timeout -k 10 300 python bench.py --envs-per-gpu 65536 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_v2_65536.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v2_65536.log
TAG=r1k PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_v2.log 2>&1 || exit $?
TAG=r1k_mgr BENCH_ARGS="--task manager" PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_mgr.log 2>&1 || exit $?
TAG=r1k_v4 BENCH_ARGS="--task v4" PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_v4.log 2>&1 || exit $?
TAG=r1k_su BENCH_ARGS="--task standup" PSTEPS=50 bash scripts/gpu_profile.sh > gpurun_out/prof_su.log 2>&1 || exit $?
echo done
