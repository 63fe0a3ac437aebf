#!/usr/bin/env bash
# Evidence pass after the LDS diet (two waves per SIMD): all GPU tests, bench lines of every task,
# walking v2 at 8192 / 65536 envs per GPU, rocprof summaries r1n* (4096 envs; 8192 envs for v2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/test_gpu_all.log 2>&1 || { tail -30 gpurun_out/test_gpu_all.log; exit 1; }
tail -2 gpurun_out/test_gpu_all.log
b() {  # log args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/bench_$n.log 2>&1 || { echo "bench $n failed"; tail -5 gpurun_out/bench_$n.log; exit 1; }
  tail -1 gpurun_out/bench_$n.log
}
b v2 --steps 1000 --warmup 100
b manager --task manager --steps 1000 --warmup 100
b v4 --task v4 --steps 1000 --warmup 100
b standup --task standup --steps 500 --warmup 50
b v2_8192 --envs-per-gpu 8192 --steps 500 --warmup 50 --no-cpu-baseline
b v2_65536 --envs-per-gpu 65536 --steps 200 --warmup 20 --no-cpu-baseline
b manager_8192 --task manager --envs-per-gpu 8192 --steps 500 --warmup 50 --no-cpu-baseline
b v4_8192 --task v4 --envs-per-gpu 8192 --steps 500 --warmup 50 --no-cpu-baseline
b standup_65536 --task standup --envs-per-gpu 65536 --steps 200 --warmup 20 --no-cpu-baseline
p() {  # tag bench-args
  TAG=$1 BENCH_ARGS="$2" PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_$1.log 2>&1 || { echo "profile $1 failed"; tail -5 gpurun_out/prof_$1.log; exit 1; }
  echo "profile $1 ok"
}
p r1n ""
p r1n_mgr "--task manager"
p r1n_v4 "--task v4"
p r1n_su "--task standup"
p r1n_8192 "--envs-per-gpu 8192"
