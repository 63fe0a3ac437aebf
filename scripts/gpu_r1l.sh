#!/usr/bin/env bash
# Evidence pass, part 1: all GPU tests, staged-store A/B, v2 / manager / 65536-env benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/test_gpu_all.log 2>&1 || { tail -30 gpurun_out/test_gpu_all.log; exit 1; }
tail -3 gpurun_out/test_gpu_all.log
for r in 1 2; do
  for lib in libzbot.so libzbot_nostage.so; do
    for task in walking manager; do
      ZBOT_LIB=$lib timeout -k 10 120 python bench.py --task $task --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/ab_$task.$lib.$r.log 2>&1 || exit $?
      echo "$task $lib $r $(tail -1 gpurun_out/ab_$task.$lib.$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M/s kernel_ms", round(d["roofline"]["kernel_ms"],4))')"
    done
  done
done
timeout -k 10 300 python bench.py > gpurun_out/bench_v2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v2.log
timeout -k 10 300 python bench.py --envs-per-gpu 65536 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_v2_65536.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v2_65536.log
