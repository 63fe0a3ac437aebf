#!/usr/bin/env bash
# Round-1 evidence pass + staged-store A/B: all GPU tests, A/B benches (staged vs per-lane stores),
# v2 / manager benches, rocprof passes, C4 on one GPU (v2 PPO 2000 iterations), phase stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/test_gpu_all.log 2>&1; rc=$?
tail -15 gpurun_out/test_gpu_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
  for lib in libzbot.so libzbot_nostage.so; do
    for task in walking manager; do
      ZBOT_LIB=$lib timeout -k 10 120 python bench.py --task $task --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/ab_$task.$lib.$r.log 2>&1 || exit $?
      echo "$task $lib $r $(tail -1 gpurun_out/ab_$task.$lib.$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M/s kernel_ms", round(d["roofline"]["kernel_ms"],4))')"
    done
  done
done
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 > gpurun_out/bench_v2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v2.log
timeout -k 10 300 python bench.py --task manager --steps 1000 --warmup 100 > gpurun_out/bench_manager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_manager.log
timeout -k 10 300 python bench.py --envs-per-gpu 65536 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_v2_65536.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v2_65536.log
TAG=r1h PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_v2.log 2>&1 || exit $?
TAG=r1h_mgr BENCH_ARGS="--task manager" PSTEPS=100 bash scripts/gpu_profile.sh > gpurun_out/prof_mgr.log 2>&1 || exit $?
timeout -k 10 600 python scripts/train.py --task zbot-6b-walking-v2 --num_envs 4096 --max_iterations 2000 \
  --log-every 20 --log_dir /tmp/zb_train_v2 > gpurun_out/train_v2_full.log 2>&1 || exit $?
tail -2 gpurun_out/train_v2_full.log
timeout -k 10 300 python scripts/stamps.py > gpurun_out/stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps.log
