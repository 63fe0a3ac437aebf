#!/usr/bin/env bash
# per-physics-step contact sensor (v2 / v4) + manager env: diagnostics, all GPU tests, benches, profiles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/dev/diag_mgr.py > gpurun_out/diag_mgr.log 2>&1 || { cat gpurun_out/diag_mgr.log; exit 1; }
cat gpurun_out/diag_mgr.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/test_gpu_all.log 2>&1; rc=$?
tail -15 gpurun_out/test_gpu_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --cpu-baseline-seconds 10 > gpurun_out/bench_v2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v2.log
timeout -k 10 300 python bench.py --task manager --steps 300 --warmup 30 --cpu-baseline-seconds 10 > gpurun_out/bench_manager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_manager.log
