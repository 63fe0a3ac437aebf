#!/usr/bin/env bash
# quick loop: gpu tests, stamps breakdown, bench (each step time-limited; stop on crash)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export ZB_NAN_DUMP=$PWD/gpurun_out/nan_case.npz
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | head -12
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/stamps.py > gpurun_out/stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps.log
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print('bench value %.4e  ms/step %.4f  kernel_ms %.4f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms']))"
