#!/usr/bin/env bash
# GPU check: the gpu test suite (or the files given in TESTS), then the default bench line.
# Usage (from the repo root): /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_check.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/test_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/test_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/test_gpu.log | head -20; exit $rc; fi
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
fi
