#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export ZB_NAN_DUMP=$PWD/gpurun_out/nan_case.npz
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo rc=$?; grep -E "passed|failed|non-finite|Error" gpurun_out/pytest_gpu.log | head -20
