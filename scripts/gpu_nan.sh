#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 400 python scripts/diag_nan2.py > gpurun_out/nan.log 2>&1; echo rc=$?; tail -30 gpurun_out/nan.log
