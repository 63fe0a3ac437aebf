#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/diag_parity.py > gpurun_out/diag.log 2>&1; echo rc=$?; tail -60 gpurun_out/diag.log
