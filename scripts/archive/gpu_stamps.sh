#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/stamps.py > gpurun_out/stamps.log 2>&1; echo rc=$?; cat gpurun_out/stamps.log | grep -v amdgpu.ids
