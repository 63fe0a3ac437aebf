#!/usr/bin/env bash
# Round-4: the TGS refresh (solver_mode 2) parity tests first, then the round evidence (gpu_round4.sh).
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r4_refresh.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; TAG=${1:-r4g}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_fullstate.py tests/test_gpu_fullsize.py -m gpu -v -s -k "refresh" \
  --timeout 300 --timeout-method thread > $O/test_refresh.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed|unexplained" $O/test_refresh.log | tail -12
case $rc in 0|1) ;; *) exit $rc ;; esac
bash scripts/gpu_round4.sh $TAG
timeout -k 10 300 env ZBOT_LIB=libzbot_stamps_t.so python scripts/wave_times.py > $O/wave_times.log 2>&1 || { tail -5 $O/wave_times.log; exit 1; }
grep -v amdgpu.ids $O/wave_times.log | head -30
