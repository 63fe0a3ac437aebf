#!/usr/bin/env bash
# Round-4: the rim manifold's GPU tests (per pair + full state), then the default bench line with
# self_manifold 2 / 1 / 0 (ROUNDS interleaved rounds).
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r4_rim_ab.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r4l}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_selfcollision.py tests/test_gpu_fullstate.py -k manifold -m gpu -v -s \
  --timeout 300 --timeout-method thread > $O/test_rim.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed|manifold pairs|outside the point" $O/test_rim.log | tail -10
case $rc in 0|1) ;; *) exit $rc ;; esac
ROUNDS=2 bash scripts/gpu_env_ab.sh ${T}_ab "ZB_AB=2" "ZB_AB=1 -- --self-manifold 1" "ZB_AB=0 -- --self-manifold 0"
