#!/usr/bin/env bash
# The whole GPU suite + smoke at HEAD (what the driver runs at round end).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r4r}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/test_gpu.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/test_gpu.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
