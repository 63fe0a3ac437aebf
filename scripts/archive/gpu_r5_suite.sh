#!/usr/bin/env bash
# Round-5 GPU evidence: the whole GPU suite (-s: the parity tables), smoke, the default bench line,
# then (optional 2nd argument "pmc") the PPO PMC passes of scripts/gpu_r5_ppo_pmc.sh.
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_suite.sh <tag> [pmc]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5a}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 ${SUITE_LIMIT:-700} python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
  > $O/test_gpu.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/test_gpu.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
if [ "${2:-}" = pmc ]; then bash scripts/gpu_r5_ppo_pmc.sh ${T}_ppo_pmc || exit 1; fi
