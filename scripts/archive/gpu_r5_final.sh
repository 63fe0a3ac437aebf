#!/usr/bin/env bash
# Round-5 evidence at HEAD: the whole GPU suite, smoke, the default bench line (with the CPU leg),
# then the rocprofv3 passes on bench.py (scripts/gpu_profile.sh: kernel trace + stats, FETCH / WRITE
# / SQ PMC passes) for profiles/<tag> (scripts/prof_summary.py).
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_final.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5z}; export TMPDIR=/tmp
SUITE_LIMIT=${SUITE_LIMIT:-700} bash scripts/gpu_r5_suite.sh $T || exit $?
TAG=$T bash scripts/gpu_profile.sh || exit $?
echo done
