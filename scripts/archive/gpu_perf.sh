#!/usr/bin/env bash
# Perf snapshot: phase stamps (diagnostic build libzbot_stamps.so), the default bench line, and
# (unless NO_PROF) the rocprofv3 trace + PMC passes of scripts/gpu_profile.sh under prof_<tag>.
# Usage: /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_perf.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; TAG=${1:-perf}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/stamps.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
if [ -z "${NO_PROF:-}" ]; then TAG=$TAG bash scripts/gpu_profile.sh; fi
