#!/usr/bin/env bash
# Round evidence in one call: the GPU test suite, then (if green) phase stamps, the default bench
# line, the rocprofv3 trace + PMC passes (prof_<tag>), and bench lines of the other configs.
# Usage: /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_round.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; TAG=${1:-round}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/test_gpu.log 2>&1
rc=$?; tail -1 $O/test_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED" $O/test_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/gpu_perf.sh $TAG || exit 1
for args in "--envs-per-gpu 8192" "--envs-per-gpu 65536" "--task standup" "--task v4" "--task manager"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $O/bench_extra.log 2>&1 || { tail -5 $O/bench_extra.log; exit 1; }
  tail -1 $O/bench_extra.log >> $O/bench_lines.jsonl
done
cut -c1-160 $O/bench_lines.jsonl
