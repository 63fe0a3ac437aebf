#!/usr/bin/env bash
# Round-4 evidence in one call: GPU suite (-s: parity tables), smoke, phase stamps + default bench +
# rocprofv3 trace / PMC (gpu_perf.sh), the other bench configs, then the PPO training profile.
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_round4.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; TAG=${1:-r4}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
if [ -z "${NO_SUITE:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/test_gpu.log 2>&1
  rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/test_gpu.log | tail -6
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/gpu_perf.sh $TAG || exit 1
for args in "--envs-per-gpu 8192" "--envs-per-gpu 65536" "--task standup" "--task v4" "--task manager"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $O/bench_extra.log 2>&1 || { tail -5 $O/bench_extra.log; exit 1; }
  tail -1 $O/bench_extra.log >> $O/bench_lines.jsonl
done
cut -c1-120 $O/bench_lines.jsonl
bash scripts/gpu_train_profile.sh ${TAG}_train 4096 zbot-6b-walking-v2 1
