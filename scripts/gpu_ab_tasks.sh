#!/usr/bin/env bash
# GPU tests, then an A/B bench of libzbot builds over all four tasks:
#   bash scripts/gpu_ab_tasks.sh libA.so libB.so   (paths relative to zbot_lab_amd/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/test_gpu_all.log 2>&1 || { tail -30 gpurun_out/test_gpu_all.log; exit 1; }
  tail -2 gpurun_out/test_gpu_all.log
fi
for r in $(seq ${ROUNDS:-2}); do
  for lib in "$@"; do
    for task in ${TASKS:-walking manager v4 standup}; do
      ZBOT_LIB=$lib timeout -k 10 120 python bench.py --task $task --steps ${STEPS:-500} --warmup 50 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
      echo "$task $lib $r $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M/s kernel_ms", round(d["roofline"]["kernel_ms"],4))')"
    done
  done
done
