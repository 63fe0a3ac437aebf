#!/usr/bin/env bash
# A/B bench of several builds of libzbot in one box session: bash scripts/gpu_ab.sh libA.so libB.so ...
# (paths relative to zbot_lab_amd/). Alternates A B A B ... ROUNDS times; each run time-limited.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq $ROUNDS); do
  for lib in "$@"; do
    ZBOT_LIB=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-400} --warmup 40 --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/ab.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/ab.log; exit 1; }
    python -c "import json,sys;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);print('%-28s value %.4e  ms/step %.4f  kernel_ms %.4f'%(sys.argv[1],d['value'],d['ms_per_step'],d['roofline']['kernel_ms']))" $lib
  done
done
