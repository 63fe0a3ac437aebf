#!/usr/bin/env bash
# The substep's dt read from a copy after the model in device memory (libzbot_lc.so: a scalar load
# at the point of use) against HEAD's dt through an empty asm (libzbot.so): the GPU suite on the
# variant, then interleaved bench lines (4096 / 8192 envs, stand-up, v4, manager).
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r5_loopcfg.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; T=${1:-r5_lc}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
ZBOT_LIB=libzbot_lc.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/test_gpu_lc.log 2>&1 || { echo "suite failed"; tail -30 $O/test_gpu_lc.log; exit 1; }
tail -1 $O/test_gpu_lc.log
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  ZBOT_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -3 $O/$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); k=(d.get('roofline') or {}).get('kernel_ms')
print('$n', round(d['value']/1e6, 2), 'M env-steps/s', round(d['ms_per_step']*1e3, 1), 'us/step', 'kernel_us', round(k*1e3, 1) if k else None, flush=True)"
}
for r in 1 2 3; do
  run head_4k_$r libzbot.so || exit 1
  run lc_4k_$r libzbot_lc.so || exit 1
done
for r in 1 2; do
  run head_8k_$r libzbot.so --envs-per-gpu 8192 || exit 1
  run lc_8k_$r libzbot_lc.so --envs-per-gpu 8192 || exit 1
  for t in standup v4 manager; do
    run head_${t}_$r libzbot.so --task $t || exit 1
    run lc_${t}_$r libzbot_lc.so --task $t || exit 1
  done
done
echo done
