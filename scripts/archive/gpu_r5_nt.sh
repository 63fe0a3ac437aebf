#!/usr/bin/env bash
# Non-temporal state / obs stores (libzbot_nt.so: ZB_NT_STORES=1) against HEAD: interleaved bench
# lines (the step time includes the kernel boundaries, where the dirty L2 lines are written back),
# 4096 and 8192 envs, then a kernel trace of each (start-to-start gaps).
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r5_nt.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; T=${1:-r5_nt}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  ZBOT_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -3 $O/$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); k=(d.get('roofline') or {}).get('kernel_ms')
print('$n', round(d['value']/1e6, 2), 'M env-steps/s', round(d['ms_per_step']*1e3, 1), 'us/step', 'kernel_us', round(k*1e3, 1) if k else None, flush=True)"
}
for r in 1 2 3; do
  run head_4k_$r libzbot.so || exit 1
  run nt_4k_$r libzbot_nt.so || exit 1
done
for r in 1 2; do
  run head_8k_$r libzbot.so --envs-per-gpu 8192 || exit 1
  run nt_8k_$r libzbot_nt.so --envs-per-gpu 8192 || exit 1
done
cd /tmp
for v in head nt; do
  lib=libzbot.so; [ $v = nt ] && lib=libzbot_nt.so
  ZBOT_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 $R/bench.py --no-cpu-baseline --steps 200 --warmup 20 > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
done
echo done
