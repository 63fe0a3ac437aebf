#!/usr/bin/env bash
# Instruction-cache counters of zb_step_kernel on bench.py (one PMC pass), then HEAD against the build
# without LLVM's load-store vectorizer (libzbot_lsv.so: fewer merged scalar loads, so fewer 16-register
# tuples to spill), interleaved bench lines at 4096 envs.
# Usage: gpurun --timeout 600 -- bash scripts/gpu_r5_icache.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; T=${1:-r5_icache}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_WAVES \
  --output-format csv -d $O/pmc_icache -o run -- python3 $R/bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/pmc_icache.log 2>&1 || { echo "pmc pass failed"; tail -5 $O/pmc_icache.log; }
cd $R
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  ZBOT_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -3 $O/$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); k=(d.get('roofline') or {}).get('kernel_ms')
print('$n', round(d['value']/1e6, 2), 'M env-steps/s', round(d['ms_per_step']*1e3, 1), 'us/step', 'kernel_us', round(k*1e3, 1) if k else None, flush=True)"
}
for r in 1 2 3; do
  run head_4k_$r libzbot.so || exit 1
  run lsv_4k_$r libzbot_lsv.so || exit 1
done
echo done
