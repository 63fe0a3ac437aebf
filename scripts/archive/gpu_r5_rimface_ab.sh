#!/usr/bin/env bash
# The round-5 env-step regression (bisected to 17c1be4, the ruling-on-face manifold): HEAD against
# HEAD without the ruling-on-face code compiled in (libzbot_norf.so: ZB_RIMFACE_ON=0) and with it
# as an out-of-line call (libzbot_rfni.so), and the last tree before it (ab_trees/t_e6dd33f),
# interleaved bench lines at 4096 and 8192 envs.
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r5_rimface_ab.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; T=${1:-r5_rimface}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
run() {  # name dir lib args...
  local n=$1 d=$2 lib=$3; shift 3
  (cd $d && ZBOT_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 "$@") > $O/$n.log 2>&1 || { echo "$n failed"; tail -3 $O/$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); k=(d.get('roofline') or {}).get('kernel_ms')
print('$n', round(d['value']/1e6, 2), 'M env-steps/s', round(d['ms_per_step']*1e3, 1), 'us/step', 'kernel_us', round(k*1e3, 1) if k else None, flush=True)"
}
for r in 1 2 3; do
  run e6dd33f_4k_$r $R/ab_trees/t_e6dd33f libzbot.so || exit 1
  run head_4k_$r $R libzbot.so || exit 1
  run norf_4k_$r $R libzbot_norf.so || exit 1
  run rfni_4k_$r $R libzbot_rfni.so || exit 1
done
for r in 1 2; do
  run e6dd33f_8k_$r $R/ab_trees/t_e6dd33f libzbot.so --envs-per-gpu 8192 || exit 1
  run head_8k_$r $R libzbot.so --envs-per-gpu 8192 || exit 1
  run norf_8k_$r $R libzbot_norf.so --envs-per-gpu 8192 || exit 1
  run rfni_8k_$r $R libzbot_rfni.so --envs-per-gpu 8192 || exit 1
done
echo done
