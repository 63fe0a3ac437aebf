#!/usr/bin/env bash
# zb_step_kernel A/Bs at HEAD, interleaved rounds of bench lines (no CPU leg):
# the default build at 4096 envs against one point per self pair (self_manifold 0, the round-3 self
# contact) and against GJK stop tolerances of 30 / 100 um (variant builds libzbot_tol30.so /
# libzbot_tol100.so: ZB_GJK_TOL), then 8192 envs (default / self_manifold 0) and 65 536 envs.
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r5_bench_ab.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_bench_ab}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  ZBOT_LIB=$lib timeout -k 10 150 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -3 $O/$n.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e6, 2), 'M env-steps/s', round(d['ms_per_step']*1e3, 1), 'us/step', 'kernel_us', round(d['roofline']['kernel_ms']*1e3, 1))"
}
for r in 1 2 3; do
  run head_4k_$r libzbot.so
  run m0_4k_$r libzbot.so --self-manifold 0
  run tol30_4k_$r libzbot_tol30.so
  run tol100_4k_$r libzbot_tol100.so
done
for r in 1 2; do
  run head_8k_$r libzbot.so --envs-per-gpu 8192
  run m0_8k_$r libzbot.so --envs-per-gpu 8192 --self-manifold 0
done
run head_64k libzbot.so --envs-per-gpu 65536
echo done
