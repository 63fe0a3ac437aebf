#!/usr/bin/env bash
# Where the env step lost speed since round 3 ("account for the 8192-env loss
# with an A/B"): the bench of earlier commits, each built from its own tree (ab_trees/t_<commit>,
# extracted with git archive and built by that commit's build.py), interleaved on one box with HEAD.
#   4802a18 round-3 final (r3zf: 117.2 us, 31.4 M)    98a4830 round 4, face manifold (r4e)
#   dbf3df5 round 4 + TGS refresh templates (r4h)      3352e98 round-4 final (rim manifold default)
#   HEAD    round 5
# Usage: gpurun --timeout 1100 -- bash scripts/gpu_r5_regress_ab.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; T=${1:-r5_regress}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
run() {  # name dir args...
  local n=$1 d=$2; shift 2
  (cd $d && timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 "$@") > $O/$n.log 2>&1 || { echo "$n failed"; tail -3 $O/$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); k=(d.get('roofline') or {}).get('kernel_ms')
print('$n', round(d['value']/1e6, 2), 'M env-steps/s', round(d['ms_per_step']*1e3, 1), 'us/step', 'kernel_us', round(k*1e3, 1) if k else None, flush=True)"
}
TREES="4802a18 98a4830 dbf3df5 3352e98"
for r in 1 2 3; do
  for c in $TREES; do run ${c}_4k_$r $R/ab_trees/t_$c || exit 1; done
  run head_4k_$r $R || exit 1
done
for r in 1 2; do
  for c in $TREES; do run ${c}_8k_$r $R/ab_trees/t_$c --envs-per-gpu 8192 || exit 1; done
  run head_8k_$r $R --envs-per-gpu 8192 || exit 1
done
echo done
