#!/usr/bin/env bash
# (1) k_rows_reg with the actor and the critic in separate workgroups: the PPO GPU tests, then the v2
#     4096-env and C5 training timings (scripts/gpu_train_profile.sh);
# (2) the round-5 env-step bisect: bench lines of the round-5 commits that touched the step kernel,
#     each from its own tree (ab_trees/t_<commit>), interleaved with round-4 final and HEAD:
#     3352e98 round-4 final, e6dd33f step0 terms + term gating, 17c1be4 ruling-on-face manifold +
#     variants dropped, 61a11b1 self refresh (solver_mode 3), f7d07b3 before the dispatch events, HEAD.
# Usage: gpurun --timeout 1150 -- bash scripts/gpu_r5_split_bisect.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; T=${1:-r5_split}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py tests/test_gpu_rollout_wiring.py \
  -x -v --timeout 120 --timeout-method thread -m gpu > $O/test_ppo.log 2>&1 || { echo "ppo tests failed"; tail -30 $O/test_ppo.log; exit 1; }
tail -2 $O/test_ppo.log
bash scripts/gpu_train_profile.sh ${T}_v2 4096 zbot-6b-walking-v2 || exit 1
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0 || exit 1
run() {  # name dir args...
  local n=$1 d=$2; shift 2
  (cd $d && timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 "$@") > $O/$n.log 2>&1 || { echo "$n failed"; tail -3 $O/$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); k=(d.get('roofline') or {}).get('kernel_ms')
print('$n', round(d['value']/1e6, 2), 'M env-steps/s', round(d['ms_per_step']*1e3, 1), 'us/step', 'kernel_us', round(k*1e3, 1) if k else None, flush=True)"
}
TREES="3352e98 e6dd33f 17c1be4 61a11b1 f7d07b3"
for r in 1 2 3; do
  for c in $TREES; do run ${c}_4k_$r $R/ab_trees/t_$c || exit 1; done
  run head_4k_$r $R || exit 1
done
echo done
