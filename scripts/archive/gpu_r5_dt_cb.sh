#!/usr/bin/env bash
# (1) PPO: k_rows_reg<8,8,8> at three waves per SIMD (16-block chunks, 32 KB LDS): PPO GPU tests and
#     the v2 4096-env training timing; (2) the round-5 env-step regression: the substep's dt in its
#     own scalar register (libzbot.so) against the same source without it (libzbot_pre.so), with the
#     ruling-on-face code compiled out (libzbot_dtnorf.so) and the last tree before the regression
#     (ab_trees/t_e6dd33f), interleaved bench lines; stand-up C5 for pre / dt.
# Usage: gpurun --timeout 1000 -- bash scripts/gpu_r5_dt_cb.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; T=${1:-r5_dtcb}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py tests/test_gpu_rollout_wiring.py \
  -x -v --timeout 120 --timeout-method thread -m gpu > $O/test_ppo.log 2>&1 || { echo "ppo tests failed"; tail -30 $O/test_ppo.log; exit 1; }
tail -1 $O/test_ppo.log
bash scripts/gpu_train_profile.sh ${T}_v2 4096 zbot-6b-walking-v2 || exit 1
run() {  # name dir lib args...
  local n=$1 d=$2 lib=$3; shift 3
  (cd $d && ZBOT_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 "$@") > $O/$n.log 2>&1 || { echo "$n failed"; tail -3 $O/$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); k=(d.get('roofline') or {}).get('kernel_ms')
print('$n', round(d['value']/1e6, 2), 'M env-steps/s', round(d['ms_per_step']*1e3, 1), 'us/step', 'kernel_us', round(k*1e3, 1) if k else None, flush=True)"
}
for r in 1 2 3; do
  run e6dd33f_4k_$r $R/ab_trees/t_e6dd33f libzbot.so || exit 1
  run pre_4k_$r $R libzbot_pre.so || exit 1
  run dt_4k_$r $R libzbot.so || exit 1
  run dtnorf_4k_$r $R libzbot_dtnorf.so || exit 1
done
for r in 1 2; do
  run e6dd33f_8k_$r $R/ab_trees/t_e6dd33f libzbot.so --envs-per-gpu 8192 || exit 1
  run pre_8k_$r $R libzbot_pre.so --envs-per-gpu 8192 || exit 1
  run dt_8k_$r $R libzbot.so --envs-per-gpu 8192 || exit 1
  run dtnorf_8k_$r $R libzbot_dtnorf.so --envs-per-gpu 8192 || exit 1
  run pre_su_$r $R libzbot_pre.so --task standup || exit 1
  run dt_su_$r $R libzbot.so --task standup || exit 1
done
echo done
