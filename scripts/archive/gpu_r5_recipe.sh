#!/usr/bin/env bash
# The reference's staged walking recipe from its first stage (v2.py:78-206,
# README.md:69): step0 -> step1 (v0, "use this") -> step2 -> step3 -> step4, ITERS iterations each
# (default 2000) at NUM_ENVS envs (default 4096), seed 42, chained with --resume, then a
# deterministic play from fresh episodes (forward distance per episode, air-time statistics).
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_recipe.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_recipe}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
LR=/tmp/zb_train_logs_$T
IT=${ITERS:-2000}
X=${EXTRA:-}
run() {  # name limit args...
  local n=$1 l=$2; shift 2
  echo "== $n"
  timeout -k 10 $l python -u "$@" > $O/$n.log 2>&1; local rc=$?
  tail -n 1 $O/$n.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stop ($n rc=$rc)"; tail -20 $O/$n.log; exit $rc; fi
}
prev=""
for st in ${STAGES:-step0 step1 step2 step3 step4}; do
  res=""; [ -n "$prev" ] && res="--resume --load_run .*_$prev"
  run v2_$st 300 scripts/train.py --task zbot-6b-walking-v2 --num_envs ${NUM_ENVS:-4096} --max_iterations $IT --seed 42 \
    --log_root $LR --log-every 100 --reward_cfg $st --run_name $st $res $X
  prev=$st
done
run v2_play 300 scripts/play.py --task zbot-6b-walking-v2 --num_envs 1024 --log_root $LR --num_steps 999 --fresh_episodes $X
for f in $(find $LR -name train_log.jsonl); do cp $f $O/$(basename $(dirname $f)).jsonl; done
echo done
