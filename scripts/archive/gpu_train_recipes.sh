#!/usr/bin/env bash
# Behavioural anchors: the stand-up task at the reference's scale and the
# staged v2 recipe (step2 -> step3 -> step4, 2000 iterations each, chained with --resume), then play.
# Logs under gpurun_out/${OUT:-train}/ (copy the summaries into profiles/<round>_train/); OUT also
# separates the checkpoints of two recipes run in one call (e.g. OUT=v2_pgs, then OUT=v2_tgs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/${OUT:-train}; mkdir -p $O
export TMPDIR=/tmp
LR=/tmp/zb_train_logs_${OUT:-train}   # checkpoints stay on the box; the per-iteration logs are copied back below
IT=${ITERS:-2000}
X=${EXTRA:-}    # extra train / play arguments, e.g. EXTRA="--env=solver.iterations=8"
run() {  # name limit args...
  local n=$1 l=$2; shift 2
  echo "== $n"
  timeout -k 10 $l python -u "$@" > $O/$n.log 2>&1; local rc=$?
  tail -n 1 $O/$n.log
  if [ $rc -ne 0 ]; then echo "stop ($n rc=$rc)"; tail -20 $O/$n.log; exit $rc; fi
}
if [ -z "${SKIP_STANDUP:-}" ]; then
  run standup_train 1500 scripts/train.py --task zbot-6b-standup-v0 --num_envs 4096 --max_iterations $IT --log_root $LR --log-every 50 --run_name su4096 $X
  run standup_play 300 scripts/play.py --task zbot-6b-standup-v0 --num_envs 1024 --log_root $LR --num_steps 290 --fresh_episodes $X
fi
if [ -z "${SKIP_V2:-}" ]; then
  run v2_step2 1500 scripts/train.py --task zbot-6b-walking-v2 --num_envs ${NUM_ENVS:-4096} --max_iterations $IT --log_root $LR --log-every 50 --reward_cfg step2 --run_name step2 $X
  run v2_step3 1500 scripts/train.py --task zbot-6b-walking-v2 --num_envs ${NUM_ENVS:-4096} --max_iterations $IT --log_root $LR --log-every 50 --reward_cfg step3 --run_name step3 --resume --load_run '.*_step2' $X
  run v2_step4 1500 scripts/train.py --task zbot-6b-walking-v2 --num_envs ${NUM_ENVS:-4096} --max_iterations $IT --log_root $LR --log-every 50 --reward_cfg step4 --run_name step4 --resume --load_run '.*_step3' $X
  run v2_play 300 scripts/play.py --task zbot-6b-walking-v2 --num_envs 1024 --log_root $LR --num_steps 999 --fresh_episodes $X
fi
for f in $(find $LR -name train_log.jsonl); do cp $f $O/$(basename $(dirname $f)).jsonl; done
echo done
