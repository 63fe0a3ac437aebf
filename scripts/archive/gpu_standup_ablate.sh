#!/usr/bin/env bash
# Stand-up behavioural anchor: zbot-6b-standup-v0 at the reference's scale
# (4096 envs, Zbot6SUpEnvPPOCfg, 2000 iterations so the 1000-iteration curriculum acts), over seeds
# and one-factor simulator ablations; each run is followed by a 290-step play from fresh episodes
# whose posture summary (end-of-episode base z, feet z-axis alignment) is the outcome.
# Usage: RUNS="base_s1:--seed=1 pgs8:--env=solver.iterations=8" gpurun -- bash scripts/gpu_standup_ablate.sh
# A run's args may hold lib=<file> (a variant build, e.g. lib=libzbot_nc24.so: ZBOT_LIB for its train
# and play) and --env=solver.mode=1 (the TGS-style contact solve).
# C5 batch: NUM_ENVS=32768 ITERS=1000 RUNS="c5_hull:" (profiles/r2e_train/c5_play/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/standup_ablate; mkdir -p $O
export TMPDIR=/tmp
LR=/tmp/zb_su_logs; IT=${ITERS:-2000}
for spec in ${RUNS:-base:}; do
  name=${spec%%:*}; extra=$(echo "${spec#*:}" | tr ',' ' ')
  lib=$(echo "$extra" | tr ' ' '\n' | grep '^lib=' | cut -d= -f2 || true)
  extra=$(echo "$extra" | tr ' ' '\n' | grep -v '^lib=' | tr '\n' ' ' || true)
  export ZBOT_LIB=${lib:-libzbot.so}
  echo "== $name $extra lib=$ZBOT_LIB"
  timeout -k 10 600 python -u scripts/train.py --task zbot-6b-standup-v0 --num_envs ${NUM_ENVS:-4096} --max_iterations $IT \
    --log_root $LR --log-every 250 --run_name $name $extra > $O/$name.train.log 2>&1 || { echo "train $name rc=$?"; tail -5 $O/$name.train.log; exit 1; }
  tail -n 1 $O/$name.train.log
  pextra=$(echo "$extra" | tr ' ' '\n' | grep -- '--env' | tr '\n' ' ' || true)
  timeout -k 10 300 python -u scripts/play.py --task zbot-6b-standup-v0 --num_envs 1024 --log_root $LR \
    --load_run ".*_$name" --num_steps 290 --fresh_episodes --no_export $pextra > $O/$name.play.log 2>&1 || { echo "play $name rc=$?"; tail -5 $O/$name.play.log; exit 1; }
  tail -n 1 $O/$name.play.log
  cp $(find $LR -path "*_$name/train_log.jsonl" | head -1) $O/$name.jsonl
done
echo done
