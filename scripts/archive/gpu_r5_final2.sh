#!/usr/bin/env bash
# Round-5 evidence at HEAD (scripts/gpu_r5_final.sh: GPU suite, smoke, bench, rocprof passes), then the
# C5 and walking-v2 training kernel traces.
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_final2.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5z}; export TMPDIR=/tmp
bash scripts/gpu_r5_final.sh $T || exit $?
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0 || exit 1
bash scripts/gpu_train_profile.sh ${T}_v2 4096 zbot-6b-walking-v2
