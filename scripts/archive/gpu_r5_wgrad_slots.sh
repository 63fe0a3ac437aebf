#!/usr/bin/env bash
# k_wgrad's split-K count at walking v2's 24 576-row minibatches: workgroup slots per CU 1 / 2 (default)
# / 4 (ZBP_WGRAD_SLOTS_PER_CU), each a v2 4096-env training trace; then C5 at 4.
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r5_wgrad_slots.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_ws}; export TMPDIR=/tmp
for k in 1 2 4; do
  ZBP_WGRAD_SLOTS_PER_CU=$k bash scripts/gpu_train_profile.sh ${T}_v2_$k 4096 zbot-6b-walking-v2 || exit 1
done
ZBP_WGRAD_SLOTS_PER_CU=4 bash scripts/gpu_train_profile.sh ${T}_c5_4 32768 zbot-6b-standup-v0 || exit 1
echo done
