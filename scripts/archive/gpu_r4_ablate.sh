#!/usr/bin/env bash
# Round-4 ablations under the fixed 3-seed protocol (seeds 42, 1, 2 per physics
# change; one DESIGN §7c row per change). PART=a: stand-up at C5's batch (32768 envs, 1000
# iterations) with the face manifold on (default) and off; PART=b: stand-up with the TGS refresh
# (solver_mode 2), then the staged v2 recipe with the refresh (seed 42).
# PART=c: the rim manifold (self_manifold 2) rows.
# Usage: gpurun --timeout 1200 -- 'PART=a bash scripts/gpu_r4_ablate.sh'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "${PART:-a}" = c ]; then  # the rim manifold (self_manifold 2, the round-4 default) under the same protocol
  NUM_ENVS=32768 ITERS=1000 RUNS="c5m2_s42:--seed=42,--env=solver.self_manifold=2 c5m2_s1:--seed=1,--env=solver.self_manifold=2 c5m2_s2:--seed=2,--env=solver.self_manifold=2" \
    bash scripts/gpu_standup_ablate.sh
elif [ "${PART:-a}" = a ]; then
  NUM_ENVS=32768 ITERS=1000 RUNS="c5m1_s42:--seed=42 c5m1_s1:--seed=1 c5m1_s2:--seed=2 c5m0_s42:--seed=42,--env=solver.self_manifold=0 c5m0_s1:--seed=1,--env=solver.self_manifold=0 c5m0_s2:--seed=2,--env=solver.self_manifold=0" \
    bash scripts/gpu_standup_ablate.sh
else
  NUM_ENVS=32768 ITERS=1000 RUNS="c5r2_s42:--seed=42,--env=solver.mode=2 c5r2_s1:--seed=1,--env=solver.mode=2 c5r2_s2:--seed=2,--env=solver.mode=2" \
    bash scripts/gpu_standup_ablate.sh || exit $?
  OUT=v2_r2 SKIP_STANDUP=1 EXTRA="--env=solver.mode=2 --seed=42" bash scripts/gpu_train_recipes.sh
fi
