#!/usr/bin/env bash
# The staged v2 recipe from step0 (seed 42) under each round-5 physics option: the ruling-on-face
# manifold (self_manifold 3) and the TGS refresh of ground + self contacts (solver_mode 3).
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r5_recipe_ab.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_recipe_ab}
EXTRA="--env=solver.self_manifold=3" bash scripts/gpu_r5_recipe.sh ${T}_m3 || exit 1
EXTRA="--env=solver.mode=3" bash scripts/gpu_r5_recipe.sh ${T}_r3
