#!/usr/bin/env bash
# Round-5 ablations under the fixed 3-seed protocol (stand-up at C5's batch: 32768 envs, 1000
# iterations, seeds 42, 1, 2; played deterministically for 290 steps on 1024 fresh envs;
# scripts/gpu_standup_ablate.sh). PART=rimface: the ruling-on-face manifold (self_manifold 3);
# PART=selfref: the TGS refresh of ground and self contacts (solver_mode 3); PART=r3seeds: the seeds
# that stood at C5 with the round-3 physics (3, 5, 6), with the HEAD default and with one point per
# self pair (self_manifold 0, the round-3 self contact) -- two runs per seed that differ only in the
# manifold change.
# Usage: gpurun --timeout 1200 -- 'PART=rimface bash scripts/gpu_r5_ablate.sh'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
case "${PART:-rimface}" in
  rimface) RUNS="c5m3_s42:--seed=42,--env=solver.self_manifold=3 c5m3_s1:--seed=1,--env=solver.self_manifold=3 c5m3_s2:--seed=2,--env=solver.self_manifold=3" ;;
  selfref) RUNS="c5r3_s42:--seed=42,--env=solver.mode=3 c5r3_s1:--seed=1,--env=solver.mode=3 c5r3_s2:--seed=2,--env=solver.mode=3" ;;
  r3seeds) RUNS="c5d_s3:--seed=3 c5m0_s3:--seed=3,--env=solver.self_manifold=0 c5d_s5:--seed=5 c5m0_s5:--seed=5,--env=solver.self_manifold=0 c5d_s6:--seed=6 c5m0_s6:--seed=6,--env=solver.self_manifold=0" ;;
  *) echo "PART?"; exit 2 ;;
esac
NUM_ENVS=32768 ITERS=1000 RUNS="$RUNS" bash scripts/gpu_standup_ablate.sh
