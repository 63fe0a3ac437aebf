#!/usr/bin/env bash
# Round-4 GPU evidence: the whole GPU suite (-s: the parity tables), then the PPO training A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r4c}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/test_gpu.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/test_gpu.log | tail -8
grep -E "fused vs torch" $O/test_gpu.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_train_profile.sh ${T}_tp_fused 4096 zbot-6b-walking-v2 1
