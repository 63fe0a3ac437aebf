#!/usr/bin/env bash
# Round-4 closing evidence at HEAD: the whole GPU suite (-s: parity tables), smoke, the default
# bench line with its CPU baseline, phase stamps and per-wave timing, the self-manifold bench A/B and the
# contact-cap table (scripts/contact_caps.py).
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r4_final.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r4k}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/test_gpu.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/test_gpu.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 python scripts/stamps.py > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 1; }
timeout -k 10 300 env ZBOT_LIB=libzbot_stamps_t.so python scripts/wave_times.py > $O/wave_times.log 2>&1 || { tail -5 $O/wave_times.log; exit 1; }
grep -v amdgpu.ids $O/wave_times.log | head -8
ROUNDS=2 bash scripts/gpu_env_ab.sh ${T}_ab "ZB_AB=2" "ZB_AB=1 -- --self-manifold 1" "ZB_AB=0 -- --self-manifold 0" || exit 1
timeout -k 10 500 env ZBOT_LIB=libzbot_stamps.so python scripts/contact_caps.py 4096 300 > $O/caps.jsonl 2> $O/caps.err || { tail -5 $O/caps.err; exit 1; }
cut -c1-300 $O/caps.jsonl
