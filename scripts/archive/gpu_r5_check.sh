#!/usr/bin/env bash
# After a timing / PPO change: the fused PPO tests, the default bench line and its rocprofv3 kernel
# trace (the in-process kernel time against rocprof's), and a C5 training kernel trace.
# Usage: gpurun --timeout 900 -- bash scripts/gpu_r5_check.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_check}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_ppo_multirank.py tests/test_gpu_parity.py -m gpu -q \
  --timeout 150 --timeout-method thread > $O/test.log 2>&1 || { tail -15 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline \
  > $O/bench_prof.log 2>&1 || { tail -5 $O/bench_prof.log; exit 1; }
python3 - $O <<'PY'
import csv, json, sys
o = sys.argv[1]
k = [r for r in csv.DictReader(open(f"{o}/trace/run_kernel_stats.csv")) if "zb_step_kernel" in r["Name"]][0]
b = json.loads(open(f"{o}/bench_prof.log").read().strip().splitlines()[-1])
print("rocprof zb_step_kernel avg us", round(float(k["AverageNs"]) / 1e3, 1), "| bench in-process us", round(b["roofline"]["kernel_ms"] * 1e3, 1))
PY
bash scripts/gpu_train_profile.sh ${T}_c5 32768 zbot-6b-standup-v0
