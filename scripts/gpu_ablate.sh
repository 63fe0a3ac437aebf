#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for a in "" "--solver-iterations 4" "--solver-iterations 0" "--no-self-collision" "--solver-iterations 0 --no-self-collision" "--envs-per-gpu 8192" "--envs-per-gpu 16384" "--envs-per-gpu 65536 --steps 50"; do
  echo "== $a"
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline $a > gpurun_out/abl.log 2>&1 || { echo fail; tail -5 gpurun_out/abl.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abl.log').read().strip().splitlines()[-1]);print('  value %.3e  ms/step %.3f  kernel_ms %.3f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms']))"
done
