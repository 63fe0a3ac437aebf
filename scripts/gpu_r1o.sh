#!/usr/bin/env bash
# Diagnostic A/B: cost of the epilogue's state stores (libzbot_nost.so skips them; not a valid step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for r in 1 2; do for lib in libzbot.so libzbot_nost.so; do for n in 4096 8192; do
  ZBOT_LIB=$lib timeout -k 10 120 python bench.py --envs-per-gpu $n --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);print('%-18s %6s value %.4e  kernel_ms %.4f'%(sys.argv[1],sys.argv[2],d['value'],d['roofline']['kernel_ms']))" $lib $n
done; done; done
