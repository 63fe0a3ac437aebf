#!/usr/bin/env bash
# LDS diet (20 KB per workgroup -> 2 waves per SIMD): GPU parity of the 2-wave build, then A/B of
# old (35.9 KB, 1 wave) / new layout with 1-wave bounds / new layout with 2-wave bounds over env counts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
ZBOT_LIB=libzbot_w2.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/test_w2.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/test_w2.log; exit 1; }
tail -2 gpurun_out/test_w2.log
for cfg in "walking 4096" "walking 8192" "walking 65536" "standup 32768" "manager 8192" "v4 8192"; do
  set -- $cfg
  for lib in libzbot_old.so libzbot.so libzbot_w2.so; do
    ZBOT_LIB=$lib timeout -k 10 200 python bench.py --task $1 --envs-per-gpu $2 --steps 300 --warmup 30 --no-cpu-baseline \
      > gpurun_out/ab.log 2>&1 || { echo "$lib $cfg failed"; tail -5 gpurun_out/ab.log; exit 1; }
    python -c "import json,sys;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);print('%-16s %-8s %6s value %.4e  ms/step %.4f  kernel_ms %.4f'%(sys.argv[1],sys.argv[2],sys.argv[3],d['value'],d['ms_per_step'],d['roofline']['kernel_ms']))" $lib $1 $2
  done
done
