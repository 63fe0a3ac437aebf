#!/usr/bin/env bash
# A/B of kernel build variants (zbot_lab_amd/lib*.so built here with `python -m zbot_lab_amd.build
# -D... --out=<lib>`): the default bench line per variant, ROUNDS interleaved rounds.
# Usage: gpurun -- bash scripts/gpu_variants.sh <tag> libzbot.so libzbot_x.so ... [-- bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; TAG=${1:-var}; shift; O=gpurun_out/$TAG; mkdir -p $O
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done; [ "${1:-}" = "--" ] && shift
for r in $(seq ${ROUNDS:-3}); do
  for L in "${LIBS[@]}"; do
    ZBOT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || { echo "failed: $L"; tail -5 $O/b.log; exit 1; }
    tail -1 $O/b.log >> $O/lines_$L.jsonl
    python -c "import json,sys;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print('%-22s round %s value %.4e ms/step %.4f kernel_ms %.4f'%(sys.argv[1],sys.argv[2],d['value'],d['ms_per_step'],d['roofline']['kernel_ms']))" $L $r | tee -a $O/summary.txt
  done
done
