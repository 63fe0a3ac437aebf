#!/usr/bin/env bash
# A/B of runtime knobs (environment variables read at zb_create) on the default bench line:
# each argument is one case "VAR=val VAR2=val [-- bench args]"; ROUNDS interleaved rounds.
# Usage: gpurun -- bash scripts/gpu_env_ab.sh <tag> "ZB_SPLIT=0" "ZB_SPLIT=1 -- --no-self-collision" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; TAG=${1:-envab}; shift; O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for c in "$@"; do
    envs="${c%% -- *}"; args=""; [[ "$c" == *" -- "* ]] && args="${c#* -- }"
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline $args > $O/b.log 2>&1 || { echo "failed: $c"; tail -5 $O/b.log; exit 1; }
    python -c "import json,sys;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print('%-48s r%s value %.4e ms/step %.4f kernel_ms %.4f'%(sys.argv[1],sys.argv[2],d['value'],d['ms_per_step'],d['roofline']['kernel_ms']))" "$c" $r | tee -a $O/summary.txt
  done
done
