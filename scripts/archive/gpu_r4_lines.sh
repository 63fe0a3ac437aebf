#!/usr/bin/env bash
# Round-4: every bench line at HEAD (the default one and the other configs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r4p}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for args in "" "--envs-per-gpu 8192" "--envs-per-gpu 65536" "--task standup" "--task v4" "--task manager"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  tail -1 $O/b.log >> $O/bench_lines.jsonl
done
python -c "
import json
for l in open('$O/bench_lines.jsonl'):
    d = json.loads(l); print(d['config']['workload'][:70], round(d['value'] / 1e6, 2), 'M', round(d['ms_per_step'], 4), 'ms')"
