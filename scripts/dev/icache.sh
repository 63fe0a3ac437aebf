#!/usr/bin/env bash
# instruction-fetch counters of the step kernel (diagnostic)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out/ic; export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/ic/avail.txt 2>&1
grep -o -E "SQC?_[A-Z_]*(ICACHE|IFETCH|INST_LEVEL|WAIT_INST)[A-Z_]*" gpurun_out/ic/avail.txt | sort -u
CTRS=$(grep -o -E "SQC?_[A-Z_]*(ICACHE|IFETCH)[A-Z_]*" gpurun_out/ic/avail.txt | sort -u | grep -v -E "_sum|_avr|_min|_max" | head -4 | tr '\n' ' ')
echo "counters: $CTRS"
timeout -s KILL 120 rocprofv3 --pmc $CTRS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/ic/pmc -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/ic/pmc.log 2>&1 || { tail -5 gpurun_out/ic/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/ic/pmc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "zb_step_kernel" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, sum(v) / len(v) if v else 0, len(v))
PY
