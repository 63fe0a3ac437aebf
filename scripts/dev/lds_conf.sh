#!/usr/bin/env bash
# LDS bank-conflict / LDS-issue counters for two builds (diagnostic): bash scripts/dev/lds_conf.sh libA.so libB.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out/lds; export TMPDIR=/tmp
for L in "$@"; do
  for T in walking manager; do
    ZBOT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/lds/$L.$T -o run -- python3 bench.py --task $T --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/lds/$L.$T.log 2>&1 || { tail -5 gpurun_out/lds/$L.$T.log; exit 1; }
    python3 - "$L" "$T" <<'PY'
import csv, glob, collections, sys
f = glob.glob(f"gpurun_out/lds/{sys.argv[1]}.{sys.argv[2]}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "_step_kernel" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
w = m["SQ_WAVES"]
print(sys.argv[1], sys.argv[2], {k: round(v / w) for k, v in m.items() if k != "SQ_WAVES"})
PY
  done
done
