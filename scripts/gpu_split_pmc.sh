#!/usr/bin/env bash
# PMC passes (instruction cache; VALU issue / waits) on the walking bench, ZB_SPLIT=0 vs 1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
O=gpurun_out/split_pmc; mkdir -p $O
B="bench.py --steps 100 --warmup 10 --no-cpu-baseline"
for v in 0 1; do
  export ZB_SPLIT=$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY --output-format csv -d $O/ic$v -o run -- python3 $B > $O/ic$v.log 2>&1 || { echo "ic $v failed"; tail -5 $O/ic$v.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq$v -o run -- python3 $B > $O/sq$v.log 2>&1 || { echo "sq $v failed"; tail -5 $O/sq$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, statistics, collections
for v in (0, 1):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/split_pmc/*{v}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "zb_step" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"ZB_SPLIT={v}: " + ", ".join(f"{k} {statistics.mean(x):.4g}" for k, x in sorted(vals.items())))
PY
