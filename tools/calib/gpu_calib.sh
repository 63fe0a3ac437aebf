#!/usr/bin/env bash
# rocprofv3 FETCH_SIZE / WRITE_SIZE passes over the calibration kernels (GPU box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out/calib; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/calib/$c -o run -- python3 tools/calib/run_calib.py 65536 84 > gpurun_out/calib/$c.log 2>&1 || { tail -5 gpurun_out/calib/$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/calib/{c}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(c, k, "KiB per dispatch (mean of last 4):", sum(v[1:]) / max(1, len(v[1:])), "known KiB:", 65536 * 84 * 4 / 1024)
PY
