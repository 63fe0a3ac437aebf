#!/usr/bin/env bash
# rocprofv3 passes on bench.py (kernel trace + stats; then separate PMC passes, never combined
# with tracing domains). Outputs under gpurun_out/prof_<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="bench.py --steps ${PSTEPS:-100} --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-}"
step() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  echo "== $n"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -n 2 $OUT/$n.log
  if [ $rc -ne 0 ]; then echo "stop ($n rc=$rc)"; exit $rc; fi
}
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $B
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $B
step pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 $B
step pmc_sq2 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq2 -o run -- python3 $B
find $OUT -name "*.csv" | head -30
