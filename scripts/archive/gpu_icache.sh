#!/usr/bin/env bash
# Instruction-cache / translation PMC passes on bench.py (one rocprofv3 --pmc pass per counter set,
# no tracing domains), for each library given: LIBS="libzbot.so libzbot_lnk.so" bash scripts/gpu_icache.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
O=gpurun_out/icache; mkdir -p $O
B="bench.py --steps 100 --warmup 10 --no-cpu-baseline"
for L in ${LIBS:-libzbot.so}; do
  export ZBOT_LIB=$L
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY --output-format csv -d $O/${L%.so}_ic -o run -- python3 $B > $O/${L%.so}_ic.log 2>&1 || { echo "ic $L failed"; tail -5 $O/${L%.so}_ic.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_STALL_MULTI_MISS_sum --output-format csv -d $O/${L%.so}_tlb -o run -- python3 $B > $O/${L%.so}_tlb.log 2>&1 || { echo "tlb $L failed"; tail -5 $O/${L%.so}_tlb.log; exit 1; }
done
echo done
