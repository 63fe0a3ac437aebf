#!/usr/bin/env bash
# PMC passes on the fused PPO kernels at C5 (+ a kernel trace of the LDS row kernels, ZBP_ROWS=lds) (zbot-6b-standup-v0, 32768 envs, its PPO cfg; VERDICT r4
# item 5): kernel trace + stats, then one rocprofv3 --pmc pass per counter group restricted to the
# PPO kernels (k_rows / k_wgrad / k_act / k_reduce). Counter names are taken from `rocprofv3 -L`
# on the box; a name the box does not list is dropped from its pass.
# Usage: gpurun -- bash scripts/gpu_r5_ppo_pmc.sh <tag> [num_envs] [task]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; T=${1:-r5_ppo_pmc}; N=${2:-32768}; TASK=${3:-zbot-6b-standup-v0}
O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
TRAIN="scripts/train.py --task $TASK --num_envs $N --max_iterations 3 --seed 42"
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || { tail -3 $O/counters.txt; exit 1; }
have() { grep -qw "$1" $O/counters.txt; }
pick() { local out=""; for c in "$@"; do have $c && out="$out $c"; done; echo $out; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $TRAIN \
  --log_root $O/logs_trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
ZBP_ROWS=lds timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_lds -o run -- python3 $TRAIN \
  --log_root $O/logs_trace_lds > $O/trace_lds.log 2>&1 || { tail -5 $O/trace_lds.log; exit 1; }
KR='k_(rows|wgrad|act|reduce)'
pass() {  # name counters...
  local n=$1; shift
  local cs=$(pick "$@")
  [ -z "$cs" ] && { echo "pass $n: no counters"; return 0; }
  echo "== $n: $cs"
  timeout -s KILL 240 rocprofv3 --pmc $cs --kernel-include-regex "$KR" --output-format csv -d $O/$n -o run -- \
    python3 $TRAIN --log_root $O/logs_$n > $O/$n.log 2>&1
  local rc=$?; [ $rc -ne 0 ] && { echo "pass $n rc=$rc"; tail -3 $O/$n.log; exit $rc; }
  return 0
}
pass pmc_a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
pass pmc_b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
pass pmc_c SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM
pass pmc_d TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum
pass pmc_fetch FETCH_SIZE
pass pmc_write WRITE_SIZE
find $O -name "*counter_collection.csv" -o -name "*kernel_stats.csv" | head
