#!/usr/bin/env bash
# The one GPU-box runner (replaces the per-experiment scripts/archive/gpu_r*.sh launchers).
#   gpurun --timeout 1200 -- bash scripts/gpu.sh <tag> <step> [<step> ...]
# Every step runs under its own time limit, writes gpurun_out/<tag>/<step>.log and stops the call on
# the first failure (no GPU step starts after a fault, an abort or a time limit). Steps:
#   suite            pytest -m gpu (the driver's suite) + smoke()
#   bench            the default bench line (4096 envs, with the CPU leg)
#   lines            bench lines: 4096 / 8192 / 65536 envs and the other tasks (no CPU leg)
#   solver           bench lines at solver modes $MODES (0 3) x self_manifold $SMS (2 3) x $SIZES envs
#   prof             rocprofv3 kernel trace + stats, then separate PMC passes, on bench.py; writes
#                    roofline_pmc.json (scripts/prof_summary.py)
#   parityab         the full-state parity checks once per library in $LIBS (ZB_PARITY_STATS JSONL)
#   benchab          bench lines once per library in $LIBS, interleaved $ROUNDS times
#   recipe           the staged v2 recipe test (tests/test_gpu_recipe.py)
#   tests            pytest -m gpu on $TESTS
#   budget           tools/error_budget.py (device vs f32 oracle error against f64, per part of a substep)
#   nofin            bench lines with and without the finalize launch (ZB_DIAG_NO_FINALIZE, diagnostic)
#   train            60 walking-v2 training iterations, no profiler (the fps column)
#   train_v2 / train_c5   rocprof kernel traces of short training runs
#   rehearsal        two ranks of bench.py sharing cuda:0 over gloo (plumbing, not scaling)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  echo "== $n ($(date +%T))"
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -n 3 "$O/$n.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stop ($n rc=$rc)"; exit $rc; fi
}
PT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider"
B="bench.py --steps ${PSTEPS:-100} --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-}"
for s in "$@"; do
  case $s in
    suite)
      run test_gpu 900 $PT tests -m gpu
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      run bench 400 python bench.py ;;
    lines)
      for n in 4096 8192 65536; do run bench_$n 300 python bench.py --envs-per-gpu $n --no-cpu-baseline; done
      for t in standup v4 manager; do run bench_$t 300 python bench.py --task $t --no-cpu-baseline; done ;;
    solver)
      for n in ${SIZES:-4096 8192 65536}; do for m in ${MODES:-0 3}; do for sm in ${SMS:-2 3}; do
        run solver_n${n}_m${m}_sm${sm} 300 python bench.py --envs-per-gpu $n --solver-mode $m --self-manifold $sm \
          --no-cpu-baseline
      done; done; done ;;
    prof)
      P=$O/prof
      run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $B
      run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch -o run -- python3 $B
      run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write -o run -- python3 $B
      run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES \
        SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $P/pmc_sq -o run -- python3 $B
      run pmc_sq2 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
        SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $P/pmc_sq2 -o run -- python3 $B
      run prof_summary 120 python scripts/prof_summary.py $P --out $O/roofline_pmc.json ;;
    parityab)
      for lib in ${LIBS:-libzbot.so}; do  # (a red check is a result here; a fault / abort / time limit stops)
        ZBOT_LIB=$lib ZB_PARITY_STATS=$O/parity_stats.jsonl timeout -k 10 900 python -u -m pytest -v -s \
          --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullstate.py \
          tests/test_gpu_fullsize.py -m gpu > "$O/parity_${lib%.so}.log" 2>&1; rc=$?
        echo "   $lib rc=$rc $(tail -n 1 $O/parity_${lib%.so}.log)"
        if [ $rc -gt 1 ]; then echo "stop (parity $lib rc=$rc)"; exit $rc; fi
      done
      python scripts/parity_ab.py $O/parity_stats.jsonl > $O/parity_ab.txt; cat $O/parity_ab.txt ;;
    benchab)
      for r in $(seq ${ROUNDS:-2}); do for lib in ${LIBS:-libzbot.so}; do for n in 4096 8192; do
        run benchab_${lib%.so}_${n}_$r 300 env ZBOT_LIB=$lib python bench.py --envs-per-gpu $n --no-cpu-baseline
      done; done; done ;;
    nofin)  # diagnostic: the step without its finalize launch (wrong episode log; the launch's share)
      for r in 1 2; do for n in 4096 8192; do
        run nofin_${n}_$r 300 python bench.py --envs-per-gpu $n --no-cpu-baseline
        run nofin_diag_${n}_$r 300 env ZB_DIAG_NO_FINALIZE=1 python bench.py --envs-per-gpu $n --no-cpu-baseline
      done; done ;;
    recipe)
      run recipe 900 $PT tests/test_gpu_recipe.py -m gpu ;;
    tests)
      run tests 900 $PT ${TESTS:?TESTS=<pytest paths>} -m gpu ;;
    budget)
      for lib in ${LIBS:-libzbot.so}; do run error_budget_${lib%.so} 300 env ZBOT_LIB=$lib python tools/error_budget.py 2048; done ;;
    train)  # plain (no profiler) walking-v2 training throughput, 60 iterations
      run train 400 python scripts/train.py --task zbot-6b-walking-v2 --num_envs 4096 --max_iterations 60 \
        --log_root $O/train_logs ;;
    train_v2)
      run train_v2 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train_v2 -o run -- \
        python3 scripts/train.py --task zbot-6b-walking-v2 --num_envs 4096 --max_iterations 30 \
        --log_root $O/train_v2_logs ;;
    train_c5)
      run train_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train_c5 -o run -- \
        python3 scripts/train.py --task zbot-6b-standup-v0 --num_envs 32768 --max_iterations 10 \
        --log_root $O/train_c5_logs ;;
    rehearsal)
      run rehearsal2 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 2 --rehearsal --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "done ($(date +%T))"
