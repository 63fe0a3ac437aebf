#!/usr/bin/env bash
# GPU box session: smoke, GPU tests, short bench, kernel-trace profile. Each step has its own time
# limit; a crash / fault / timeout (exit not in {0,1}) stops the script so nothing else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,pytest,bench,prof}
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *pytest* ]] && run pytest_gpu 900 python -m pytest tests -m gpu -x -q
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps ${BENCH_STEPS:-300} --warmup 30
[[ $STEPS == *prof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline
exit 0
