#!/usr/bin/env bash
# runtime ablations of the step kernel (timing attribution only; the reported line uses defaults)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
run() {
  timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline "$@" > gpurun_out/abl2.log 2>&1 || { echo "failed: $*"; tail -5 gpurun_out/abl2.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/abl2.log').read().strip().splitlines()[-1]);print('%-40s value %.4e  kernel_ms %.4f'%(' '.join(sys.argv[1:]) or 'default',d['value'],d['roofline']['kernel_ms']))" "$@"
}
run
run --solver-iterations 0
run --no-self-collision
run --solver-iterations 0 --no-self-collision
run --solver-iterations 8
run --envs-per-gpu 2048
run --envs-per-gpu 16384
run --envs-per-gpu 65536
