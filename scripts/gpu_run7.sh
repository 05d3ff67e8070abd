#!/bin/bash
# GPU session: parity tests, smoke, bench (warm active set on/off), kernel-trace profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], {k:round(v,3) for k,v in d['kernel_ms_per_step'].items()}, d['pdhg_iters_per_step'], d['lane_certified_per_step'], d['lane_warm_certified_per_step'], 'notopt', d['not_optimal'], 'iter0_s %.2f setup_s %.2f' % (d['iter0_s'], d['setup_s']))"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu7.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu7.log; exit 1; }
tail -3 gpurun_out/pytest_gpu7.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke7.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke7.log; exit 1; }
tail -1 gpurun_out/smoke7.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench7_warm.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench7_warm.log; exit 1; }
summ gpurun_out/bench7_warm.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof7 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof7.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof7.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py gpurun_out/prof7 | head -16
