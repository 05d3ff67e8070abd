#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], {k:round(v,3) for k,v in d['kernel_ms_per_step'].items()}, d['pdhg_iters_per_step'], d['lane_certified_per_step'], 'notopt', d['not_optimal'], 'iter0_s %.2f setup_s %.2f' % (d['iter0_s'], d['setup_s']))"; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu4.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu4.log; exit 1; }
tail -2 gpurun_out/pytest_gpu4.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke4.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke4.log; exit 1; }
tail -3 gpurun_out/smoke4.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench4_lane.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench4_lane.log; exit 1; }
summ gpurun_out/bench4_lane.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --lane-solver 0 --ipm-after 0 > gpurun_out/bench4_nolane.log 2>&1 || { echo "BENCH2 FAILED"; tail -30 gpurun_out/bench4_nolane.log; exit 1; }
summ gpurun_out/bench4_nolane.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof4.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof4.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof4 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -20
