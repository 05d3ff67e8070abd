#!/bin/bash
# GPU session: parity tests, bench at 1 and 2 waves/SIMD for the warm lane kernel, kernel-trace profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], {k:round(v,3) for k,v in d['kernel_ms_per_step'].items()}, d['lane_warm_certified_per_step'][:3], 'notopt', d['not_optimal'])"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu8.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu8.log; exit 1; }
tail -2 gpurun_out/pytest_gpu8.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench8_w1.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench8_w1.log; exit 1; }
summ gpurun_out/bench8_w1.log
PHX_LANE_WAVES=2 timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench8_w2.log 2>&1 || { echo "BENCH2 FAILED"; tail -30 gpurun_out/bench8_w2.log; exit 1; }
summ gpurun_out/bench8_w2.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof8.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof8.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py gpurun_out/prof8 | head -14
