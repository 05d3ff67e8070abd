#!/bin/bash
# GPU session: bench + kernel/memory-copy trace timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'], {k:round(v,4) for k,v in d['kernel_ms_per_step'].items()}, 'notopt', d['not_optimal'])"; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu12.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu12.log; exit 1; }
tail -1 gpurun_out/pytest_gpu12.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench12.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench12.log; exit 1; }
summ gpurun_out/bench12.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof12 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof12.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof12.log; exit 1; }
ls $GRAFT_REPO_ROOT/gpurun_out/prof12
