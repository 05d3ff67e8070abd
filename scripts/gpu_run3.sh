#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu3.log 2>&1 || { echo "PYTEST FAILED"; tail -50 gpurun_out/pytest_gpu3.log; exit 1; }
tail -2 gpurun_out/pytest_gpu3.log
for A in 0 128 256 512; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --ipm-after $A > gpurun_out/bench3_ipm$A.log 2>&1 || { echo "BENCH $A FAILED"; tail -30 gpurun_out/bench3_ipm$A.log; exit 1; }
  tail -1 gpurun_out/bench3_ipm$A.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($A, 'value %.4g' % d['value'], 'ms/step %.2f' % d['ms_per_step'], {k:round(v,2) for k,v in d['kernel_ms_per_step'].items()}, d['pdhg_iters_per_step'], 'frac %.3f' % d['roofline']['frac'], 'avg_us %.0f' % d['roofline']['avg_launch_us'], 'notopt', d['not_optimal'])"
done
