#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu2.log 2>&1 || { echo "PYTEST FAILED"; tail -50 gpurun_out/pytest_gpu2.log; exit 1; }
tail -2 gpurun_out/pytest_gpu2.log
for A in 256 0 1024; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --ipm-after $A > gpurun_out/bench2_ipm$A.log 2>&1 || { echo "BENCH $A FAILED"; tail -30 gpurun_out/bench2_ipm$A.log; exit 1; }
  tail -1 gpurun_out/bench2_ipm$A.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($A, 'value %.4g' % d['value'], 'ms/step %.2f' % d['ms_per_step'], d['kernel_ms_per_step'], d['pdhg_iters_per_step'], 'frac %.3f' % d['roofline']['frac'], 'notopt', d['not_optimal'])"
done
