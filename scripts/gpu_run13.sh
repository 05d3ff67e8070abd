#!/bin/bash
# GPU session: parity tests (incl. Xhat_Eval / nonant fixing) + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu13.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu13.log; exit 1; }
tail -3 gpurun_out/pytest_gpu13.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench13.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench13.log; exit 1; }
tail -1 gpurun_out/bench13.log
