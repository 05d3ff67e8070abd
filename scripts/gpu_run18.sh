#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu18.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu18.log; exit 1; }
tail -3 gpurun_out/pytest_gpu18.log
grep -E "PASSED|FAILED" gpurun_out/pytest_gpu18.log | awk '{print $1}' | tail -30
