#!/bin/bash
# k_wg_warm with folded begin-solve/finalize: generic-path parity tests, cm=10 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "cm10 or sslp or fixed or xhat or generic or farmer3" --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu30.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu30.log; exit 1; }
tail -3 gpurun_out/pytest_gpu30.log
timeout -k 10 300 python bench.py --no-cpu-baseline --cm 10 --scens 1000 --steps 20 --warmup 3 > gpurun_out/bench30_cm10.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench30_cm10.log; exit 1; }
tail -1 gpurun_out/bench30_cm10.log | cut -c1-300
