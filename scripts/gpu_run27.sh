#!/bin/bash
# k_wg_warm phase timing (PHX_WG_PROF=1) on farmer cm=10 x1000
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
PHX_WG_PROF=1 timeout -k 10 300 python bench.py --no-cpu-baseline --cm 10 --scens 1000 --steps 5 --warmup 3 > gpurun_out/bench26_prof.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench26_prof.log; exit 1; }
grep "wg prof" gpurun_out/bench26_prof.log | tail -6
timeout -k 10 300 python bench.py --no-cpu-baseline --cm 10 --scens 1000 --steps 20 --warmup 3 > gpurun_out/bench26_cm10.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench26_cm10.log; exit 1; }
tail -1 gpurun_out/bench26_cm10.log | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "cm10 or sslp" --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu26.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu26.log; exit 1; }
tail -3 gpurun_out/pytest_gpu26.log
