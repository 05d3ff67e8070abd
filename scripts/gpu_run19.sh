#!/bin/bash
# fused phx_iterk: GPU parity tests (iterk subset first), then bench fused vs unfused
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "native_loop" --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu19.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu19.log; exit 1; }
tail -3 gpurun_out/pytest_gpu19.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench19_fused.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench19_fused.log; exit 1; }
tail -1 gpurun_out/bench19_fused.log | cut -c1-400
timeout -k 10 300 python bench.py --no-cpu-baseline --fused 0 > gpurun_out/bench19_unfused.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench19_unfused.log; exit 1; }
tail -1 gpurun_out/bench19_unfused.log | cut -c1-400
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/bench19_fused200.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench19_fused200.log; exit 1; }
tail -1 gpurun_out/bench19_fused200.log | cut -c1-400
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu19_all.log 2>&1 || { echo "PYTEST ALL FAILED"; tail -60 gpurun_out/pytest_gpu19_all.log; exit 1; }
tail -3 gpurun_out/pytest_gpu19_all.log
