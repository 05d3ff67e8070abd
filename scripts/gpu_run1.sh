#!/bin/bash
# round-1 GPU session 1: parity tests, smoke, short bench, kernel-trace profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1 || true
nproc > gpurun_out/host_info.txt; lscpu | grep "Model name" >> gpurun_out/host_info.txt
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -50 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-sample 200 > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1 || { echo "PROF FAILED"; tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof1.log"; exit 1; }
echo PROF_OK
