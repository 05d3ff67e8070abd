#!/bin/bash
# GPU session: parity tests (incl. phx_iterk) + bench (device-driven loop and host loop) + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu15.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu15.log; exit 1; }
tail -3 gpurun_out/pytest_gpu15.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench15.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench15.log; exit 1; }
tail -1 gpurun_out/bench15.log | cut -c1-400
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/bench15_200.log 2>&1 || { echo "BENCH200 FAILED"; tail -30 gpurun_out/bench15_200.log; exit 1; }
tail -1 gpurun_out/bench15_200.log | cut -c1-400
timeout -k 10 300 python bench.py --no-cpu-baseline --host-loop > gpurun_out/bench15_host.log 2>&1 || { echo "BENCH HOST FAILED"; tail -30 gpurun_out/bench15_host.log; exit 1; }
tail -1 gpurun_out/bench15_host.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof15 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof15.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof15.log; exit 1; }
ls $GRAFT_REPO_ROOT/gpurun_out/prof15
