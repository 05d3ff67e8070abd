#!/bin/bash
# GPU session: bench (with CPU baseline), kernel-trace stats, counter list, HBM PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu9.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu9.log; exit 1; }
tail -1 gpurun_out/pytest_gpu9.log
timeout -k 10 600 python bench.py > gpurun_out/bench9.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench9.log; exit 1; }
tail -1 gpurun_out/bench9.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof9 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof9.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof9.log; exit 1; }
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt 2>&1 || echo "LIST FAILED (ignored)"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc9_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc9_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc9_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc9_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc9_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc9_write.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py gpurun_out/prof9 | head -8
ls gpurun_out/pmc9_fetch gpurun_out/pmc9_write
