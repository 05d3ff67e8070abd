#!/bin/bash
# Round-end evidence: full GPU test suite, headline bench (CPU baseline + time to conv),
# farmer cm=10 x1000 bench (workgroup path, CPU baseline), rocprof kernel stats of the cm=10 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu29.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu29.log; exit 1; }
tail -3 gpurun_out/pytest_gpu29.log
timeout -k 10 400 python bench.py --conv > gpurun_out/bench29.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench29.log; exit 1; }
tail -1 gpurun_out/bench29.log | cut -c1-300
timeout -k 10 400 python bench.py --cm 10 --scens 1000 --steps 20 --warmup 3 --cpu-scens 2000 > gpurun_out/bench29_cm10.log 2>&1 || { echo "BENCH CM10 FAILED"; tail -30 gpurun_out/bench29_cm10.log; exit 1; }
tail -1 gpurun_out/bench29_cm10.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof29 -o run -- python3 $R/bench.py --no-cpu-baseline --cm 10 --scens 1000 --steps 20 --warmup 3 > $R/gpurun_out/prof29.log 2>&1 || { echo "PROF FAILED"; tail -30 $R/gpurun_out/prof29.log; exit 1; }
cd $R
python scripts/prof_summary.py gpurun_out/prof29 | head -12
