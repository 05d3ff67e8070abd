#!/bin/bash
# workgroup warm pass (k_wg_warm): GPU parity (cm10 1000, sslp), then the farmer cm=10 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "cm10 or sslp or farmer3_golden" --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu22.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu21.log; exit 1; }
tail -6 gpurun_out/pytest_gpu22.log
timeout -k 10 300 python bench.py --no-cpu-baseline --cm 10 --scens 1000 --steps 20 --warmup 3 > gpurun_out/bench22_cm10.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench22_cm10.log; exit 1; }
tail -1 gpurun_out/bench22_cm10.log | cut -c1-2500
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof22 -o run -- python3 $R/bench.py --no-cpu-baseline --cm 10 --scens 1000 --steps 20 --warmup 3 > $R/gpurun_out/prof22.log 2>&1 || { echo "PROF FAILED"; tail -30 $R/gpurun_out/prof22.log; exit 1; }
cd $R
python scripts/prof_summary.py gpurun_out/prof22 | head -14
