#!/bin/bash
# GPU session: farmer cm=10 (generic path) + aircond
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --cm 10 --scens 1000 --steps 5 --warmup 1 > gpurun_out/bench16_cm10.log 2>&1 || { echo "BENCH CM10 FAILED"; tail -30 gpurun_out/bench16_cm10.log; exit 1; }
tail -1 gpurun_out/bench16_cm10.log | cut -c1-1500
