#!/bin/bash
# GPU session: host-side step profile + HBM PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/host_profile.py > gpurun_out/host14.log 2>&1 || { echo "HOSTPROF FAILED"; tail -30 gpurun_out/host14.log; exit 1; }
head -60 gpurun_out/host14.log
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc14_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc14_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc14_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc14_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc14_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc14_write.log; exit 1; }
cd $GRAFT_REPO_ROOT
for k in phx_lane_warm k_xbar k_update_w_seg; do python scripts/pmc_summary.py $k gpurun_out/pmc14_fetch gpurun_out/pmc14_write > gpurun_out/pmc14_$k.json; done
cat gpurun_out/pmc14_phx_lane_warm.json
