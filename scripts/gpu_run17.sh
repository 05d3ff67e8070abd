#!/bin/bash
# GPU session: bench + rocprof kernel stats + HBM PMC passes for the round's profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench17.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench17.log; exit 1; }
tail -1 gpurun_out/bench17.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof17 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof17.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof17.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc17_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc17_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc17_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc17_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc17_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc17_write.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc17_sq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc17_sq.log 2>&1 || { echo "PMC SQ FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc17_sq.log; exit 1; }
cd $GRAFT_REPO_ROOT
for k in phx_lane_warm phx_lane_cold k_xbar k_update_w_seg; do python scripts/pmc_summary.py $k gpurun_out/pmc17_fetch gpurun_out/pmc17_write gpurun_out/pmc17_sq > gpurun_out/pmc17_$k.json; done
python scripts/prof_summary.py gpurun_out/prof17 | head -12
cat gpurun_out/pmc17_phx_lane_warm.json
