#!/bin/bash
# Round evidence for the fused device loop: bench (with CPU baseline and time to conv),
# rocprof kernel stats, HBM + SQ PMC passes of the same bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --conv > gpurun_out/bench20.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench20.log; exit 1; }
tail -1 gpurun_out/bench20.log | cut -c1-600
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof20 -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof20.log 2>&1 || { echo "PROF FAILED"; tail -30 $R/gpurun_out/prof20.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc20_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc20_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -20 $R/gpurun_out/pmc20_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc20_write -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc20_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -20 $R/gpurun_out/pmc20_write.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv -d $R/gpurun_out/pmc20_sq -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc20_sq.log 2>&1 || { echo "PMC SQ FAILED"; tail -20 $R/gpurun_out/pmc20_sq.log; exit 1; }
cd $R
for k in phx_lane_warm phx_lane_cold k_xbar k_update_w_seg; do python scripts/pmc_summary.py $k gpurun_out/pmc20_fetch gpurun_out/pmc20_write gpurun_out/pmc20_sq > gpurun_out/pmc20_$k.json; done
python scripts/prof_summary.py gpurun_out/prof20 | head -14
cat gpurun_out/pmc20_phx_lane_warm.json
