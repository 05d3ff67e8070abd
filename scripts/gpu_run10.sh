#!/bin/bash
# GPU session: refine-loop A/B, SQ + SQC (icache) counters for phx_lane_warm
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'], {k:round(v,4) for k,v in d['kernel_ms_per_step'].items()}, 'notopt', d['not_optimal'])"; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu10.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu10.log; exit 1; }
tail -1 gpurun_out/pytest_gpu10.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench10_loop.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench10_loop.log; exit 1; }
summ gpurun_out/bench10_loop.log
PHX_LANE_DEFS=PHX_REFINE_UNROLL timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench10_unroll.log 2>&1 || { echo "BENCH2 FAILED"; tail -30 gpurun_out/bench10_unroll.log; exit 1; }
summ gpurun_out/bench10_unroll.log
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_SALU SQ_IFETCH --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc10_sq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc10_sq.log 2>&1 || { echo "PMC SQ FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc10_sq.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc10_ic -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc10_ic.log 2>&1 || { echo "PMC IC FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc10_ic.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/pmc_summary.py phx_lane_warm gpurun_out/pmc10_sq gpurun_out/pmc10_ic
