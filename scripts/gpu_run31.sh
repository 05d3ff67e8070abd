#!/bin/bash
# netdes GPU parity + full GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_netdes.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r31_netdes.log 2>&1 || { tail -40 gpurun_out/r31_netdes.log; exit 1; }
tail -5 gpurun_out/r31_netdes.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r31_gpu_all.log 2>&1 || { tail -40 gpurun_out/r31_gpu_all.log; exit 1; }
tail -5 gpurun_out/r31_gpu_all.log
