set -o pipefail
B="--configs none --no-cpu-baseline --no-conv --steps 50"
O="--configs none --no-cpu-baseline --no-conv --steps 20 --warmup 1 --scens 1000000"
bash scripts/gpu_job.sh "test:tests/test_gpu_parity.py -k workgroup" "bench:r02_s9_c2:--only C2 --no-cpu-baseline --no-conv --steps 20" \
  "bench:r02_s9_w2:$B" && PHX_LANE_WAVES=1 bash scripts/gpu_job.sh "bench:r02_s9_w1:$B" && \
  bash scripts/gpu_job.sh "bench:r02_s9_1m:$O" "pmc:r02_s9_pmc1m_fetch:FETCH_SIZE:$O" "pmc:r02_s9_pmc1m_write:WRITE_SIZE:$O"
