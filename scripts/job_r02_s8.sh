set -o pipefail
B="--configs none --no-cpu-baseline --no-conv --steps 50"
O="--configs none --no-cpu-baseline --no-conv --steps 20 --scens 2000000"
bash scripts/gpu_job.sh "test:tests" "bench:r02_s8_bench:" "prof:r02_s8_prof:$B" \
  "pmc:r02_s8_pmc_fetch:FETCH_SIZE:$B" "pmc:r02_s8_pmc_write:WRITE_SIZE:$B" \
  "pmc:r02_s8_pmc_sq:SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU_FLOPS_FP64,SQ_INSTS_SALU:$B" \
  "bench:r02_s8_bench_2m:$O" "pmc:r02_s8_pmc2m_fetch:FETCH_SIZE:$O" "pmc:r02_s8_pmc2m_write:WRITE_SIZE:$O"
