set -o pipefail
B="--configs none --no-cpu-baseline --no-conv --steps 50"
bash scripts/gpu_job.sh "test:tests" "bench:r02_s10_bench:" "prof:r02_s10_prof:$B" \
  "pmc:r02_s10_pmc_fetch:FETCH_SIZE:$B" "pmc:r02_s10_pmc_write:WRITE_SIZE:$B"
