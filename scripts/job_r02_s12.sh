set -o pipefail
A="--no-cpu-baseline --no-conv --steps 10 --warmup 1"
bash scripts/gpu_job.sh \
  "pmc:r02_s12_c2_fetch:FETCH_SIZE:--only C2 $A" "pmc:r02_s12_c2_write:WRITE_SIZE:--only C2 $A" \
  "pmc:r02_s12_c5a_fetch:FETCH_SIZE:--only C5a $A" "pmc:r02_s12_c5a_write:WRITE_SIZE:--only C5a $A" \
  "pmc:r02_s12_c4_fetch:FETCH_SIZE:--only C4 $A" "pmc:r02_s12_c4_write:WRITE_SIZE:--only C4 $A"
