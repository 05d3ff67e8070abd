set -o pipefail
bash scripts/gpu_job.sh "py:r02_s11_first:scripts/probe_first.py" "py:r02_s11_wall:scripts/iter0_wall.py" \
  "bench:r02_s11_c5b:--only C5b --no-cpu-baseline --no-conv --steps 10 --warmup 1" \
  "pmc:r02_s11_c5b_fetch:FETCH_SIZE:--only C5b --no-cpu-baseline --no-conv --steps 10 --warmup 1" \
  "pmc:r02_s11_c5b_write:WRITE_SIZE:--only C5b --no-cpu-baseline --no-conv --steps 10 --warmup 1"
