set -o pipefail
bash scripts/gpu_job.sh "py:r02_s16_c2loop:scripts/probe_c2_loop.py" \
  "trace:r02_s16_c2trace:--only C2 --no-cpu-baseline --no-conv --steps 20 --warmup 1"
