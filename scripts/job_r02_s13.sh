set -o pipefail
bash scripts/gpu_job.sh "py:r02_s13_hostops:scripts/probe_host_ops.py" \
  "bench:r02_s13_bench:--configs none --no-cpu-baseline --no-conv" "py:r02_s13_wall:scripts/iter0_wall.py"
