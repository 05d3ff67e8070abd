set -o pipefail
B="--configs none --no-cpu-baseline --no-conv --steps 50"
bash scripts/gpu_job.sh "py:r02_s19_smoke:scripts/run_smoke.py" "test:tests" "bench:r02_s19_bench:" \
  "prof:r02_s19_prof:$B"
