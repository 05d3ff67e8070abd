set -o pipefail
bash scripts/gpu_job.sh "test:tests/test_gpu_parity.py tests/test_sslp.py tests/test_netdes.py" \
  "py:r02_s17_c2loop:scripts/probe_c2_loop.py" \
  "bench:r02_s17_c5a:--only C5a --no-cpu-baseline --no-conv --steps 10 --warmup 1"
