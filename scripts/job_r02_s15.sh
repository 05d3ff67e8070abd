set -o pipefail
bash scripts/gpu_job.sh "py:r02_s15_hostops:scripts/probe_host_ops.py"
