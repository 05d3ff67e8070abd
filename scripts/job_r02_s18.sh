set -o pipefail
bash scripts/gpu_job.sh "py:r02_s18_wgrounds:scripts/probe_wg_rounds.py"
