set -o pipefail
bash scripts/gpu_job.sh "py:r02_s14_wall:scripts/iter0_wall.py"
