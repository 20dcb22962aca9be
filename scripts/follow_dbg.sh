set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests bench full3
