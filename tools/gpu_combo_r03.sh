set -o pipefail
bash tools/gpu_pn.sh r03m && bash tools/gpu_share_ab.sh r03n
