set -o pipefail
bash tools/gpu_pn_ab.sh r03q stamps stamps_nb2 stamps stamps_nb2 && bash tools/gpu_trace_pipe.sh r03p_trace --steps 40
