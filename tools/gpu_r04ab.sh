#!/bin/bash
# Chain-kernel scheduler-strategy A/B (pointnet TU built with -amdgpu-sched-strategy=...).
set -o pipefail
bash tools/ab_variants.sh r04ab base s_max-ilp s_max-memory-clause s_iterative-ilp base
