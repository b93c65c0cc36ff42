#!/bin/bash
# Chain kernel on the 95-VGPR build: 1024/512-wide x6 layers as RB 4 x NB 1 instead of NB 2.
set -o pipefail
bash tools/ab_variants.sh r04ay base nb1 base nb1
