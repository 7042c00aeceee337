#!/bin/bash
# conv1 reduce + update launch: upper bounds (C1_UB=1 no reduce, 2 no hold, 3 neither), B = 200
set -o pipefail
mkdir -p gpurun_out/ab_c1ub
bash tools/ab_ext.sh c1ub "c1_ub1 c1_ub2 c1_ub3" --steps 600 --warmup 50 | tee gpurun_out/ab_c1ub/summary.txt
