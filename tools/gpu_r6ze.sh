#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab_hr
bash tools/ab_ext.sh hr "hr1 hr2" --steps 600 --warmup 50 | tee gpurun_out/ab_hr/summary.txt
