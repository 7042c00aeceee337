#!/bin/bash
set -o pipefail
bash tools/gpu_profiles.sh r6final4 > /dev/null 2>&1 || { echo profiles failed; exit 1; }
timeout -k 10 300 python tools/timeline_tl.py --steps 300 --graph-steps 50 --out gpurun_out/r6final4/timeline_b200.md > gpurun_out/r6final4/tl.log 2>&1 || { tail -20 gpurun_out/r6final4/tl.log; exit 1; }
head -20 gpurun_out/r6final4/roofline_b200.md; sed -n 3,20p gpurun_out/r6final4/timeline_b200.md
