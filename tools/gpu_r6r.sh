#!/bin/bash
# fc1 K-split A/B (16 / 32 / 48 chunks), B = 200, 600 steps, same box interleaved
set -o pipefail
mkdir -p gpurun_out/ab_ks
bash tools/ab_ext.sh ks "ks16 ks48" --steps 600 --warmup 50 | tee gpurun_out/ab_ks/summary.txt
