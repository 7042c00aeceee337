#!/bin/bash
set -o pipefail
O=gpurun_out/r6s; mkdir -p $O
for m in null stream null stream; do echo "== $m"; timeout -k 10 60 ./tools/exp/first_launch $m; done 2>&1 | tee $O/first_launch.txt
