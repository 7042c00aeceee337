#!/bin/bash
# A/B an env knob on the GPU box: bench.py --no-full-run at two knob values, alternating (4 runs).
# usage: bash tools/ab_knob.sh TAG KNOB A B [bench args...]
T=$1; K=$2; VA=$3; VB=$4; shift 4
set -o pipefail
for v in $VA $VB $VA $VB; do
  env $K=$v timeout -k 10 200 python bench.py --no-full-run "$@" > gpurun_out/ab_${T}_$v.log 2>&1 || { tail -20 gpurun_out/ab_${T}_$v.log; exit 1; }
  echo "$T $K=$v $(tail -1 gpurun_out/ab_${T}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
