#!/bin/bash
# Bench several env settings back to back on the GPU box (each twice, interleaved).
# usage: bash tools/ab_multi.sh TAG "ENV1=a ENV2=b" "ENV1=c" ... -- [bench args...]
T=$1; shift
cfgs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do cfgs+=("$1"); shift; done
[ "$1" = "--" ] && shift
set -o pipefail
for rep in 1 2; do
  i=0
  for c in "${cfgs[@]}"; do
    i=$((i+1))
    env $c timeout -k 10 200 python bench.py --no-full-run "$@" > gpurun_out/abm_${T}_${i}_$rep.log 2>&1 || { tail -20 gpurun_out/abm_${T}_${i}_$rep.log; exit 1; }
    echo "$T [$c] $(tail -1 gpurun_out/abm_${T}_${i}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("last_train_loss"))')"
  done
done
