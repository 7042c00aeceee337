#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab_hr2
for r in 1 2 3; do
for n in head hr1; do
  if [ $n = head ]; then e=""; else e="MNIST_AMD_EXT_PATH=$PWD/tools/so/$n.so"; fi
  env $e timeout -k 10 240 python bench.py --no-full-run --steps 600 --warmup 50 > gpurun_out/ab_hr2/${n}_$r.log 2>&1 || exit 1
  echo "$n $r $(tail -1 gpurun_out/ab_hr2/${n}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000, 2))')" | tee -a gpurun_out/ab_hr2/summary.txt
done
done
