#!/bin/bash
set -o pipefail
O=gpurun_out/r6zj; mkdir -p $O
for r in 1 2 3; do
for n in head fcbmr1 fc1mr1; do
  if [ $n = head ]; then e=""; else e="MNIST_AMD_EXT_PATH=$PWD/tools/so/$n.so"; fi
  env $e timeout -k 10 240 python bench.py --no-full-run --steps 600 --warmup 50 > $O/${n}_$r.log 2>&1 || { tail -5 $O/${n}_$r.log; exit 1; }
  echo "$n $r $(tail -1 $O/${n}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000, 2), d.get("last_train_loss"))')" | tee -a $O/summary.txt
done
done
