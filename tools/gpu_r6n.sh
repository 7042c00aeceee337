#!/bin/bash
# wgrad group cap (conv2 slab count) A/B: single GPU and world-1 XGMI, B = 200
set -o pipefail
O=gpurun_out/r6n; mkdir -p $O
W1="python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --allreduce xgmi --steps 600 --warmup 50 --no-full-run"
for i in 1 2; do
  for v in head wg128 wg192; do
    if [ $v = head ]; then e=""; else e="MNIST_AMD_EXT_PATH=$PWD/tools/so/$v.so"; fi
    env $e timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/single_${v}_$i.log 2>&1 || { tail -20 $O/single_${v}_$i.log; exit 1; }
    env $e timeout -k 10 300 $W1 > $O/xgmi_${v}_$i.log 2>&1 || { tail -20 $O/xgmi_${v}_$i.log; exit 1; }
    echo "$v $i single $(tail -1 $O/single_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2), d.get("last_train_loss"))') xgmi $(tail -1 $O/xgmi_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2), d["config"].get("allreduce"))')" | tee -a $O/ab_summary.txt
  done
done
