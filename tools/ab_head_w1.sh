#!/bin/bash
# HEAD: OVERLAP 600 steps x 2, the driver's window, XGMI / RCCL world-1 600 steps x 3 / x 1
O=gpurun_out/hw1; mkdir -p $O
W1="python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --steps 600 --warmup 50 --no-full-run"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/exact.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 $W1 --allreduce xgmi > $O/xgmi_$i.log 2>&1 || exit 1
  [ $i -le 2 ] && { timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/overlap_$i.log 2>&1 || exit 1; }
done
timeout -k 10 300 $W1 --allreduce rccl > $O/rccl_1.log 2>&1 || exit 1
for f in $O/*.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1) $(grep -o '"total_cost_time_s": [0-9.]*' $f | tail -1)"; done
