#!/bin/bash
# XGMI world-1 schedule: equal-count dgrad grid (default) vs 2 x CUs (--hook dgrad_grid=512), 600 steps
O=gpurun_out/dgx; mkdir -p $O
for i in 1 2; do
  for g in 0 512; do
    timeout -k 10 300 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --hook dgrad_grid=$g --force-comm --allreduce xgmi --steps 600 --warmup 50 --no-full-run > $O/x_g${g}_$i.log 2>&1 || exit 1
  done
done
for f in $O/x_*.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1) $(grep -o '"allreduce_schedule_us": {[^}]*}' $f)"; done
