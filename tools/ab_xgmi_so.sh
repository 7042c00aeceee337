#!/bin/bash
# XGMI world-1 600-step A/B: the in-tree build vs tools/so/$1.so (MNIST_AMD_EXT_PATH), interleaved
V=$1; O=gpurun_out/abx_$V; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --allreduce xgmi --steps 600 --warmup 50 --no-full-run > $O/head_$i.log 2>&1 || exit 1
  MNIST_AMD_EXT_PATH=$PWD/tools/so/$V.so timeout -k 10 300 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --allreduce xgmi --steps 600 --warmup 50 --no-full-run > $O/${V}_$i.log 2>&1 || exit 1
done
for f in $O/*.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1) $(grep -o '"allreduce_schedule_us": {[^}]*}' $f)"; done
