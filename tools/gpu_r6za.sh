#!/bin/bash
set -o pipefail
O=gpurun_out/r6za; mkdir -p $O
export MNIST_AMD_ONE_GPU=1 GPU_MAX_HW_QUEUES=2
timeout -k 10 120 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 2 mnist_ddp.py --batch-size 200 --epochs 2 --synthetic --dist-backend gloo --allreduce xgmi > $O/child.log 2>&1; echo "rc=$?"
grep -v "^Train Epoch" $O/child.log | tail -40
