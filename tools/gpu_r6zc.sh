#!/bin/bash
# production-command startup table W = 2 / 4 with the non-blocking engine streams; stream kind per run
set -o pipefail
O=gpurun_out/r6zc; mkdir -p $O
timeout -k 10 600 python tools/startup_table.py --production --world 2 4 --reps 2 --out $O/startup_production.md > $O/startup.log 2>&1 || { echo startup fail; tail -30 $O/startup.log; exit 1; }
grep "setup_total_s" $O/startup_production.md
export MNIST_AMD_ONE_GPU=1 GPU_MAX_HW_QUEUES=2
timeout -k 10 120 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 2 mnist_ddp.py --batch-size 200 --epochs 2 --synthetic --json-log $O/w2.jsonl > $O/w2.log 2>&1 || { tail -20 $O/w2.log; exit 1; }
grep -h '"streams"' $O/w2.jsonl | python -c 'import json,sys; [print({k: json.loads(l).get(k) for k in ("streams","schedule","allreduce")}) for l in sys.stdin]'
grep "Total cost" $O/w2.log
