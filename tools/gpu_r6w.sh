#!/bin/bash
set -o pipefail
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 120 python mnist_ddp.py --batch-size 200 --epochs 3 --synthetic --log-interval 100000 --json-log $O/a.jsonl > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
grep -h '"schedule"' $O/a.jsonl | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ("schedule","graph_steps","allreduce")})'
grep -h '"epoch"' $O/a.jsonl | cut -c1-300
