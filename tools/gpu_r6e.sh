#!/bin/bash
set -o pipefail
O=gpurun_out/r6e; mkdir -p $O
for m in pool reuse dedicated raw; do
  timeout -k 10 200 python tools/queue_mapping.py --mode $m --trainers 10 > $O/qm_$m.jsonl 2> $O/qm_$m.err || { echo "$m fail"; tail -20 $O/qm_$m.err; exit 1; }
  tail -1 $O/qm_$m.jsonl
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python tools/queue_mapping.py --mode pool --trainers 10 > $O/qm_pool_q8.jsonl 2> $O/qm_pool_q8.err || { echo "q8 fail"; exit 1; }
echo "q8 $(tail -1 $O/qm_pool_q8.jsonl)"
