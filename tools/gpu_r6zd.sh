#!/bin/bash
set -o pipefail
O=gpurun_out/r6zd; mkdir -p $O
for i in 1 2; do
  for g in 50 100 150 300; do
    timeout -k 10 120 python mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --graph-steps $g --json-log $O/g${g}_$i.jsonl > $O/g${g}_$i.log 2>&1 || { tail -20 $O/g${g}_$i.log; exit 1; }
    python - $O/g${g}_$i.jsonl "$(grep 'Total cost' $O/g${g}_$i.log)" $g <<'PY' | tee -a $O/summary.txt
import json, sys
recs = [json.loads(l) for l in open(sys.argv[1])]
ep = [r for r in recs if "epoch" in r]
d = [1e6 * (r.get("device_train_s") or 0) / 300 for r in ep]
print("graph_steps", sys.argv[3], sys.argv[2], "epoch1 %.1f" % d[0], "epochs 2-20 mean %.2f" % (sum(d[1:]) / len(d[1:])))
PY
  done
done
