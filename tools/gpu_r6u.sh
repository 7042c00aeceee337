#!/bin/bash
set -o pipefail
O=gpurun_out/r6u; mkdir -p $O
run() {  # tag args...
  local t=$1; shift
  timeout -k 10 120 python mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --json-log $O/$t.jsonl "$@" > $O/$t.log 2>&1 || { tail -20 $O/$t.log; exit 1; }
  python - $O/$t.jsonl $t "$(grep 'Total cost' $O/$t.log)" <<'PY'
import json, sys
recs = [json.loads(l) for l in open(sys.argv[1])]
ep = [r for r in recs if "epoch" in r]
print(sys.argv[2], sys.argv[3], "device us/step", [round(1e6 * (r.get("device_train_s") or 0) / 300, 1) for r in ep][:6])
PY
}
for i in 1 2; do
  run log10_$i
  run log100k_$i --log-interval 100000
done
