#!/bin/bash
set -o pipefail
O=gpurun_out/r6zk; mkdir -p $O
run() {
  local t=$1; shift
  timeout -k 10 120 python mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --json-log $O/$t.jsonl "$@" > $O/$t.log 2>&1 || { tail -20 $O/$t.log; exit 1; }
  python - $O/$t.jsonl $t "$(grep 'Total cost' $O/$t.log)" <<'PY' | tee -a $O/summary.txt
import json, sys
recs = [json.loads(l) for l in open(sys.argv[1])]
ep = [r for r in recs if "epoch" in r]
d = [1e6 * (r.get("device_train_s") or 0) / 300 for r in ep]
print(sys.argv[2], sys.argv[3], "epoch1 %.1f" % d[0], "epochs 2-20 mean %.2f" % (sum(d[1:]) / len(d[1:])))
PY
}
for i in 1 2; do
  run log10_$i
  run log100k_$i --log-interval 100000
done
timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/b.log 2>&1 && tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench window", round(d["ms_per_step"]*1000,2))' | tee -a $O/summary.txt
