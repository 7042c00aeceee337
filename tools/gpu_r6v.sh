#!/bin/bash
set -o pipefail
O=gpurun_out/r6v; mkdir -p $O
timeout -k 10 200 python mnist_ddp.py --batch-size 200 --epochs 80 --synthetic --log-interval 100000 --json-log $O/e80.jsonl > $O/e80.log 2>&1 || { tail -20 $O/e80.log; exit 1; }
python - <<'PY'
import json
recs = [json.loads(l) for l in open("gpurun_out/r6v/e80.jsonl")]
ep = [r for r in recs if "epoch" in r]
print("device us/step by epoch", [round(1e6 * (r.get("device_train_s") or 0) / 300, 1) for r in ep])
PY
timeout -k 10 100 python bench.py --steps 600 --warmup 50 --no-full-run --no-warm-replay > $O/b_nowarm.log 2>&1 && tail -1 $O/b_nowarm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench no warm replay", round(d["ms_per_step"]*1000,2))'
timeout -k 10 100 python bench.py --steps 600 --warmup 50 --no-full-run > $O/b_warm.log 2>&1 && tail -1 $O/b_warm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench warm", round(d["ms_per_step"]*1000,2))'
