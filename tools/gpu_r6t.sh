#!/bin/bash
set -o pipefail
O=gpurun_out/r6t; mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --json-log $O/run_$i.jsonl > $O/run_$i.log 2>&1 || { tail -20 $O/run_$i.log; exit 1; }
  tail -1 $O/run_$i.log
done
python - <<'PY'
import json
for i in (1, 2):
    recs = [json.loads(l) for l in open(f"gpurun_out/r6t/run_{i}.jsonl")]
    ep = [r for r in recs if "epoch" in r]
    dev = sum(r.get("device_train_s") or 0 for r in ep)
    host = [r.get("host_train_s") for r in ep]
    tl = [r for r in recs if "timeline_s" in r][-1]["timeline_s"]
    print(i, "epochs", len(ep), "device train s sum", round(dev, 4), "per-epoch device", [round(r.get("device_train_s") or 0, 4) for r in ep][:5])
    print(i, "host enqueue s", [round(h, 4) if h else h for h in host][:5])
    print(i, "timeline", {k: v for k, v in tl.items() if k.startswith("epoch1") or k.startswith("epoch2_") or k.startswith("epoch20") or k in ("trainer", "hip_native", "train_done")})
PY
