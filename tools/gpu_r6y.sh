#!/bin/bash
# non-blocking engine streams created first: tests, queue mapping, benches, the reference command
set -o pipefail
O=gpurun_out/r6y; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_xgmi.py tests/test_gpu_rccl.py tests/test_gpu_race_widen.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/queue_mapping.py --mode product --trainers 10 > $O/qm_product.log 2>&1 || { tail -20 $O/qm_product.log; exit 1; }
tail -3 $O/qm_product.log
for i in 1 2; do
  timeout -k 10 120 python mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --json-log $O/ref_$i.jsonl > $O/ref_$i.log 2>&1 || { tail -20 $O/ref_$i.log; exit 1; }
  python - $O/ref_$i.jsonl "$(grep 'Total cost' $O/ref_$i.log)" <<'PY' | tee -a $O/summary.txt
import json, sys
recs = [json.loads(l) for l in open(sys.argv[1])]
ep = [r for r in recs if "epoch" in r]
print("ref", sys.argv[2], "device us/step", [round(1e6 * (r.get("device_train_s") or 0) / 300, 1) for r in ep][:6])
PY
done
W1="python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --steps 600 --warmup 50 --no-full-run"
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("bench", round(d["ms_per_step"]*1000,2), d.get("total_cost_time_s"), c.get("streams"), c.get("slow_mode"))' | tee -a $O/summary.txt
for a in xgmi rccl auto; do
  if [ $a = auto ]; then x=""; else x="--allreduce $a"; fi
  timeout -k 10 300 $W1 $x > $O/w1_$a.log 2>&1 || { tail -20 $O/w1_$a.log; exit 1; }
  tail -1 $O/w1_$a.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("world1", c.get("allreduce"), round(d["ms_per_step"]*1000,2), c.get("allreduce_schedule_us"), c.get("slow_mode"))' | tee -a $O/summary.txt
done
