#!/bin/bash
set -o pipefail
O=gpurun_out/r6zl; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_module_api.py tests/test_gpu_ddp_one_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 120 python mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --json-log $O/r_$i.jsonl > $O/r_$i.log 2>&1 || { tail -20 $O/r_$i.log; exit 1; }
  python - $O/r_$i.jsonl "$(grep 'Total cost' $O/r_$i.log)" <<'PY' | tee -a $O/summary.txt
import json, sys
recs = [json.loads(l) for l in open(sys.argv[1])]
ep = [r for r in recs if "epoch" in r]
d = [1e6 * (r.get("device_train_s") or 0) / 300 for r in ep]
print("batched loss reads", sys.argv[2], "epoch1 %.1f" % d[0], "epochs 2-20 mean %.2f" % (sum(d[1:]) / len(d[1:])))
PY
done
grep -c "^Train Epoch" $O/r_1.log; grep "Test set" $O/r_1.log | tail -1
