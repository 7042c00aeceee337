#!/bin/bash
# conv1 reduce + update on one-wave workgroups: bitwise tests, A/B at B = 200
set -o pipefail
O=gpurun_out/r6k; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_engine.py > $O/pytest_engine.log 2>&1 || { tail -40 $O/pytest_engine.log; exit 1; }
tail -1 $O/pytest_engine.log
timeout -k 10 300 env MNIST_AMD_RACE_WIDEN=1 python tools/race_widen_check.py --case overlap > $O/rw_overlap.log 2>&1 || { tail -20 $O/rw_overlap.log; exit 1; }
tail -2 $O/rw_overlap.log
for i in 1 2 3; do
  for h in 1 0; do
    timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run --hook c1_lanes=$h > $O/lanes${h}_$i.log 2>&1 || { tail -20 $O/lanes${h}_$i.log; exit 1; }
    echo "c1_lanes=$h $i $(tail -1 $O/lanes${h}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2), d.get("last_train_loss"))')" | tee -a $O/ab_summary.txt
  done
done
