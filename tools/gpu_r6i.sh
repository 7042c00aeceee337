#!/bin/bash
# conv1 tail inside the dgrad launch: bitwise tests, race widening, A/B at B = 200
set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_numerics.py > $O/pytest_engine.log 2>&1 || { tail -40 $O/pytest_engine.log; exit 1; }
tail -2 $O/pytest_engine.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_xgmi.py tests/test_gpu_rccl.py tests/test_gpu_race_widen.py > $O/pytest_ddp.log 2>&1 || { tail -40 $O/pytest_ddp.log; exit 1; }
tail -2 $O/pytest_ddp.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/tail_$i.log 2>&1 || { tail -20 $O/tail_$i.log; exit 1; }
  timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run --hook dgrad_c1_tail=0 > $O/notail_$i.log 2>&1 || { tail -20 $O/notail_$i.log; exit 1; }
done
for f in $O/tail_*.log $O/notail_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2))')"; done | tee $O/ab_summary.txt
timeout -k 10 300 python tools/timeline_tl.py --steps 300 --graph-steps 50 --out $O/timeline_b200_tail.md > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 1; }
grep "^period" $O/timeline_b200_tail.md
