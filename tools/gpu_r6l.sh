#!/bin/bash
# HEAD timeline + default-command bench after the one-wave conv1 kernel
set -o pipefail
O=gpurun_out/r6l; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/timeline_tl.py --steps 300 --graph-steps 50 --out $O/timeline_b200.md > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 1; }
grep "^period" $O/timeline_b200.md
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/default_$i.log 2>&1 || { tail -20 $O/default_$i.log; exit 1; }
  tail -1 $O/default_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("default", round(d["ms_per_step"]*1000,2), d.get("total_cost_time_s"), c.get("schedule"))'
  timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/s600_$i.log 2>&1 || { tail -20 $O/s600_$i.log; exit 1; }
  tail -1 $O/s600_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("s600", round(d["ms_per_step"]*1000,2))'
done
