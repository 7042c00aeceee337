#!/bin/bash
set -o pipefail
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 700 python tools/startup_table.py --production --world 2 4 8 --reps 2 --out $O/startup_production.md > $O/startup.log 2>&1 || { echo startup fail; tail -30 $O/startup.log; exit 1; }
grep "setup_total_s" $O/startup_production.md
W1="python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --steps 600 --warmup 50 --no-full-run"
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/single_$i.log 2>&1 || exit 1
  timeout -k 10 300 $W1 --allreduce xgmi > $O/xgmi_$i.log 2>&1 || { tail -20 $O/xgmi_$i.log; exit 1; }
  timeout -k 10 300 $W1 --allreduce rccl > $O/rccl_$i.log 2>&1 || { tail -20 $O/rccl_$i.log; exit 1; }
  timeout -k 10 300 $W1 > $O/auto_$i.log 2>&1 || { tail -20 $O/auto_$i.log; exit 1; }
done
for f in $O/single_*.log $O/xgmi_*.log $O/rccl_*.log $O/auto_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(round(d["ms_per_step"]*1000,2), c.get("allreduce"), c.get("allreduce_schedule_us"), c.get("slow_mode"), c.get("rccl_init"))')"; done | tee $O/world1_summary.txt
timeout -k 10 300 python tools/timeline_tl.py --steps 300 --graph-steps 50 --out $O/timeline_b200_head.md > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 1; }
grep "^period" $O/timeline_b200_head.md
