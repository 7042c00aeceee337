#!/bin/bash
# reproduce the world-1 XGMI bimodal slowdown on its known triggers and time the steps
# from inside the kernels.  Triggers: the equal-count dgrad grid (--hook dgrad_grid=400) and the
# VGPR-capped W = 1 fused fc kernel (tools/so/capped.so, -DXGMI_FC_W1_MINBLOCKS=6).
set -o pipefail
O=gpurun_out/bimodal; mkdir -p $O
W1="python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --allreduce xgmi --steps 600 --warmup 50 --no-full-run"
js() { python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d["config"]; print(round(d["ms_per_step"]*1000,2), "us/step; validation replay", c.get("allreduce_schedule_us"), "slowdown", c.get("schedule_slowdown"))' $1; }
for i in 1 2 3; do
  timeout -k 10 300 $W1 > $O/head_$i.log 2>&1 || { echo head fail; tail -20 $O/head_$i.log; exit 1; }
  timeout -k 10 300 $W1 --hook dgrad_grid=400 > $O/dg400_$i.log 2>&1 || { echo dg400 fail; tail -20 $O/dg400_$i.log; exit 1; }
  MNIST_AMD_EXT_PATH=$PWD/tools/so/capped.so timeout -k 10 300 $W1 > $O/capped_$i.log 2>&1 || { echo capped fail; tail -20 $O/capped_$i.log; exit 1; }
  for t in head dg400 capped; do echo "$t $i: $(js $O/${t}_$i.log)"; done
done | tee $O/summary.txt
for i in 1 2; do
  timeout -k 10 300 python tools/timeline_tl.py --sched xgmi --steps 600 --warmup 50 --graph-steps 50 --hook dgrad_grid=400 --no-product --out $O/tl_dg400_$i.md > $O/tl_dg400_$i.log 2>&1 || { echo tl fail; tail -20 $O/tl_dg400_$i.log; exit 1; }
  MNIST_AMD_EXT_PATH=$PWD/tools/so/capped_tl.so timeout -k 10 300 python tools/timeline_tl.py --sched xgmi --steps 600 --warmup 50 --graph-steps 50 --no-product --out $O/tl_capped_$i.md > $O/tl_capped_$i.log 2>&1 || { echo tl fail; tail -20 $O/tl_capped_$i.log; exit 1; }
  timeout -k 10 300 python tools/timeline_tl.py --sched xgmi --steps 600 --warmup 50 --graph-steps 50 --no-product --out $O/tl_head_$i.md > $O/tl_head_$i.log 2>&1 || { echo tl fail; tail -20 $O/tl_head_$i.log; exit 1; }
  grep -h "^period" $O/tl_*_$i.md
done
