#!/bin/bash
# in-kernel timelines with per-wave statistics: single GPU and world-1 XGMI, B = 200
set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 300 python tools/timeline_tl.py --steps 300 --graph-steps 50 --out $O/tl_single.md > $O/tl1.log 2>&1 || { tail -20 $O/tl1.log; exit 1; }
timeout -k 10 300 python tools/timeline_tl.py --sched xgmi --steps 300 --warmup 50 --graph-steps 50 --out $O/tl_xgmi.md > $O/tl2.log 2>&1 || { tail -20 $O/tl2.log; exit 1; }
sed -n 7,22p $O/tl_single.md; sed -n 7,22p $O/tl_xgmi.md
