#!/bin/bash
# A/B: persistent dgrad grid at B = 200 (bench.py --hook dgrad_grid=N; 0 = default), 600 steps, interleaved
O=gpurun_out/dgrid; mkdir -p $O
for i in 1 2; do
  for g in ${GRIDS:-0 400 448}; do
    timeout -k 10 200 python bench.py --hook dgrad_grid=$g --steps 600 --warmup 50 --no-full-run > $O/g${g}_$i.log 2>&1 || exit 1
  done
done
for f in $O/g*.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
