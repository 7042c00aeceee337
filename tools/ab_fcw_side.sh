#!/bin/bash
# A/B: fc weight gradients (fc_bwd roles C + A) on the comm stream at B = 200 (bench.py --hook fc_dw1_side=1,
# default) vs inside the compute-stream fc_bwd (=0).  usage (box): bash tools/ab_fcw_side.sh TAG [tests]
T=${1:-fcw}; O=gpurun_out/$T; mkdir -p $O
if [ "$2" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
  tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --hook fc_dw1_side=$v --steps 600 --warmup 50 --no-full-run > $O/s600_$v.$i.log 2>&1 || exit 1
  done
done
for v in 0 1; do
  timeout -k 10 200 python bench.py --hook fc_dw1_side=$v --steps 20 --warmup 5 --no-full-run > $O/s20_$v.log 2>&1 || exit 1
done
for f in $O/s*.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
if [ "$3" = timeline ]; then
  timeout -k 10 200 python tools/timeline_tl.py --batch 200 --steps 300 --graph-steps 50 --out $O/timeline_on.md > $O/tl_on.log 2>&1 || exit 1
fi
