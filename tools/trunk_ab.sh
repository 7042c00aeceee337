#!/bin/bash
# A/B of the trunk_fwd variants (whole-image WG vs strip WGs): numerics, bench step time, kernel time.
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_numerics.py -x -q > gpurun_out/ab_numerics.log 2>&1; echo NUM_EXIT $?; tail -2 gpurun_out/ab_numerics.log
for v in img strip; do
  if [ $v = strip ]; then export MNIST_TRUNK_STRIP=1; fi
  timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "$v b200 $(tail -1 gpurun_out/ab_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  timeout -k 10 200 python bench.py --batch-size 8192 --steps 20 --warmup 5 --no-full-run --graph-steps 5 > gpurun_out/ab_big_$v.log 2>&1 || exit 1
  echo "$v b8192 $(tail -1 gpurun_out/ab_big_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_prof_$v -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 20 --no-full-run > $R/gpurun_out/ab_prof_$v.log 2>&1) || exit 1
done
unset MNIST_TRUNK_STRIP
find gpurun_out/ab_prof_* -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -9; done
