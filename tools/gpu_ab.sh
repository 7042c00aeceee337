#!/bin/bash
# A/B on the GPU box: engine/numerics tests, then bench with an env knob at two values (alternating),
# then rocprof stats of the default build.
# usage: bash tools/gpu_ab.sh TAG KNOB [A B]   (defaults: A=0 B=1)
R=$PWD; T=${1:-x}; K=${2:-MNIST_AMD_FUSE_FC}; VA=${3:-0}; VB=${4:-1}
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_numerics.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/t_$T.log 2>&1 || { tail -30 gpurun_out/t_$T.log; exit 1; }
tail -2 gpurun_out/t_$T.log
for v in $VA $VB $VA $VB; do
  env $K=$v timeout -k 10 200 python bench.py --no-full-run > gpurun_out/bench_${T}_$v.log 2>&1 || { tail -20 gpurun_out/bench_${T}_$v.log; exit 1; }
  echo "$K=$v $(tail -1 gpurun_out/bench_${T}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py > gpurun_out/bench_${T}_full.log 2>&1 && tail -1 gpurun_out/bench_${T}_full.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-full-run > $R/gpurun_out/prof_$T.log 2>&1; echo PROF_EXIT $?
python $R/tools/kstats.py $R/gpurun_out/prof_$T
