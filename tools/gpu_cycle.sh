#!/bin/bash
# One GPU iteration: numerics/engine tests, headline bench, rocprofv3 kernel stats.
# usage (on the box): bash tools/gpu_cycle.sh TAG
R=$PWD; T=${1:-x}
timeout -k 10 600 python -m pytest tests/test_gpu_numerics.py tests/test_gpu_engine.py -q -m gpu > gpurun_out/t_$T.log 2>&1; echo TEST_EXIT $?
grep -E "^E |passed|failed" gpurun_out/t_$T.log | head -20
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.log 2>&1; echo BENCH_EXIT $?; tail -1 gpurun_out/bench_$T.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-full-run > $R/gpurun_out/prof_$T.log 2>&1; echo PROF_EXIT $?
