#!/bin/bash
# Round-5 validation at HEAD on the GPU box: full GPU suite, smoke, the driver's bench command, 600
# steps, B = 8192, fp32 (600 steps), rocprofv3 kernel stats of bf16 B = 200 / 8192 and fp32.
# usage (on the box): bash tools/gpu_round5_final.sh TAG      -> gpurun_out/TAG/
R=$PWD; T=${1:-final}; O=gpurun_out/$T; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2: stopping"; exit $1;; esac; [ $1 -eq 0 ] || { echo "step $2 failed ($1)"; exit $1; }; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "TEST_EXIT $rc"; tail -2 $O/gpu_tests.log; fatal $rc tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_exact.log 2>&1; fatal $? bench
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-full-run > $O/bench_exact2.log 2>&1; fatal $? bench2
timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/bench_s600.log 2>&1; fatal $? bench600
timeout -k 10 200 python bench.py --no-full-run --batch-size 8192 --steps 100 --warmup 10 > $O/bench_b8192.log 2>&1; fatal $? bench8192
timeout -k 10 200 python bench.py --no-full-run --dtype fp32 --steps 600 --warmup 50 > $O/bench_fp32.log 2>&1; fatal $? benchfp32
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_b200 -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-full-run --warm-replay-steps 0 > $R/$O/prof_b200.log 2>&1; fatal $? prof200
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_b8192 -o run --output-format csv -- python3 $R/bench.py --batch-size 8192 --steps 30 --warmup 5 --no-full-run --warm-replay-steps 0 > $R/$O/prof_b8192.log 2>&1; fatal $? prof8192
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_fp32 -o run --output-format csv -- python3 $R/bench.py --dtype fp32 --steps 50 --warmup 5 --no-full-run --warm-replay-steps 0 > $R/$O/prof_fp32.log 2>&1; fatal $? proffp32
cd $R
for b in b200 b8192 fp32; do python tools/kstats.py $O/prof_$b > $O/kernel_stats_$b.txt; done
python tools/bench_exact_summary.py $O/bench_*.log
