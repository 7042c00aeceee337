#!/bin/bash
# Round-6 HEAD validation, part A: full GPU test suite, smoke, the driver's bench command, steady state,
# B = 8192 stress, fp32 step.  usage (on the box): bash tools/gpu_r6final_a.sh TAG -> gpurun_out/TAG/
R=$PWD; T=${1:-r6final}; O=gpurun_out/$T; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2: stopping"; exit $1;; esac; [ $1 -eq 0 ] || { echo "step $2 failed ($1)"; exit $1; }; }
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "TEST_EXIT $rc"; tail -2 $O/gpu_tests.log; fatal $rc tests
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 300 python bench.py > $O/bench_exact.log 2>&1; rc=$?; grep '^{' $O/bench_exact.log | cut -c1-300; fatal $rc bench
timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/bench_s600.log 2>&1; rc=$?; grep '^{' $O/bench_s600.log | cut -c1-200; fatal $rc bench600
timeout -k 10 200 python bench.py --no-full-run --batch-size 8192 --steps 100 --warmup 10 > $O/bench_b8192.log 2>&1; rc=$?; grep '^{' $O/bench_b8192.log | cut -c1-200; fatal $rc bench8192
timeout -k 10 200 python bench.py --no-full-run --dtype fp32 --steps 300 --warmup 20 > $O/bench_fp32.log 2>&1; rc=$?; grep '^{' $O/bench_fp32.log | cut -c1-200; fatal $rc benchfp32
