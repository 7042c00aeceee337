#!/bin/bash
# Round-end validation on the GPU box: full GPU test suite, smoke, the driver's bench command (+ the
# reference-timer child job), 600-step steady state, B = 8192 stress, rocprofv3 kernel stats of the
# DEFAULT (overlapped, split-graph) schedule and PMC passes + per-kernel roofline of both configs.
# usage (on the box): bash tools/gpu_final.sh TAG      -> gpurun_out/TAG/
R=$PWD; T=${1:-final}; O=gpurun_out/$T; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2: stopping"; exit $1;; esac; [ $1 -eq 0 ] || { echo "step $2 failed ($1)"; exit $1; }; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "TEST_EXIT $rc"; tail -2 $O/gpu_tests.log; fatal $rc tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_exact.log 2>&1; rc=$?; grep '^{' $O/bench_exact.log | cut -c1-300; fatal $rc bench
timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/bench_s600.log 2>&1; rc=$?; grep '^{' $O/bench_s600.log | cut -c1-200; fatal $rc bench600
timeout -k 10 200 python bench.py --no-full-run --batch-size 8192 --steps 100 --warmup 10 > $O/bench_b8192.log 2>&1; rc=$?; grep '^{' $O/bench_b8192.log | cut -c1-200; fatal $rc bench8192
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_b200 -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-full-run > $R/$O/prof_b200.log 2>&1; fatal $? prof200
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_b8192 -o run --output-format csv -- python3 $R/bench.py --batch-size 8192 --steps 30 --warmup 5 --no-full-run > $R/$O/prof_b8192.log 2>&1; fatal $? prof8192
cd $R
bash tools/pmc.sh b200 && bash tools/pmc.sh b8192 --batch-size 8192 --steps 20 --warmup 5 || exit 1
for b in 200 8192; do
  python tools/roofline.py --stats $O/prof_b$b --pmc gpurun_out/pmc1_b$b gpurun_out/pmc2_b$b gpurun_out/pmc3_b$b gpurun_out/pmc4_b$b --batch $b > $O/roofline_b$b.md 2>&1
  python tools/kstats.py $O/prof_b$b > $O/kernel_stats_b$b.txt
done
python tools/timeline.py $(find $O/prof_b200 -name '*kernel_trace.csv' | head -1) > $O/timeline_b200.txt 2>&1
cat $O/roofline_b200.md $O/roofline_b8192.md
