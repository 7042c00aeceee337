#!/bin/bash
# Round-end validation on the GPU box: full GPU test suite, smoke, headline bench (+ reference-timer
# full run), B = 8192 stress bench, rocprofv3 kernel stats and PMC passes of both configs.
# usage (on the box): bash tools/gpu_final.sh TAG
R=$PWD; T=${1:-final}; O=gpurun_out/$T; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "TEST_EXIT $rc"; tail -3 $O/gpu_tests.log; fatal $rc tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 400 python bench.py > $O/bench_1gpu.log 2>&1; rc=$?; tail -1 $O/bench_1gpu.log | cut -c1-400; fatal $rc bench
timeout -k 10 200 python bench.py --no-full-run --batch-size 8192 --steps 100 --warmup 10 > $O/bench_b8192.log 2>&1; rc=$?; tail -1 $O/bench_b8192.log | cut -c1-200; fatal $rc bench8192
cd /tmp && export TMPDIR=/tmp
export MNIST_AMD_OVERLAP_FC=0   # serial single-GPU schedule: per-kernel times without the trunk's completion hold
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_b200 -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-full-run > $R/$O/prof_b200.log 2>&1; fatal $? prof200
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_b8192 -o run --output-format csv -- python3 $R/bench.py --batch-size 8192 --steps 30 --warmup 5 --no-full-run > $R/$O/prof_b8192.log 2>&1; fatal $? prof8192
cd $R
bash tools/pmc.sh b200 && bash tools/pmc.sh b8192 --batch-size 8192 --steps 20 --warmup 5 || exit 1
for b in 200 8192; do
  python tools/roofline.py --stats $O/prof_b$b --pmc gpurun_out/pmc1_b$b gpurun_out/pmc2_b$b gpurun_out/pmc3_b$b gpurun_out/pmc4_b$b --batch $b > $O/roofline_b$b.md 2>&1
done
python tools/kstats.py $O/prof_b200 > $O/kernel_stats_b200.txt; python tools/kstats.py $O/prof_b8192 > $O/kernel_stats_b8192.txt
cat $O/roofline_b200.md $O/roofline_b8192.md
