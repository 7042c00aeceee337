#!/bin/bash
# Profiles only (the validation half of tools/gpu_final.sh skipped): rocprofv3 kernel stats of the
# default schedule at B = 200 / 8192, the four PMC passes of each, per-kernel roofline tables.
# usage (on the box): bash tools/gpu_profiles.sh TAG      -> gpurun_out/TAG/
R=$PWD; T=${1:-prof}; O=gpurun_out/$T; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2: stopping"; exit $1;; esac; [ $1 -eq 0 ] || { echo "step $2 failed ($1)"; exit $1; }; }
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
