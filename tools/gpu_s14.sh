set -o pipefail
R=$PWD; O=gpurun_out/split; mkdir -p $O
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
export MASTER_PORT=$((20000 + RANDOM % 20000))
bash tools/ab_multi.sh split "MNIST_AMD_CONV_SPLIT=0" "MNIST_AMD_CONV_SPLIT=1" -- --force-comm --allreduce xgmi --steps 600 || exit 1
grep -o '"allreduce[^,]*' gpurun_out/abm_split_1_1.log | head -2
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  export MASTER_PORT=$((20000 + RANDOM % 20000))
  MNIST_AMD_CONV_SPLIT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_split$v -o run --output-format csv -- python3 $R/bench.py --force-comm --allreduce xgmi --steps 100 --warmup 20 --no-full-run > $R/$O/prof_split$v.log 2>&1 || exit 1
  python3 $R/tools/timeline.py $(find $R/$O/prof_split$v -name '*kernel_trace.csv' | head -1) > $R/$O/timeline_split$v.txt; cat $R/$O/timeline_split$v.txt | head -24
done
