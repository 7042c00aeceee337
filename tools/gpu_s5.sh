set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_numerics.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/s5_t.log 2>&1 || { tail -30 gpurun_out/s5_t.log; exit 1; }
tail -2 gpurun_out/s5_t.log
bash tools/ab_sos.sh b200 "base cur" --steps 1000 && bash tools/ab_sos.sh b512 "base cur" --batch-size 512 && \
R=$PWD && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cur200 -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-full-run > $R/gpurun_out/prof_cur200.log 2>&1 && \
python3 $R/tools/kstats.py $R/gpurun_out/prof_cur200 > $R/gpurun_out/prof_cur200_stats.txt && cat $R/gpurun_out/prof_cur200_stats.txt | head -14 && \
python3 $R/tools/timeline.py $(ls $R/gpurun_out/prof_cur200/*/*kernel_trace.csv 2>/dev/null || find $R/gpurun_out/prof_cur200 -name '*kernel_trace.csv' | head -1) > $R/gpurun_out/prof_cur200_timeline.txt; cat $R/gpurun_out/prof_cur200_timeline.txt | head -30
