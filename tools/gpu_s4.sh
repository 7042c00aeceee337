set -o pipefail
export MNIST_AMD_DGRAD_PERSIST=0
bash tools/ab_sos.sh big "base cur p28 noswz" --batch-size 8192 --steps 60 --warmup 10 && \
bash tools/ab_sos.sh b200 "base cur p28 noswz" && \
R=$PWD && cd /tmp && export TMPDIR=/tmp && \
cp $R/tools/so/base.so $R/pytorch_mnist_ddp_amd/_C.cpython-310-x86_64-linux-gnu.so && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_base8k -o run --output-format csv -- python3 $R/bench.py --batch-size 8192 --steps 30 --warmup 5 --no-full-run > $R/gpurun_out/prof_base8k.log 2>&1 && \
cp $R/tools/so/cur.so $R/pytorch_mnist_ddp_amd/_C.cpython-310-x86_64-linux-gnu.so && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cur8k -o run --output-format csv -- python3 $R/bench.py --batch-size 8192 --steps 30 --warmup 5 --no-full-run > $R/gpurun_out/prof_cur8k.log 2>&1 && \
python3 $R/tools/kstats.py $R/gpurun_out/prof_base8k && echo ---- && python3 $R/tools/kstats.py $R/gpurun_out/prof_cur8k
