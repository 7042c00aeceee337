set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_numerics.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/s20_t.log 2>&1 || { tail -30 gpurun_out/s20_t.log; exit 1; }
tail -2 gpurun_out/s20_t.log
bash tools/ab_so_env.sh big "head cur" --batch-size 8192 --steps 60 --warmup 10 && bash tools/ab_so_env.sh b200 "head cur" --steps 1000
