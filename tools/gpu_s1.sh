set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_numerics.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/s1_t.log 2>&1 || { tail -30 gpurun_out/s1_t.log; exit 1; }
tail -2 gpurun_out/s1_t.log
bash tools/ab_knob.sh b200 MNIST_AMD_DGRAD_PERSIST 0 1 && bash tools/ab_knob.sh b8192 MNIST_AMD_DGRAD_PERSIST 0 1 --batch-size 8192 --steps 100 --warmup 10
