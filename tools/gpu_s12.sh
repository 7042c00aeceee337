set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_numerics.py tests/test_gpu_module_api.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/s12_t.log 2>&1 || { tail -30 gpurun_out/s12_t.log; exit 1; }
tail -2 gpurun_out/s12_t.log
bash tools/ab_multi.sh auto "MNIST_AMD_WGRAD_STAG=auto" -- --steps 1000 && bash tools/ab_multi.sh auto8k "MNIST_AMD_WGRAD_STAG=auto" -- --batch-size 8192 --steps 60 --warmup 10 && bash tools/ab_multi.sh b512 "MNIST_AMD_WGRAD_STAG=0" "MNIST_AMD_WGRAD_STAG=1" -- --batch-size 512 --steps 400
