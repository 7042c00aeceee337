set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_numerics.py tests/test_gpu_module_api.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/s23_t.log 2>&1 || { tail -30 gpurun_out/s23_t.log; exit 1; }
tail -2 gpurun_out/s23_t.log
bash tools/ab_multi.sh mr "MNIST_AMD_FC1_MR=1" "MNIST_AMD_FC1_MR=2" "MNIST_AMD_FC1_MR=4" -- --steps 1000
