set -o pipefail
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s0_tests.log 2>&1; echo TEST_EXIT $?; tail -3 gpurun_out/s0_tests.log
timeout -k 10 300 python bench.py > gpurun_out/s0_bench.log 2>&1 && tail -1 gpurun_out/s0_bench.log | cut -c1-600
timeout -k 10 200 python bench.py --no-full-run --batch-size 8192 --steps 100 --warmup 10 > gpurun_out/s0_b8192.log 2>&1 && tail -1 gpurun_out/s0_b8192.log | cut -c1-300
