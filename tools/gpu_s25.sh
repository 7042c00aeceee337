set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s25_t.log 2>&1 || { tail -30 gpurun_out/s25_t.log; exit 1; }
tail -2 gpurun_out/s25_t.log
timeout -k 10 300 python bench.py > gpurun_out/s25_bench.log 2>&1 && tail -1 gpurun_out/s25_bench.log | cut -c1-300
