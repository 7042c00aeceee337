set -o pipefail
O=gpurun_out/dw1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_engine.py -k "large_batch" tests/test_gpu_ddp_one_gpu.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/kernel_bench.py 8192 > $O/kb8192.txt 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python bench.py --hook fc_dw1_side=0 --no-full-run --batch-size 8192 --steps 100 --warmup 10 > $O/b8192_off_$i.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-full-run --batch-size 8192 --steps 100 --warmup 10 > $O/b8192_on_$i.log 2>&1 || exit 1
done
for f in $O/b8192_*.log; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $f); done
