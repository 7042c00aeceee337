#!/bin/bash
set -o pipefail
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_fp32.py tests/test_gpu_numerics.py > $O/pytest.log 2>&1 || { echo "pytest fail"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/accuracy_parity.sh $O/accuracy || { echo accuracy fail; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo bench fail; tail -20 $O/bench_default.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_exact.log 2>&1 || { echo bench fail; tail -20 $O/bench_exact.log; exit 1; }
for f in bench_default bench_exact; do tail -1 $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['ms_per_step'], d['value'], d.get('total_cost_time_s'), d.get('final_test_acc'))"; done
bash tools/ab_ext.sh dgub "dg_ub_areuse dg_ub_anone" --batch-size 8192 --steps 100 --warmup 10 || exit 1
