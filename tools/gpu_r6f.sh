#!/bin/bash
# round 6 check 4: full GPU suite with dedicated engine queues, queue-mapping check, accuracy parity, benches
set -o pipefail
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 200 python tools/queue_mapping.py --mode product --trainers 10 > $O/qm_product.jsonl 2> $O/qm_product.err || { echo "qm fail"; tail -20 $O/qm_product.err; exit 1; }
tail -1 $O/qm_product.jsonl
timeout -k 10 1100 python -u -m pytest -v --timeout 280 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
bash tools/accuracy_parity.sh $O/accuracy || { echo accuracy fail; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo bench fail; tail -20 $O/bench_default.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_exact.log 2>&1 || { echo bench fail; tail -20 $O/bench_exact.log; exit 1; }
timeout -k 10 300 python bench.py --batch-size 8192 --steps 100 --warmup 10 --no-full-run > $O/bench_b8192.log 2>&1 || { echo bench fail; exit 1; }
for f in bench_default bench_exact bench_b8192; do tail -1 $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['ms_per_step'], d['value'], d.get('total_cost_time_s'), d.get('final_test_acc'))"; done
