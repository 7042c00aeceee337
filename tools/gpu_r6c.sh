#!/bin/bash
# round 6 check 3: device render == host render, difficulty sweep, startup with device-rendered data
set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_datagen.py tests/test_gpu_engine.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python tools/synth_difficulty.py > $O/difficulty.jsonl 2> $O/difficulty.err || { echo sweep fail; tail -20 $O/difficulty.err; exit 1; }
python -c "
import json
for ln in open('$O/difficulty.jsonl'):
    d=json.loads(ln); print(d['set'], d['final_test_acc'], d['final_test_loss'], d['test_acc_per_epoch'][:3], d['seconds'])"
timeout -k 10 400 python tools/startup_table.py --production --world 2 4 --reps 2 --out $O/startup_production_w2_w4.md > $O/startup.log 2>&1 || { echo startup fail; tail -30 $O/startup.log; exit 1; }
grep "setup_total_s" $O/startup_production_w2_w4.md
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_exact.log 2>&1 || { echo bench fail; tail -20 $O/bench_exact.log; exit 1; }
tail -1 $O/bench_exact.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['total_cost_time_s'], d['final_test_acc'], d['synthetic_data'], d['reference_script'].get('setup_phases_s'))"
