#!/bin/bash
set -o pipefail
O=gpurun_out/r6final_d; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["ms_per_step"]*1000,2), d["value"], "total_cost", d.get("total_cost_time_s"), "acc", d.get("final_test_acc"))'
done
W1="python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --steps 600 --warmup 50 --no-full-run"
timeout -k 10 300 $W1 > $O/w1.log 2>&1 || { tail -20 $O/w1.log; exit 1; }
tail -1 $O/w1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("world1", d["config"].get("allreduce"), round(d["ms_per_step"]*1000,2), d["config"].get("slow_mode"))'
