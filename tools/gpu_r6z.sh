#!/bin/bash
set -o pipefail
O=gpurun_out/r6z; mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["reference_script"]; print("bench", round(d["ms_per_step"]*1000,2), "total_cost", d.get("total_cost_time_s"), r.get("order"), r.get("setup_phases_s",{}).get("hip_init"), "wall20", d.get("wallclock_20ep_s"), "acc", d.get("final_test_acc"))'
done
timeout -k 10 300 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm > $O/w1.log 2>&1 || { tail -20 $O/w1.log; exit 1; }
tail -1 $O/w1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["reference_script"]; print("world1", d["config"].get("allreduce"), round(d["ms_per_step"]*1000,2), "total_cost", d.get("total_cost_time_s"), r.get("order"))'
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_ddp_one_gpu.py -k "bench" > $O/pytest_bench.log 2>&1 || { tail -40 $O/pytest_bench.log; exit 1; }
tail -1 $O/pytest_bench.log
