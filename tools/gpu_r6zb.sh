#!/bin/bash
# streams: non-blocking pair probed, CU-masked fallback; tests incl. one-GPU multi-rank; benches
set -o pipefail
O=gpurun_out/r6zb; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ddp_one_gpu.py tests/test_gpu_engine.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["reference_script"]; print("bench", round(d["ms_per_step"]*1000,2), "total_cost", d.get("total_cost_time_s"), r.get("order"), d["config"].get("streams"), r.get("setup_phases_s",{}).get("hip_init"))'
done
