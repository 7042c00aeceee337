#!/bin/bash
# Host wait policy A/B: ROC_ACTIVE_WAIT_TIMEOUT (us of active polling before an interrupt wait)
# default vs long, on the driver's bench command (interleaved, 3 rounds)
for rep in 1 2 3; do
  for w in default 5000; do
    if [ $w = default ]; then
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/wait_${w}_$rep.log 2>&1 || exit 1
    else
      ROC_ACTIVE_WAIT_TIMEOUT=$w timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/wait_${w}_$rep.log 2>&1 || exit 1
    fi
    echo "wait=$w $(grep '^{' gpurun_out/wait_${w}_$rep.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1000, "us/step device", d.get("timed_device_ms"), "ref", d.get("total_cost_time_s"))')"
  done
done
