#!/bin/bash
# conv reduce trees on lane moves: bitwise tests + A/B (single GPU and world-1 XGMI) vs the previous commit
set -o pipefail
O=gpurun_out/r6m; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_xgmi.py tests/test_gpu_rccl.py tests/test_gpu_race_widen.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
W1="python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --allreduce xgmi --steps 600 --warmup 50 --no-full-run"
for i in 1 2; do
  for v in head prev; do
    if [ $v = head ]; then e=""; else e="MNIST_AMD_EXT_PATH=$PWD/tools/so/prev.so"; fi
    env $e timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/single_${v}_$i.log 2>&1 || { tail -20 $O/single_${v}_$i.log; exit 1; }
    env $e timeout -k 10 300 $W1 > $O/xgmi_${v}_$i.log 2>&1 || { tail -20 $O/xgmi_${v}_$i.log; exit 1; }
    echo "$v $i single $(tail -1 $O/single_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2))') xgmi $(tail -1 $O/xgmi_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2), d["config"].get("allreduce"))')" | tee -a $O/ab_summary.txt
  done
done
