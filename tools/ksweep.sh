#!/bin/bash
# Per-step time vs timed-window length K (warmup 5) for one build: bash tools/ksweep.sh [SO_NAME]
# (tools/so/SO_NAME.so swapped in for the run, the working-tree .so restored after)
SO=pytorch_mnist_ddp_amd/_C.cpython-310-x86_64-linux-gnu.so
[ -n "$1" ] && { cp $SO /tmp/_C_ks.so && cp tools/so/$1.so $SO || exit 1; }
rc=0
for k in 20 40 100 300; do
  timeout -k 10 200 python bench.py --no-full-run --steps $k --warmup 5 > gpurun_out/ksweep_$k.log 2>&1 || { rc=1; break; }
  echo "K=$k $(tail -1 gpurun_out/ksweep_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1000, "us/step device", d.get("timed_device_ms"))')"
done
[ -n "$1" ] && cp /tmp/_C_ks.so $SO
exit $rc
