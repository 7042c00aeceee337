#!/bin/bash
# Same-box A/B of several builds of the extension: bench.py with each tools/so/NAME.so in turn
# (interleaved, 2 rounds), the working-tree .so restored at the end.
# usage (on the box): bash tools/ab_sos.sh TAG "name1 name2 ..." [bench args...]
T=$1; NAMES=$2; shift 2
SO=pytorch_mnist_ddp_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_C_keep.so || exit 1
for rep in 1 2; do
  for n in $NAMES; do
    cp tools/so/$n.so $SO
    timeout -k 10 240 python bench.py --no-full-run "$@" > gpurun_out/abs_${T}_${n}_$rep.log 2>&1 || { echo "bench $n failed"; tail -5 gpurun_out/abs_${T}_${n}_$rep.log; cp /tmp/_C_keep.so $SO; exit 1; }
    echo "$T $n $(tail -1 gpurun_out/abs_${T}_${n}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"]*1000, "us/step loss", d.get("last_train_loss"))')"
  done
done
cp /tmp/_C_keep.so $SO
