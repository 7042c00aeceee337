#!/bin/bash
# Same-box A/B over (build, env) pairs: each arg "SO_NAME[:ENV=V[,ENV=V]]" (tools/so/SO_NAME.so), interleaved
# 2 rounds; the working-tree .so is restored at the end.
# usage (on the box): bash tools/ab_so_env.sh TAG "persist cur:MNIST_AMD_WGRAD_STAG=0 ..." [bench args...]
T=$1; CFGS=$2; shift 2
SO=pytorch_mnist_ddp_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_C_keep.so || exit 1
for rep in 1 2; do
  i=0
  for c in $CFGS; do
    i=$((i+1)); n=${c%%:*}; e=""; [ "$c" != "$n" ] && e=${c#*:}
    cp tools/so/$n.so $SO
    env ${e//,/ } timeout -k 10 240 python bench.py --no-full-run "$@" > gpurun_out/abe_${T}_${i}_$rep.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/abe_${T}_${i}_$rep.log; cp /tmp/_C_keep.so $SO; exit 1; }
    echo "$T $c $(tail -1 gpurun_out/abe_${T}_${i}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], round(d["ms_per_step"]*1000, 2), "us/step loss", d.get("last_train_loss"))')"
  done
done
cp /tmp/_C_keep.so $SO
