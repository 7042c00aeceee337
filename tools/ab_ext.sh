#!/bin/bash
# Same-box A/B: the in-tree build vs tools/so/<name>.so builds (MNIST_AMD_EXT_PATH), interleaved, 2 rounds.
# usage: bash tools/ab_ext.sh TAG "name1 name2 ..." [bench args...]
T=$1; NAMES=$2; shift 2
O=gpurun_out/ab_$T; mkdir -p $O
for rep in 1 2; do
  for n in head $NAMES; do
    if [ $n = head ]; then e=""; else e="MNIST_AMD_EXT_PATH=$PWD/tools/so/$n.so"; fi
    env $e timeout -k 10 240 python bench.py --no-full-run "$@" > $O/${n}_$rep.log 2>&1 || { echo "bench $n failed"; tail -5 $O/${n}_$rep.log; exit 1; }
    echo "$T $n $rep $(tail -1 $O/${n}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000, 2), "us/step loss", d.get("last_train_loss"))')"
  done
done
