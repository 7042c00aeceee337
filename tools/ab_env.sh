#!/bin/bash
# Same-box A/B of runtime environment settings, interleaved, 2 rounds.
# usage: bash tools/ab_env.sh TAG "label1:VAR=V,VAR2=W label2:VAR=X ..." [bench args...]
# ("base" = the environment as given)
T=$1; VARIANTS=$2; shift 2
O=gpurun_out/ab_$T; mkdir -p $O
for rep in 1 2; do
  for v in base $VARIANTS; do
    n=${v%%:*}; e=""
    [ "$v" != base ] && e=$(echo "${v#*:}" | tr ',' ' ')
    env $e timeout -k 10 240 python bench.py --no-full-run "$@" > $O/${n}_$rep.log 2>&1 || { echo "bench $n failed"; tail -5 $O/${n}_$rep.log; exit 1; }
    echo "$T $n $rep $(tail -1 $O/${n}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000, 2), "us/step loss", d.get("last_train_loss"))')"
  done
done
