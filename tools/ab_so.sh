#!/bin/bash
# A/B of two builds of the extension on one box: bench.py with tools/_C_base.so (A) and the
# working-tree .so (B), alternating, N rounds.  usage (on the box): bash tools/ab_so.sh OUTDIR [N] [bench args...]
OUT=$1; N=${2:-2}; shift 2
SO=pytorch_mnist_ddp_amd/_C.cpython-310-x86_64-linux-gnu.so
mkdir -p "$OUT" && cp $SO "$OUT/_C_new.so" || exit 1
for i in $(seq 1 "$N"); do
  for v in A B; do
    if [ $v = A ]; then cp tools/_C_base.so $SO; else cp "$OUT/_C_new.so" $SO; fi
    timeout -k 10 240 python bench.py --no-script-run "$@" > "$OUT/bench_${v}_$i.log" 2>&1 || { echo "bench $v $i failed"; cp "$OUT/_C_new.so" $SO; exit 1; }
    echo "$v $i $(tail -1 "$OUT/bench_${v}_$i.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1000, "us/step")')"
  done
done
cp "$OUT/_C_new.so" $SO
