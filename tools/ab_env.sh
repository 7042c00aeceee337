#!/bin/bash
# A/B of an environment switch on one box: bench.py with VAR=A and VAR=B alternating, N rounds.
# usage (on the box): bash tools/ab_env.sh OUTDIR VAR A B [N] [bench args...]
OUT=$1; VAR=$2; VA=$3; VB=$4; N=${5:-2}; shift 5
mkdir -p "$OUT" || exit 1
for i in $(seq 1 "$N"); do
  for v in "$VA" "$VB"; do
    env "$VAR=$v" timeout -k 10 240 python bench.py --no-script-run "$@" > "$OUT/bench_${v}_$i.log" 2>&1 || { echo "bench $VAR=$v $i failed"; exit 1; }
    echo "$VAR=$v $i $(tail -1 "$OUT/bench_${v}_$i.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1000, "us/step")')"
  done
done
