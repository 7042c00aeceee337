#!/bin/bash
# Graph-chunk length sweep (one build, interleaved twice): bash tools/gs_sweep.sh "GS_LIST" [bench args]
L=$1; shift
for rep in 1 2; do
  for gs in $L; do
    timeout -k 10 200 python bench.py --no-full-run --graph-steps $gs "$@" > gpurun_out/gs_${gs}_$rep.log 2>&1 || exit 1
    echo "gs=$gs $(tail -1 gpurun_out/gs_${gs}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1000, "us/step")')"
  done
done
