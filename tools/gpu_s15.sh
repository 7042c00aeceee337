set -o pipefail
for gs in ${GS_LIST:-25 75 150 300}; do
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --no-full-run --steps 600 --warmup 50 --graph-steps $gs > gpurun_out/gs_${gs}_$rep.log 2>&1 || { tail -5 gpurun_out/gs_${gs}_$rep.log; exit 1; }
    echo "graph_steps=$gs $(tail -1 gpurun_out/gs_${gs}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
