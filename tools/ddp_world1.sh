#!/bin/bash
# World-1 DDP schedule cost on one GPU: the single-GPU OVERLAP step against the XGMI and RCCL
# production schedules (torch.distributed.run, one rank, communicator attached), same box,
# interleaved.  Each run: 600 timed steps (steady state) and the driver's 20-step window.
# usage (on the box): bash tools/ddp_world1.sh TAG [REPS] [KINDS]   -> gpurun_out/w1_TAG/
#   KINDS: space-separated subset of "overlap xgmi rccl" (default all three)
R=${GRAFT_REPO_ROOT:-$PWD}; cd "$R" || exit 1
T=${1:-w1}; N=${2:-2}; KINDS=${3:-overlap xgmi rccl}; O=gpurun_out/w1_$T; mkdir -p "$O"
fatal() { case $1 in 124|134|137|139) echo "FATAL exit $1 in $2: stopping"; exit "$1";; esac; [ "$1" -eq 0 ] || { echo "step $2 failed ($1)"; exit "$1"; }; }
one() {   # KIND STEPS WARMUP TAG
  local kind=$1 s=$2 w=$3 tag=$4 log
  log=$O/${kind}_s${s}_$tag.log
  case $kind in
    overlap) timeout -k 10 300 python bench.py --steps "$s" --warmup "$w" --no-full-run > "$log" 2>&1;;
    xgmi|rccl) timeout -k 10 300 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 \
        --nproc-per-node 1 bench.py --force-comm --allreduce "$kind" --steps "$s" --warmup "$w" --no-full-run > "$log" 2>&1;;
  esac
  local rc=$?
  python - "$log" "$kind" "$s" <<'EOF'
import json, sys
log, kind, s = sys.argv[1:]
js = [l for l in open(log) if l.startswith("{")]
if not js:
    print(f"{kind:8s} s{s}: no JSON"); sys.exit(0)
d = json.loads(js[-1]); c = d.get("config", {})
print(f"{kind:8s} s{s:>4}: {1000*d['ms_per_step'] if d.get('ms_per_step') else float('nan'):7.2f} us/step  "
      f"sched={c.get('schedule')} ar={c.get('allreduce')} dev_ms={d.get('timed_device_ms')} "
      f"probe={c.get('allreduce_schedule_us')}")
EOF
  fatal $rc "$kind s$s"
}
for r in $(seq 1 "$N"); do
  for k in $KINDS; do
    one $k 600 50 r$r
    one $k 20 5 r$r
  done
done | tee "$O/summary.txt"
