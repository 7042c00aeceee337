#!/bin/bash
# Session-3 check at HEAD: GPU suite, smoke, the driver's bench command, 600 steps x 2, B = 8192,
# world-1 XGMI, in-kernel timeline.  usage (box): bash tools/gpu_s3_check.sh TAG -> gpurun_out/TAG/
T=${1:-s3chk}; O=gpurun_out/$T; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; [ $1 -eq 0 ] || { echo "step $2 failed ($1)"; exit $1; }; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -1 $O/gpu_tests.log; fatal $rc tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; fatal $? smoke
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_exact.log 2>&1; fatal $? bench
for i in 1 2; do timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/bench_s600_$i.log 2>&1; fatal $? s600; done
timeout -k 10 200 python bench.py --no-full-run --batch-size 8192 --steps 100 --warmup 10 > $O/bench_b8192.log 2>&1; fatal $? b8192
timeout -k 10 300 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes 1 --nproc-per-node 1 bench.py --force-comm --allreduce xgmi --steps 600 --warmup 50 --no-full-run > $O/xgmi_s600.log 2>&1; fatal $? xgmi
timeout -k 10 200 python tools/timeline_tl.py --batch 200 --steps 300 --graph-steps 50 --out $O/timeline_overlap.md > $O/tl.log 2>&1; fatal $? tl
for f in $O/bench*.log $O/xgmi*.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1) $(grep -o '"total_cost_time_s": [0-9.]*' $f | tail -1)"; done
