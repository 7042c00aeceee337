#!/bin/bash
# round 6 check 2: bimodal XGMI hunt, production-command startup table, accuracy on generator v3
set -o pipefail
O=gpurun_out/r6b; mkdir -p $O
MNIST_AMD_RACE_WIDEN=1 timeout -k 10 200 python tools/race_widen_check.py --case broken_w1t > $O/race_widen_broken_w1t.txt 2>&1; echo "broken_w1t rc=$?"; cat $O/race_widen_broken_w1t.txt | grep -v Gloo
MNIST_AMD_RACE_WIDEN=1 timeout -k 10 200 python tools/race_widen_check.py --case overlap > $O/race_widen_overlap.txt 2>&1 || { echo widen overlap fail; exit 1; }
timeout -k 10 600 python tools/startup_table.py --production --world 2 4 8 --reps 2 --out $O/startup_production_w2_w4_w8.md > $O/startup.log 2>&1 || { echo startup fail; tail -30 $O/startup.log; exit 1; }
grep "setup_total_s" $O/startup_production_w2_w4_w8.md
bash tools/accuracy_parity.sh $O/accuracy || { echo accuracy fail; exit 1; }
bash tools/bimodal.sh || { echo bimodal fail; exit 1; }
