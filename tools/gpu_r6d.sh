#!/bin/bash
set -o pipefail
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 600 python tools/synth_difficulty.py --sets default ov0.7 ov0.75 ov0.8 ov0.85 ov0.9 ov0.7_warp ov0.75_noise > $O/difficulty.jsonl 2> $O/difficulty.err || { echo sweep fail; tail -20 $O/difficulty.err; exit 1; }
python -c "
import json
for ln in open('$O/difficulty.jsonl'):
    d=json.loads(ln); print(d['set'], d['final_test_acc'], d['final_test_loss'], d['test_acc_per_epoch'][:3], d['test_acc_per_epoch'][-3:], d['seconds'])"
