#!/bin/bash
# trunk A/B: bitwise fingerprint of the trunk outputs (tools/trunk_bits.py) for HEAD and tools/so/NAME.so,
# then same-box step timings at B = 200 and 8192 (tools/ab_ext.sh).  usage: bash tools/gpu_ab_trunk.sh NAME
set -o pipefail
N=$1; O=gpurun_out/$N; mkdir -p $O
timeout -k 10 120 python tools/trunk_bits.py > $O/bits_head.txt 2>&1 || { cat $O/bits_head.txt; exit 1; }
MNIST_AMD_EXT_PATH=$PWD/tools/so/$N.so timeout -k 10 120 python tools/trunk_bits.py > $O/bits_$N.txt 2>&1 || { cat $O/bits_$N.txt; exit 1; }
grep sha256 $O/bits_head.txt > $O/h.txt; grep sha256 $O/bits_$N.txt > $O/v.txt
paste $O/h.txt $O/v.txt
cmp -s $O/h.txt $O/v.txt && echo BITWISE_SAME || { echo BITS_DIFFER; exit 3; }
bash tools/ab_ext.sh $N "$N" && bash tools/ab_ext.sh ${N}8k "$N" --batch-size 8192 --steps 200 --warmup 20
