#!/bin/bash
# The reference's own timer (mnist_ddp.py, B = 200, 20 epochs, 1 GPU) with two chunk lengths,
# interleaved twice, and the printed lines of both compared (Total cost time lines excluded).
# usage (on the box): bash tools/ref_timer_ab.sh GS_A GS_B
A=${1:-10}; B=${2:-50}
for rep in 1 2; do
  for gs in $A $B; do
    timeout -k 10 200 python mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --graph-steps $gs \
      > gpurun_out/ref_gs${gs}_$rep.log 2>&1 || { echo "run gs=$gs failed"; tail -5 gpurun_out/ref_gs${gs}_$rep.log; exit 1; }
    echo "gs=$gs $(grep 'Total cost time' gpurun_out/ref_gs${gs}_$rep.log | tail -1)"
  done
done
grep -v "Total cost time" gpurun_out/ref_gs${A}_1.log > /tmp/ra.txt
grep -v "Total cost time" gpurun_out/ref_gs${B}_1.log > /tmp/rb.txt
if cmp -s /tmp/ra.txt /tmp/rb.txt; then echo "printed lines identical ($(wc -l < /tmp/ra.txt) lines)"; else echo "printed lines DIFFER"; diff /tmp/ra.txt /tmp/rb.txt | head -10; fi
