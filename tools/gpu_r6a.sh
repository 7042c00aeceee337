#!/bin/bash
# round 6 check 1: transport-selection + race-widening + engine tests, generator timing, a quick bench
set -o pipefail
O=gpurun_out/r6a; mkdir -p $O
python -c "
import time,torch,os
from pytorch_mnist_ddp_amd.data import synthetic as S
for i in range(3):
  t=time.perf_counter(); a,b=S.synthetic_mnist(True); t1=time.perf_counter(); c,d=S.synthetic_mnist(False); t2=time.perf_counter()
  print('datagen threads', S._threads(), 'train', round(t1-t,4), 'test', round(t2-t1,4))
" > $O/datagen.txt 2>&1; cat $O/datagen.txt
timeout -k 10 1000 python -u -m pytest -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_race_widen.py tests/test_gpu_ddp_one_gpu.py tests/test_gpu_rccl.py tests/test_gpu_xgmi.py tests/test_gpu_engine.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -60 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
timeout -k 10 200 python bench.py --steps 600 --warmup 50 --no-full-run > $O/bench_s600.log 2>&1 || { echo bench fail; tail -20 $O/bench_s600.log; exit 1; }
tail -1 $O/bench_s600.log
