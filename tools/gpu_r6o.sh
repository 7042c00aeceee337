#!/bin/bash
# dgrad dy-tile store order (LDS bank spread): bitwise tests, A/B vs the previous build, PMC conflicts
set -o pipefail
R=$PWD; O=gpurun_out/r6o; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_numerics.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 env MNIST_AMD_RACE_WIDEN=1 python tools/race_widen_check.py --case overlap > $O/rw.log 2>&1 || { tail -20 $O/rw.log; exit 1; }
tail -1 $O/rw.log
for i in 1 2; do
  for v in head prev; do
    if [ $v = head ]; then e=""; else e="MNIST_AMD_EXT_PATH=$R/tools/so/prev.so"; fi
    env $e timeout -k 10 200 python bench.py --no-full-run --batch-size 8192 --steps 100 --warmup 10 > $O/b8192_${v}_$i.log 2>&1 || { tail -20 $O/b8192_${v}_$i.log; exit 1; }
    env $e timeout -k 10 200 python bench.py --no-full-run --steps 600 --warmup 50 > $O/b200_${v}_$i.log 2>&1 || { tail -20 $O/b200_${v}_$i.log; exit 1; }
    echo "$v $i b8192 $(tail -1 $O/b8192_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1), d.get("last_train_loss"))') b200 $(tail -1 $O/b200_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2), d.get("last_train_loss"))')" | tee -a $O/ab_summary.txt
  done
done
cd /tmp && export TMPDIR=/tmp
for v in head prev; do
  if [ $v = head ]; then e=""; else e="$R/tools/so/prev.so"; fi
  MNIST_AMD_EXT_PATH=$e timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS -d $R/$O/pmc_$v -o run --output-format csv -- python3 $R/bench.py --batch-size 8192 --steps 20 --warmup 5 --no-full-run > $R/$O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 $R/tools/pmc_kernel.py $(find $R/$O/pmc_$v -name '*counter_collection.csv' | head -1) conv2_dgrad | sed "s/^/$v /" | tee -a $R/$O/pmc_summary.txt
done
