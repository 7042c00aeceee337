#!/bin/bash
set -o pipefail
O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_engine.py -k "one_wave or overlap_schedule_bitwise" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
