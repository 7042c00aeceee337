#!/bin/bash
# PMC counter passes over a short bench run (run on the GPU box): bash tools/pmc.sh TAG [bench args...]
# (default bench args: the B = 200 headline config; e.g. `--batch-size 8192 --graph-steps 5` for the
# stress config).  One rocprofv3 run per pass, counters only (never combined with tracing), each pass
# within the per-block limits (8 SQ, 4 TCC: FETCH_SIZE takes 3, WRITE_SIZE 2 -> separate passes).
R=$PWD; T=${1:-x}; shift
ARGS=${*:---steps 30 --warmup 10}
cd /tmp && export TMPDIR=/tmp
pass() {
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc${n}_$T -o run --output-format csv -- \
    python3 $R/bench.py $ARGS --no-full-run > $R/gpurun_out/pmc${n}_$T.log 2>&1 || { echo "PMC pass $n failed"; exit 1; }
}
pass 1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS
pass 2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAVES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VALU
pass 3 FETCH_SIZE
pass 4 WRITE_SIZE
echo PMC_OK
