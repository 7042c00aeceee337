#!/bin/bash
# PMC counter passes over a short bench run (run on the GPU box): bash tools/pmc.sh TAG [bench args...]
# (default bench args: the B = 200 headline config; e.g. `--batch-size 8192 --graph-steps 5` for the stress config)
R=$PWD; T=${1:-x}; shift
ARGS=${*:---steps 30 --warmup 10}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS -d $R/gpurun_out/pmc1_$T -o run --output-format csv -- python3 $R/bench.py $ARGS --no-full-run > $R/gpurun_out/pmc1_$T.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAVES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VALU -d $R/gpurun_out/pmc2_$T -o run --output-format csv -- python3 $R/bench.py $ARGS --no-full-run > $R/gpurun_out/pmc2_$T.log 2>&1 || exit 1
echo PMC_OK
