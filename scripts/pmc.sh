#!/bin/bash
# PMC passes (separate runs, kernel counters only) over one microbenchmark mode.
# Usage: bash scripts/pmc.sh <microbench mode> <out tag>
mode=$1; tag=$2
mkdir -p gpurun_out/pmc_$tag
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc_$tag/p1 -o run --output-format csv -- python scripts/microbench.py $mode > gpurun_out/pmc_$tag/p1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU -d gpurun_out/pmc_$tag/p2 -o run --output-format csv -- python scripts/microbench.py $mode > gpurun_out/pmc_$tag/p2.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_$tag/p3 -o run --output-format csv -- python scripts/microbench.py $mode > gpurun_out/pmc_$tag/p3.log 2>&1
echo DONE $?
