#!/bin/bash
# PMC passes (separate runs, no tracing domains) over the fused narrow-stage kernel microbenchmark.
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc/p1 -o run --output-format csv -- python scripts/microbench.py amp1 > gpurun_out/pmc/p1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -d gpurun_out/pmc/p2 -o run --output-format csv -- python scripts/microbench.py amp1 > gpurun_out/pmc/p2.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/p3 -o run --output-format csv -- python scripts/microbench.py amp1 > gpurun_out/pmc/p3.log 2>&1
echo DONE $?
