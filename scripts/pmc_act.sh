#!/bin/bash
# SQ counter passes (one rocprofv3 run each) over `microbench.py act1`: standalone Activation1d and a fused tail conv.
out=gpurun_out/pmc_act; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $out/p1 -o run --output-format csv -- python scripts/microbench.py act1 > $out/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_LDS -d $out/p2 -o run --output-format csv -- python scripts/microbench.py act1 > $out/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/t -o run --output-format csv -- python scripts/microbench.py act1 > $out/t.log 2>&1
echo DONE $?
