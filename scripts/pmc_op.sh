#!/bin/bash
# SQ / TA / TCC counter passes (one rocprofv3 run each) over `microbench.py op1`.
out=gpurun_out/pmc_op; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $out/p1 -o run --output-format csv -- python scripts/microbench.py op1 > $out/p1.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d $out/p2 -o run --output-format csv -- python scripts/microbench.py op1 > $out/p2.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p3 -o run --output-format csv -- python scripts/microbench.py op1 > $out/p3.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $out/p4 -o run --output-format csv -- python scripts/microbench.py op1 > $out/p4.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/t -o run --output-format csv -- python scripts/microbench.py op1 > $out/t.log 2>&1
echo DONE
