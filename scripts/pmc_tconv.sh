#!/bin/bash
# SQ counter passes (one rocprofv3 run each) over `microbench.py tail1d` (one dense narrow conv as the model runs it:
# TC channels, TK taps, TMODE conv1 / conv2), with and without its fused epilogue (ALCM_TCONV_ABLATE=1).
# Usage: bash scripts/pmc_tconv.sh <tag>   (TC, TK, TMODE from the environment)
out=gpurun_out/pmc_tconv_$1; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for ab in 0 1; do
  ALCM_TCONV_ABLATE=$ab SPIN=1 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $out/p1_$ab -o run --output-format csv -- python scripts/microbench.py tail1d > $out/p1_$ab.log 2>&1 || exit $?
  ALCM_TCONV_ABLATE=$ab SPIN=1 timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES -d $out/p2_$ab -o run --output-format csv -- python scripts/microbench.py tail1d > $out/p2_$ab.log 2>&1 || exit $?
done
echo DONE
