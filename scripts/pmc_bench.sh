#!/bin/bash
# SQ counter passes (one rocprofv3 run each) over one bench step with the resblock chains serialised, for the
# per-kernel wait / issue / LDS breakdown (summarise with scripts/pmc_summary.py <dir>/p* <kernel substring>).
# Usage: bash scripts/pmc_bench.sh <tag>
out=gpurun_out/pmc_bench_$1; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--steps 1 --warmup 0 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $out/p1 -o run --output-format csv -- python bench.py $B > $out/p1.log 2>&1 || exit $?
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d $out/p2 -o run --output-format csv -- python bench.py $B > $out/p2.log 2>&1 || exit $?
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p3 -o run --output-format csv -- python bench.py $B > $out/p3.log 2>&1 || exit $?
echo DONE
