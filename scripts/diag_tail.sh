#!/bin/bash
# Round-6 diagnosis of the BigVGAN tail convs: per-launch timings resident vs streamed weights,
# the per-phase shader-clock trace, and SQ / TA / TD counter passes of one C = 48 conv (TC, TK, TMODE) under the
# resident kernel (one workgroup per CU) and the streamed one (two per CU).  Usage: bash scripts/diag_tail.sh <tag>
out=gpurun_out/$1; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
TC_SHAPES=48,24,96 VARS="ALCM_TCONV=3,ALCM_TCONV=2,ALCM_TCONV=1" timeout -k 10 300 python -u scripts/microbench.py tconv > $out/tconv.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/microbench.py tphase > $out/tphase.log 2>&1 || exit $?
export TC=${TC:-48} TK=${TK:-3} TMODE=${TMODE:-conv2}
for tk in 3 2; do
  ALCM_TCONV=$tk timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p1_$tk -o run --output-format csv -- python scripts/microbench.py tail1d > $out/p1_$tk.log 2>&1 || exit $?
  python3 scripts/pmc_compact.py $out/p1_$tk tconv
  ALCM_TCONV=$tk timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $out/p2_$tk -o run --output-format csv -- python scripts/microbench.py tail1d > $out/p2_$tk.log 2>&1 || exit $?
  python3 scripts/pmc_compact.py $out/p2_$tk tconv
  ALCM_TCONV=$tk timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES -d $out/p3_$tk -o run --output-format csv -- python scripts/microbench.py tail1d > $out/p3_$tk.log 2>&1 || exit $?
  python3 scripts/pmc_compact.py $out/p3_$tk tconv
done
for tk in 3 2; do
  ALCM_TCONV=$tk timeout -k 10 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr TD_TD_BUSY_sum TD_BUSY_avr -d $out/p4_$tk -o run --output-format csv -- python scripts/microbench.py tail1d > $out/p4_$tk.log 2>&1 || exit $?
  python3 scripts/pmc_compact.py $out/p4_$tk tconv
done
echo DONE
