#!/bin/bash
# GPU-box recipe: rocprofv3 kernel-trace stats of the bench command, then separate PMC passes over one bench
# step: FETCH_SIZE, WRITE_SIZE (HBM bytes) and the MFMA pass (MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES /
# (GRBM_GUI_ACTIVE x SIMDs), MFMA op counts per dtype).  Resblock chains serialised (ALCM_SERIAL_RESBLOCKS=1)
# so every kernel's counters are its own.   Usage: bash scripts/profile_bench.sh <tag> [bench args]
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python bench.py --steps 2 --warmup 1 $B "$@" > $out/bench_traced.log 2>&1 || exit $?
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 $B "$@" > $out/pmc_fetch.log 2>&1 || exit $?
python3 scripts/pmc_compact.py $out/pmc_fetch
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 $B "$@" > $out/pmc_write.log 2>&1 || exit $?
python3 scripts/pmc_compact.py $out/pmc_write
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CU_CYCLES -d $out/pmc_mfma -o run --output-format csv -- python bench.py --steps 1 --warmup 0 $B "$@" > $out/pmc_mfma.log 2>&1 || exit $?
python3 scripts/pmc_compact.py $out/pmc_mfma
echo DONE
