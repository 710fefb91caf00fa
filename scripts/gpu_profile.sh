#!/bin/bash
# GPU-box recipe (run via gpurun): parity tests, bench, rocprofv3 kernel-trace stats and HBM PMC passes.
# Usage: bash scripts/gpu_profile.sh [pytest -k expression]
mkdir -p gpurun_out/prof
timeout -k 10 400 python -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -q -m gpu -s ${1:+-k "$1"} > gpurun_out/tests.log 2>&1; rc=$?; echo EXIT $rc >> gpurun_out/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --also-other-mode 1 --cpu-baseline 0 > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --also-other-mode 0 --cpu-baseline 0 > gpurun_out/prof/bench_traced.log 2>&1 || exit $?
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --also-other-mode 0 --cpu-baseline 0 > gpurun_out/prof/pmc_fetch.log 2>&1 || exit $?
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --also-other-mode 0 --cpu-baseline 0 > gpurun_out/prof/pmc_write.log 2>&1
echo DONE $?
