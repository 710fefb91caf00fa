#!/bin/bash
# GPU-box recipe: rocprofv3 kernel-trace stats of the bench command, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) over one bench step.  Usage: bash scripts/profile_bench.sh <tag> [bench args]
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --also-other-mode 0 --cpu-baseline 0 "$@" > $out/bench_traced.log 2>&1 || exit $?
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --also-other-mode 0 --cpu-baseline 0 "$@" > $out/pmc_fetch.log 2>&1 || exit $?
ALCM_SERIAL_RESBLOCKS=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --also-other-mode 0 --cpu-baseline 0 "$@" > $out/pmc_write.log 2>&1 || exit $?
echo DONE
