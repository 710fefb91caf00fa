#!/bin/bash
# round 6, call p: kernel trace of the headline bench (resblock chains concurrent, as timed) for the per-step idle gaps
out=gpurun_out/r6p; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/trace -o run --output-format csv -- python bench.py --steps 4 --warmup 1 $B > $out/bench.log 2>&1 || exit $?
python3 scripts/trace_gaps.py $out/trace > $out/gaps.txt 2>&1

cat $out/gaps.txt
