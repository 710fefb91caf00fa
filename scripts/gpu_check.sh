#!/bin/bash
# GPU-box check: the full -m gpu suite then the default bench line.  Usage: bash scripts/gpu_check.sh <tag>
tag=${1:-check}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/$tag/tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc" >> gpurun_out/$tag/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/$tag/bench.log 2>&1
