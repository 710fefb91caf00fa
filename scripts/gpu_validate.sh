#!/bin/bash
# GPU-box validation of HEAD: the -m gpu suite, smoke(), the default bench line.  Usage: bash scripts/gpu_validate.sh <tag>
tag=${1:-validate}
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc" >> $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1
