#!/bin/bash
# round 6, last call: the whole -m gpu suite and smoke() on the final build (no profiling)
out=gpurun_out/r6end; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc" >> $out/tests.log
grep -E "FAILED|passed|failed" $out/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -2 $out/smoke.log
