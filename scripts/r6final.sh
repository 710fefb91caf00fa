#!/bin/bash
# round 6: the new opconv_sum fallback / error test and the opconv_sum family on the final tree
out=gpurun_out/r6final; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "opconv_sum or skinny" > $out/tests.log 2>&1
echo "rc $?" >> $out/tests.log
tail -3 $out/tests.log
