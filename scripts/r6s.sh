#!/bin/bash
# round 6, call s: sum-form conv writing the next stage's upsampler planes: op + model tests, then the bench
# alternating ALCM_WCONV_SUM=1 (planes) / 2 (fp32 + to_planes)
out=gpurun_out/r6s; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k "opconv_sum or wconv3 or bigvgan or end_to_end or batch32 or shard or config5" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=3 bash scripts/gpu_ab.sh r6s_ab "ALCM_WCONV_SUM=1" "ALCM_WCONV_SUM=2"
