#!/bin/bash
# round 6, call r: sum-form last conv2 of the wide stages' three chains (alcm_opconv_sum): op + model tests, then
# the bench alternating ALCM_WCONV_SUM=1 / 0
out=gpurun_out/r6r; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k "opconv_sum or wconv3 or conv1_fp16 or bigvgan or e2e or batch32" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=3 bash scripts/gpu_ab.sh r6r_ab "ALCM_WCONV_SUM=1" "ALCM_WCONV_SUM=0"
