#!/bin/bash
# round 6, call m: wconv3 with swapped MFMA operands (16-B epilogue pieces): bit-identity + wconv3 tests, then the
# bench alternating ALCM_W3_TR=1 / 0 with per-kernel rows
tag=${1:-r6m}
out=gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "wconv3 or conv1_fp16" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=3 bash scripts/gpu_ab.sh ${tag}_ab "ALCM_W3_TR=1" "ALCM_W3_TR=0"
