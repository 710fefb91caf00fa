#!/bin/bash
# round 6, call y: BigVGAN conv_pre on the window conv (mel channels padded to 96): BigVGAN / e2e tests, then the bench
# alternating ALCM_NCT_CL=1 / 0 (0: the NCT gather on the generic GEMM)
out=gpurun_out/r6y; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "bigvgan or end_to_end or batch32 or config5" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6y_ab "ALCM_NCT_CL=1" "ALCM_NCT_CL=0"
