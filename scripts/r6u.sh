#!/bin/bash
# round 6, call u: skinny-row GEMMs (DiT embedders), 64-row narrow-N tiles, 160-row strided upsampler tiles: op tests,
# the DiT / BigVGAN / e2e model tests, then the bench alternating the three switches on / off
out=gpurun_out/r6u; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k "gemm or linear or strided or dit or bigvgan or end_to_end or batch32 or cfg or config" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=3 bash scripts/gpu_ab.sh r6u_ab "ALCM_GEMM_SKINNY=1 ALCM_UPS_T160=1" "ALCM_GEMM_SKINNY=0 ALCM_UPS_T160=0"
