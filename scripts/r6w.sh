#!/bin/bash
# round 6, call w: NCT conv inputs as channels-last rows (DiT proj_in, VAE conv_in, BigVGAN conv_pre): model tests,
# then the bench alternating ALCM_NCT_CL=1 / 0
out=gpurun_out/r6w; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_api.py > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=3 bash scripts/gpu_ab.sh r6w_ab "ALCM_NCT_CL=1" "ALCM_NCT_CL=0"
