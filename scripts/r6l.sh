#!/bin/bash
# round 6, call l: GroupNorm statistics in float4 pieces (VAE / DiT tests), then the round-6 tree against the round-5
# library (ablib/libbase.so) alternating in one call
out=gpurun_out/r6l; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_audio_in.py -k "vae or e2e or batch32 or dit or encode" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=3 bash scripts/gpu_ab.sh r6l_ab "ALCM_LIB=$GRAFT_REPO_ROOT/ablib/libbase.so" "ALCM_X=0"
