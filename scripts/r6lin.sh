#!/bin/bash
# round 6: lin_plane 96-column tiles (DiT / text q,k,v): op tests + DiT / text / e2e model tests, then the bench
# alternating ALCM_LIN_BN96=1 / 0
out=gpurun_out/r6lin; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_text.py -k "lin_plane or k1 or dit or text or end_to_end or batch32" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=3 bash scripts/gpu_ab.sh r6lin_ab "ALCM_LIN_BN96=1" "ALCM_LIN_BN96=0"
