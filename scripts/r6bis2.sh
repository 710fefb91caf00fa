#!/bin/bash
# round 6: skinny GEMM in fixed 32-row blocks (batch-split invariant): op tests, the dist tests, the model tests
out=gpurun_out/r6bis2; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_dist.py tests/test_gpu_models.py -k "skinny or gemm or linear or dist or world or spawn or dit or end_to_end or batch32 or shard" > $out/tests.log 2>&1
echo "rc $?" >> $out/tests.log
tail -3 $out/tests.log
