#!/bin/bash
# round 6, call a: the new parity tests (tail multi-tile vs the oracle, bench --gpus spawn), then the diagnostics
# compile-out A/B (ablib/libbase.so = the round-5 tail kernels) alternating in one call
out=gpurun_out/r6a; mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_dist.py -k "multitile or dense_resident or bench" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6a_ab "ALCM_LIB=$GRAFT_REPO_ROOT/ablib/libbase.so" "ALCM_X=0"
