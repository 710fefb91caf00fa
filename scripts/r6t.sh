#!/bin/bash
# round 6, call t: wconv3 K-split form as its own instantiation: wconv3 tests, then the bench alternating with the
# r6x library, and one per-shape pass (ALCM_PROF_SHAPES=1)
out=gpurun_out/r6t; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "wconv3 or opconv_sum or conv1_fp16" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6t_ab "ALCM_X=0" "ALCM_LIB=$GRAFT_REPO_ROOT/ablib/libr6x.so" || exit $?
ALCM_PROF_SHAPES=1 ALCM_BENCH_ALL_KERNELS=1 timeout -k 10 300 python -u bench.py --steps 3 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0 > $out/shapes.json 2> $out/shapes.err
