#!/bin/bash
# round 6, call b: the tail diagnosis (scripts/diag_tail.sh) and the new tests' measured errors
out=gpurun_out/r6b; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "multitile or fp16_handoff" > $out/tests.log 2>&1 || exit $?
bash scripts/diag_tail.sh r6b_diag
