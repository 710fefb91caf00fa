#!/bin/bash
# round 6, call d: C = 48 tail conv at two / three workgroups per CU (ALCM_TCONV=4 / 5) vs the one-workgroup resident
# kernel: oracle parity, per-launch timings, phase trace, end-to-end A/B
out=gpurun_out/r6d; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "multitile or fp16_handoff" > $out/tests.log 2>&1 || exit $?
TC_SHAPES=48 VARS="ALCM_TCONV=1,ALCM_TCONV=4,ALCM_TCONV=5" timeout -k 10 300 python -u scripts/microbench.py tconv > $out/tconv.log 2>&1 || exit $?
TCONFIGS="48:3:conv2,48:11:conv2,48:3:conv1,48:11:conv1" XP_NAME=ALCM_TCONV XP_VALS=1,4,5 timeout -k 10 300 python -u scripts/microbench.py tphase > $out/tphase.log 2>&1 || exit $?
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6d_ab "ALCM_TCONV=1" "ALCM_TCONV=4" "ALCM_TCONV=5"
