#!/bin/bash
# round 6, call k: the wide stages' three first Activation1d in one MFMA-FIR pass (act_mfma3_kernel, ALCM_ACT_X3_MFMA):
# waveforms bit-identical to three act_mfma launches, B = 32 parity, A/B
out=gpurun_out/r6k; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--steps 2 --warmup 1 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
ALCM_ACT_X3_MFMA=0 timeout -k 10 300 python -u bench.py $B --dump-wav $out/w0.npy > $out/c0.json 2> $out/c0.err || exit $?
timeout -k 10 300 python -u bench.py $B --dump-wav $out/w1.npy > $out/c1.json 2> $out/c1.err || exit $?
python -c "
import numpy as np; a=np.load('$out/w0.npy'); b=np.load('$out/w1.npy')
print('act_mfma3: waveforms bit-identical to three act_mfma launches:', np.array_equal(a,b))" > $out/cmp.txt
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "batch32 or concurrent or M1872" > $out/tests.log 2>&1 || exit $?
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6k_ab "ALCM_ACT_X3_MFMA=0" "ALCM_ACT_X3_MFMA=1"
