#!/bin/bash
# round 6, call h: the resident tail conv's residual epilogues from the accumulator layout (ALCM_TCONV_CFR) and
# wconv2's three weight buffers on 256 x 96 tiles (ALCM_WCONV2_NB): parity tests, bit-identical bench waveforms vs
# the previous forms, A/B
out=gpurun_out/r6h; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "multitile or dense_resident or fused_activation or ksplit or three_weight or opconv_wide or tile160" > $out/tests.log 2>&1 || exit $?
B="--steps 2 --warmup 1 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
ALCM_TCONV_CFR=0 ALCM_WCONV2_NB=2 timeout -k 10 300 python -u bench.py $B --dump-wav $out/w0.npy > $out/c0.json 2> $out/c0.err || exit $?
timeout -k 10 300 python -u bench.py $B --dump-wav $out/w1.npy > $out/c1.json 2> $out/c1.err || exit $?
python -c "
import numpy as np; a=np.load('$out/w0.npy'); b=np.load('$out/w1.npy')
print('CF epilogue + three weight buffers: waveforms bit-identical to the previous forms:', np.array_equal(a,b))" > $out/cmp.txt
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6h_ab "ALCM_TCONV_CFR=0 ALCM_WCONV2_NB=2" "ALCM_TCONV_CFR=1 ALCM_WCONV2_NB=2" "ALCM_TCONV_CFR=1 ALCM_WCONV2_NB=3"
