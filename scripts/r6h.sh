#!/bin/bash
# round 6, call h: the resident tail conv's residual epilogues from the accumulator layout (ALCM_TCONV_CFR): parity
# tests, bit-identical bench waveforms vs the staged form, per-kernel A/B
out=gpurun_out/r6h; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "multitile or dense_resident or fused_activation" > $out/tests.log 2>&1 || exit $?
B="--steps 2 --warmup 1 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
ALCM_TCONV_CFR=0 timeout -k 10 300 python -u bench.py $B --dump-wav $out/w0.npy > $out/c0.json 2> $out/c0.err || exit $?
timeout -k 10 300 python -u bench.py $B --dump-wav $out/w1.npy > $out/c1.json 2> $out/c1.err || exit $?
python -c "
import numpy as np; a=np.load('$out/w0.npy'); b=np.load('$out/w1.npy')
print('CF epilogue: waveforms bit-identical to the staged form:', np.array_equal(a,b))" > $out/cmp.txt
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6h_ab "ALCM_TCONV_CFR=0" "ALCM_TCONV_CFR=1"
