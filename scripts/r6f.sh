#!/bin/bash
# round 6, call f: (1) the new GPU tests (K-split, tail variants); (2) act_coop's shared up FIR: waveforms bit-identical
# to the round-5 library (ablib/libbase.so) with the K split off; (3) A/B: base, new without K split, new
out=gpurun_out/r6f; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "ksplit or multitile" > $out/tests.log 2>&1 || exit $?
B="--steps 2 --warmup 1 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
ALCM_LIB=$GRAFT_REPO_ROOT/ablib/libbase.so timeout -k 10 300 python -u bench.py $B --dump-wav $out/w_base.npy > $out/base.json 2> $out/base.err || exit $?
ALCM_KSPLIT=0 timeout -k 10 300 python -u bench.py $B --dump-wav $out/w_new.npy > $out/new.json 2> $out/new.err || exit $?
timeout -k 10 300 python -u bench.py $B --dump-wav $out/w_ks.npy > $out/ks.json 2> $out/ks.err || exit $?
python -c "
import numpy as np; a=np.load('$out/w_base.npy'); b=np.load('$out/w_new.npy'); c=np.load('$out/w_ks.npy')
print('act_coop shared up FIR, waveforms bit-identical to round 5:', np.array_equal(a,b), a.shape)
print('K split on: waveform rel-L2 vs off', float(np.linalg.norm(c.astype(np.float64)-b)/np.linalg.norm(b)))" > $out/cmp.txt
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6f_ab "ALCM_LIB=$GRAFT_REPO_ROOT/ablib/libbase.so" "ALCM_KSPLIT=0" "ALCM_X=0"
