#!/bin/bash
# round 6, call j: act_coop's three-set kernel (now also in the serialised profile pass) with the UpSample1d FIR
# computed once for the three sets (ablib/libhoist.so) vs per set (HEAD), alternating
out=gpurun_out/r6j; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--steps 2 --warmup 1 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
ALCM_LIB=$GRAFT_REPO_ROOT/ablib/libhoist.so timeout -k 10 300 python -u bench.py $B --dump-wav $out/w_h.npy > $out/h.json 2> $out/h.err || exit $?
timeout -k 10 300 python -u bench.py $B --dump-wav $out/w_0.npy > $out/o.json 2> $out/o.err || exit $?
python -c "
import numpy as np; a=np.load('$out/w_h.npy'); b=np.load('$out/w_0.npy')
print('hoisted up FIR: waveforms bit-identical:', np.array_equal(a,b))" > $out/cmp.txt
TESTS=0 ROUNDS=2 bash scripts/gpu_ab.sh r6j_ab "ALCM_X=0" "ALCM_LIB=$GRAFT_REPO_ROOT/ablib/libhoist.so"
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_dist.py > $out/dist.log 2>&1
echo "dist rc $?" >> $out/dist.log
