#!/bin/bash
# round 6, call i: K split on the wide convs (wconv3 DiT FFN down, wconv2 text out-projections): parity tests, text
# encoder parity, component timing with and without (ALCM_KSPLIT)
out=gpurun_out/r6i; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_text.py -k "ksplit or text" > $out/tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  ALCM_KSPLIT=$v ALCM_BENCH_ALL_KERNELS=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 1 > $out/b_$v.json 2>> $out/b_$v.err || exit $?
  python -c "import json;d=json.load(open('$out/b_$v.json'));c=d['components']['text_encode'];print('KSPLIT=$v', d['value'], d['ms_per_step'], 'text', c['ms_per_call'], c['roofline']['kernel'], c['roofline']['kernel_share'])" >> $out/ab.txt
done
cat $out/ab.txt
