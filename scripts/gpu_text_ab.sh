#!/bin/bash
# GPU-box A/B of the text encoders' linears: operand planes + plane conv (default) vs the fp32-A GEMM
# (ALCM_TEXT_GEMM=1), after the full -m gpu suite.  Usage: bash scripts/gpu_text_ab.sh <tag>
tag=${1:-text_ab}
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc" >> $out/tests.log
[ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for v in "ALCM_TEXT_GEMM=" "ALCM_TEXT_GEMM=1"; do
    env $v timeout -k 10 300 python -u bench.py --steps 3 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 > $out/bench_${round}_${v#*=}.json 2> $out/bench_${round}_${v#*=}.err || exit $?
    echo "$v: $(python -c "import json;d=json.load(open('$out/bench_${round}_${v#*=}.json'));c=d['components'];print(d['value'], c['text_encode']['ms_per_call'], c['text_encode']['roofline']['kernel'], c['text_encode']['roofline']['kernel_frac'], c['mel_vae_encode']['ms_per_call'])")" >> $out/ab.txt
  done
done
cat $out/ab.txt
