#!/bin/bash
# GPU-box validation of HEAD: the -m gpu suite, smoke(), the default bench line.  Usage: bash scripts/gpu_validate.sh <tag>
tag=${1:-validate}
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc" >> $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || exit $?
# text encode: 96-column tiles for under-filled N % 128 problems (default) vs 128 x 128 (ALCM_OPCONV_TILE=-1)
for round in 1 2; do
  for v in "ALCM_OPCONV_TILE=" "ALCM_OPCONV_TILE=-1"; do
    env $v timeout -k 10 300 python -u bench.py --steps 3 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 > $out/ab_${round}_${v#*=}.json 2> $out/ab_${round}_${v#*=}.err || exit $?
    echo "$v: $(python -c "import json;d=json.load(open('$out/ab_${round}_${v#*=}.json'));c=d['components'];print(d['value'], c['text_encode']['ms_per_call'], c['text_encode']['roofline']['kernel'], c['mel_vae_encode']['ms_per_call'])")" >> $out/ab.txt
  done
done
cat $out/ab.txt
