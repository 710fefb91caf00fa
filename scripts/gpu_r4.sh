#!/bin/bash
# Round-4 GPU call: the new / changed GPU tests, then an A/B of the fused AMPBlock pair (ALCM_AMPAIR=1 default vs 0,
# alternating in one call) on the default bench workload with per-kernel rows.  Usage: bash scripts/gpu_r4.sh <tag> [k]
tag=${1:-r4}
sel=${2:-"ampblock or bigvgan or batch32 or rccl or world2 or bench_batch32"}
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "$sel" \
  > $out/tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc" >> $out/tests.log
tail -3 $out/tests.log
[ $rc -eq 0 ] || exit $rc
ARGS="--steps 5 --warmup 2 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
for round in 1 2; do
  for v in 1 0; do
    ALCM_AMPAIR=$v ALCM_BENCH_ALL_KERNELS=1 timeout -k 10 300 python -u bench.py $ARGS \
      > $out/ab_${round}_$v.json 2> $out/ab_${round}_$v.err || exit $?
    echo "AMPAIR=$v: $(python -c "import json;d=json.load(open('$out/ab_${round}_$v.json'));print(d['value'], d['ms_per_step'])")" >> $out/ab.txt
  done
done
cat $out/ab.txt
