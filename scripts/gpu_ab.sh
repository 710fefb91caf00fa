#!/bin/bash
# GPU-box A/B: the -m gpu suite, then the bench (no CPU baseline / extra configs) under each ALCM_* setting given,
# alternating, with per-kernel rows (ALCM_BENCH_ALL_KERNELS).  Usage: bash scripts/gpu_ab.sh <tag> "<env A>" "<env B>" ...
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
  rc=$?
  echo "TESTS EXIT $rc" >> $out/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
i=0
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    i=$((i+1))
    env $v ALCM_BENCH_ALL_KERNELS=1 timeout -k 10 300 python -u bench.py --steps 5 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0 > $out/bench_${round}_$i.json 2> $out/bench_${round}_$i.err || exit $?
    echo "$v: $(python -c "import json;d=json.load(open('$out/bench_${round}_$i.json'));print(d['value'], d['ms_per_step'])")" >> $out/ab.txt
  done
done
cat $out/ab.txt
