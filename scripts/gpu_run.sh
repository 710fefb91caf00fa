#!/bin/bash
# GPU call: selected GPU tests, optional microbench modes, then an A/B of knob settings on the default bench
# workload (alternating, two rounds, per-kernel rows in the .err files).
# Usage: bash scripts/gpu_run.sh <tag> "<pytest -k expr>" "<microbench modes>" "<variant> ..."
#   variant = a space-free env assignment list joined by commas, e.g. ALCM_CONV1_H16=0,ALCM_ACT_MFMA=0 ("-" = defaults)
tag=${1:-run}
sel=${2:-"bigvgan or bench_batch32"}
micro=${3:-""}
variants=${4:-"-"}
out=gpurun_out/$tag; mkdir -p $out
if [ "$sel" != "none" ]; then
  # no -x: test failures (exit 1) are reported and the measurements still run; anything else (a crash, a time
  # limit) ends the call here
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread -k "$sel" \
    > $out/tests.log 2>&1
  rc=$?
  echo "TESTS EXIT $rc" >> $out/tests.log
  grep -E "FAILED|ERROR|passed|failed" $out/tests.log | tail -60
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for m in $micro; do
  timeout -k 10 600 python -u scripts/microbench.py $m > $out/micro_$m.txt 2>&1 || exit $?
  cat $out/micro_$m.txt
done
ARGS="--steps 5 --warmup 2 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0"
for round in 1 2; do
  for v in $variants; do
    envs=""
    [ "$v" != "-" ] && envs=$(echo "$v" | tr ',' ' ')
    name=$(echo "$v" | tr ',=/' '_-_')
    env $envs ALCM_BENCH_ALL_KERNELS=1 timeout -k 10 300 python -u bench.py $ARGS \
      > $out/ab_${round}_$name.json 2> $out/ab_${round}_$name.err || exit $?
    echo "$v: $(python -c "import json;d=json.load(open('$out/ab_${round}_$name.json'));print(d['value'], d['ms_per_step'])")" >> $out/ab.txt
  done
done
cat $out/ab.txt
