#!/bin/bash
# GPU-box validation of HEAD in two calls (each fits gpurun's limit):
#   bash scripts/gpu_validate.sh <tag> tests   -> the whole -m gpu suite, smoke(), rocprofv3 stats + PMC passes
#   bash scripts/gpu_validate.sh <tag> bench   -> the driver's bench command (default cpu_baseline included)
tag=${1:-validate}; what=${2:-tests}
out=gpurun_out/$tag; mkdir -p $out
if [ "$what" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
  rc=$?
  echo "TESTS EXIT $rc" >> $out/tests.log
  grep -E "FAILED|ERROR|passed|failed" $out/tests.log | tail -20
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
  tail -3 $out/smoke.log
  bash scripts/profile_bench.sh $tag || exit $?
else
  timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit $?
  cat $out/bench.json
fi
