set -o pipefail
mkdir -p gpurun_out/r2a
(rocprofv3 -L > gpurun_out/r2a/counters.txt 2>&1 || true)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/r2a/tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc" >> gpurun_out/r2a/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r2a/bench.log 2>&1
