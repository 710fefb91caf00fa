#!/bin/bash
# Round-3 closing call: FETCH/WRITE calibration probe, -m gpu suite + A/B of the wconv3 epilogue, default bench line
# (with the §8(f) component lines), rocprofv3 stats + PMC passes of HEAD.
bash scripts/fetch_calib.sh || exit $?
TESTS=1 ROUNDS=2 bash scripts/gpu_ab.sh r3z_ab "ALCM_W3_EPI=1" "ALCM_W3_EPI=0" || exit $?
mkdir -p gpurun_out/r3z
timeout -k 10 400 python -u bench.py > gpurun_out/r3z/bench.log 2>&1 || exit $?
bash scripts/profile_bench.sh r3z
