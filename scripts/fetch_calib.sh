#!/bin/bash
# GPU-box recipe: FETCH_SIZE / WRITE_SIZE calibration against known byte counts (scripts/probes/fetch_probe.hip,
# built here by hipcc into scripts/probes/bin/).  Separate --pmc passes, as MI355X_MICROARCH.md prescribes.
out=gpurun_out/fetch_calib
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=scripts/probes/bin/fetch_probe
timeout -k 10 60 $P > $out/plain.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- $P > $out/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- $P > $out/write.log 2>&1 || exit $?
python3 scripts/fetch_calib.py $out > $out/SUMMARY.md
echo DONE
