#!/bin/bash
out=gpurun_out/r6g; mkdir -p $out
timeout -k 10 400 python -u scripts/sens_ksplit.py > $out/sens.log 2>&1
echo "rc $?" >> $out/sens.log
