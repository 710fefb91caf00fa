#!/bin/bash
# round 6, call o: wconv3 MFMA operand order A/B per shape (ALCM_W3_TR 0 / 1 / 2), outputs compared bit for bit
out=gpurun_out/r6o; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
XP_NAME=ALCM_W3_TR XP_VALS=0,1,2 timeout -k 10 400 python -u scripts/microbench.py xp > $out/xp.txt 2>&1
cat $out/xp.txt
