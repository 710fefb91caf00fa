#!/bin/bash
# round 6, call e: workgroup residency of the C = 48 tail conv variants (is the second workgroup per CU resident?)
out=gpurun_out/r6e; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TCONFIGS="48:3:conv2,48:11:conv2,48:11:conv1" XP_VALS=1,4,5 timeout -k 10 300 python -u scripts/microbench.py tres > $out/tres.log 2>&1
echo "rc $?" >> $out/tres.log
