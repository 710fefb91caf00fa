#!/bin/bash
# wconv2 workgroup-order A/B: timings, then L2 hit / HBM fetch counters of one shape per order
o=gpurun_out/word
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
WCONV_VARS=8 ORDERS=0,1 ABLATE=0,1 timeout -k 10 300 python -u scripts/microbench.py wablate > $o/wablate.log 2>&1 || exit $?
for ord in 0 1; do
  ALCM_WCONV_ORDER=$ord WSHAPES="s0 C768 k11,s1 C384 k11" timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $o/l2_$ord -o run --output-format csv -- python scripts/microbench.py wone > $o/l2_$ord.log 2>&1 || exit $?
  ALCM_WCONV_ORDER=$ord WSHAPES="s0 C768 k11,s1 C384 k11" timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $o/fetch_$ord -o run --output-format csv -- python scripts/microbench.py wone > $o/fetch_$ord.log 2>&1 || exit $?
done
echo DONE
