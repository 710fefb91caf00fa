#!/bin/bash
# round 6: which round-6 switch makes the world-2 bench waveforms differ from the 64-prompt single run
out=gpurun_out/r6bis; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "ALCM_GEMM_SKINNY=0 ALCM_UPS_T160=0 ALCM_NCT_CL=0" "ALCM_UPS_T160=0" "ALCM_GEMM_SKINNY=0" "ALCM_NCT_CL=0"; do
  env $v timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_dist.py -k world2_gathers > $out/t.log 2>&1
  echo "$v: rc $? $(tail -1 $out/t.log)" >> $out/res.txt
done
cat $out/res.txt
