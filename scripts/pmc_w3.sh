#!/bin/bash
# wconv3 HBM read attribution: FETCH_SIZE / WRITE_SIZE per BigVGAN stage 0-2 shape, conv2 form
# (residual, + accumulate at k3) and conv1 form (fp16 plane out), 5 launches each (scripts/microbench.py wone), then
# scripts/w3_fetch_table.py compares them with the per-launch byte model.  Usage: bash scripts/pmc_w3.sh <tag>
out=gpurun_out/$1; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export WSHAPES="s0 C768 k11,s0 C768 k3,s1 C384 k11,s1 C384 k3,s2 C192 k11,s2 C192 k3"
for pl in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE ${EXTRA_PMC}; do
    WONE_PLANE=$pl timeout -k 10 150 rocprofv3 --pmc $c -d $out/${c}_$pl -o run --output-format csv -- python scripts/microbench.py wone > $out/${c}_$pl.log 2>&1 || exit $?
    python3 scripts/pmc_compact.py $out/${c}_$pl wconv3
  done
done
echo DONE
