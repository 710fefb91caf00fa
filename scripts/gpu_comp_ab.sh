#!/bin/bash
# A/B of knob settings on bench.py's SURVEY §8(f) component lines (text encoders, mel + Encoder1D), alternating,
# two rounds.  Usage: bash scripts/gpu_comp_ab.sh <tag> "<variant> ..." (variant as in gpu_run.sh)
tag=${1:-comp}
variants=${2:-"-"}
out=gpurun_out/$tag; mkdir -p $out
ARGS="--steps 5 --warmup 2 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 1"
for round in 1 2; do
  for v in $variants; do
    envs=""
    [ "$v" != "-" ] && envs=$(echo "$v" | tr ',' ' ')
    name=$(echo "$v" | tr ',=' '_-')
    env $envs ALCM_PROF_SHAPES=1 ALCM_BENCH_ALL_KERNELS=1 timeout -k 10 300 python -u bench.py $ARGS \
      > $out/c_${round}_$name.json 2> $out/c_${round}_$name.err || exit $?
    echo "$v: $(python -c "
import json;d=json.load(open('$out/c_${round}_$name.json'))
print(d['ms_per_step'], {k: c.get('ms_per_call') for k, c in d.get('components', {}).items()})")" >> $out/ab.txt
  done
done
cat $out/ab.txt
