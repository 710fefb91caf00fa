#!/bin/bash
# Round-3 final call: -m gpu suite + text-encoder A/B (scripts/gpu_text_ab.sh), the default bench line, rocprofv3 stats + PMC passes of HEAD (scripts/profile_bench.sh).  Usage: bash scripts/gpu_final.sh <tag>
tag=${1:-r3f}
bash scripts/gpu_text_ab.sh ${tag}_text || exit $?
mkdir -p gpurun_out/$tag
timeout -k 10 400 python -u bench.py > gpurun_out/$tag/bench.log 2>&1 || exit $?
bash scripts/profile_bench.sh $tag
