set -o pipefail
mkdir -p gpurun_out/r4l
ALCM_PROF_SHAPES=1 ALCM_BENCH_ALL_KERNELS=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --also-other-mode 0 --cpu-baseline 0 --extra-configs 0 --components 0 > gpurun_out/r4l/shapes.json 2> gpurun_out/r4l/shapes.err || exit $?
bash scripts/profile_bench.sh r4l
