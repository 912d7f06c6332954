# round 4: full check after the stream changes + the 2-rank launcher rehearsal on one GPU
set -o pipefail
bash tools/r04_check.sh r04_j18 || exit 1
WS_BENCH_RANKS_PER_GPU=2 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-e2e > gpurun_out/r04_j18_gpus2.json 2> gpurun_out/r04_j18_gpus2.err || exit 1
cut -c1-400 gpurun_out/r04_j18_gpus2.json
