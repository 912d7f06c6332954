# round-3 final GPU evidence: full GPU suite, the driver-style bench, profiles of the final code
set -o pipefail
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03_gputest_final.log 2>&1
tail -2 gpurun_out/r03_gputest_final.log
grep -q 'Fatal\|core dumped\|failed' gpurun_out/r03_gputest_final.log && exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03_bench_final.json 2> gpurun_out/r03_bench_final.err || exit 1
bash tools/gpu_profile_all.sh r03 piece piece_cfg3 > gpurun_out/r03_prof_final.log 2>&1 || exit 1
