# round-4 final evidence after the occupancy rule: piece profiles (cfg4 first), smoke, full GPU suite, driver bench
set -o pipefail
bash tools/gpu_profile_all.sh r04 piece_cfg4 piece piece_cfg3 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_final_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r04_final_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r04_final_gputest.log 2>&1
rc=$?; tail -2 gpurun_out/r04_final_gputest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_final_bench.json 2> gpurun_out/r04_final_bench.err || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04_final_bench.json
