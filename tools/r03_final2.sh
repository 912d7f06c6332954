# round-3 final check on the final code: smoke, full GPU suite, driver-style bench
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03_gputest_final2.log 2>&1
tail -2 gpurun_out/r03_gputest_final2.log
grep -q 'Fatal\|core dumped\|failed' gpurun_out/r03_gputest_final2.log && exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03_bench_final2.json 2> gpurun_out/r03_bench_final2.err || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03_bench_final2.json
