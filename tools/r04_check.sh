# round-4 check: smoke, full GPU suite, driver-style bench (--steps 20 --warmup 5)
set -o pipefail
T=${1:-r04}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gputest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_bench.json
