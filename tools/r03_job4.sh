set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_graph.py tests/test_gpu_options.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03_rwdev_tests.log 2>&1
tail -2 gpurun_out/r03_rwdev_tests.log
grep -q 'Fatal\|core dumped\|failed' gpurun_out/r03_rwdev_tests.log && exit 1
for r in 1 2 1 2; do WSFRAME_AMD_OPTIONS=stream_rw=$r timeout -k 10 150 python bench.py --op stream --config cfg3 --steps 10 --warmup 2 > gpurun_out/r03_stream3_rw$r.json 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03_stream3_rw$r.json; done
timeout -k 10 150 python bench.py --op stream --config cfg2 --steps 20 --warmup 5 > gpurun_out/r03_stream2.json 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03_stream2.json
