set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py tests/test_gpu_reasm.py tests/test_gpu_graph.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r03_segrec_tests.log 2>&1
tail -2 gpurun_out/r03_segrec_tests.log
grep -q 'Fatal\|core dumped\|failed' gpurun_out/r03_segrec_tests.log && exit 1
EXP_MODES=0:0,1:0 timeout -k 10 200 python tools/exp_k1k2.py 3 40 > gpurun_out/r03_exp_segrec2.log 2>&1 || exit 1
EXP_CFG=cfg3 EXP_MODES=0:0,1:0 timeout -k 10 200 python tools/exp_k1k2.py 2 8 > gpurun_out/r03_exp_segrec3.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e > gpurun_out/r03_bench_segrec20.json 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu --no-e2e --no-xor-stream > gpurun_out/r03_bench_segrec100.json 2>&1 || exit 1
