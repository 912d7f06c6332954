set -o pipefail
timeout -k 10 200 python tools/exp_stream_k2.py cfg3 2 6 > gpurun_out/r03_exp_stream_k2b.log 2>&1 || exit 1
tail -1 gpurun_out/r03_exp_stream_k2b.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -m gpu -q --timeout 120 --timeout-method thread -k stream > gpurun_out/r03_r3_tests2.log 2>&1
tail -2 gpurun_out/r03_r3_tests2.log
grep -q 'Fatal\|core dumped\|failed' gpurun_out/r03_r3_tests2.log && exit 1
PROFILE_NO_FULL=1 bash tools/profile.sh gpurun_out/r03y_stream_cfg3_graph --op stream --config cfg3 --graph --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
