# round-3 GPU job (owner-walk speculation check + K2 clock counters, batch vs raw stream on cfg3)
set -o pipefail
timeout -k 10 200 python tools/exp_stream_k2.py cfg3 2 6 > gpurun_out/r03_exp_stream_k2.log 2>&1 || exit 1
tail -1 gpurun_out/r03_exp_stream_k2.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_graph.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03_r3_tests.log 2>&1
tail -2 gpurun_out/r03_r3_tests.log
grep -q 'Fatal\|core dumped\|failed' gpurun_out/r03_r3_tests.log && exit 1
PROFILE_NO_FULL=1 bash tools/profile.sh gpurun_out/r03x_stream_cfg3_graph --op stream --config cfg3 --graph --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
timeout -k 10 150 python bench.py --op stream --config cfg3 --steps 10 --warmup 2 > gpurun_out/r03_stream_cfg3.json 2>&1 || exit 1
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r03_clk_batch -o run -- python3 bench.py --config cfg3 --steps 4 --warmup 1 --no-cpu --no-e2e --no-xor-stream > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r03_clk_stream -o run -- python3 bench.py --op stream --config cfg3 --steps 4 --warmup 1 > /dev/null 2>&1 || exit 1
