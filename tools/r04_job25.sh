# round 4: adaptive speculative width in the stream walk — stream/graph parity, then profiles
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_graph.py tests/test_gpu_c_api.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job25_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_job25_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_options.py -x -q --timeout 120 --timeout-method thread -k "stream" > gpurun_out/r04_job25_opts.log 2>&1
rc=$?; tail -1 gpurun_out/r04_job25_opts.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_profile_all.sh r04 stream_cfg3 stream_cfg3_graph stream_cfg2 || exit 1
