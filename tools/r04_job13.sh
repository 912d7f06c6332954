# round 4: captured stream replays skip the pass rounds on the device; re-profile the stream,
# encode, segfuse and reassembly workloads on the final K2
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job13_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_job13_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_profile_all.sh r04 stream_cfg3 stream_cfg3_graph stream_cfg2 encode_cfg2 segfuse_cfg5 reasm_fused || exit 1
