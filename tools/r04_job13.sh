# round 4: captured stream replays skip the pass rounds on the device; R1 checks each
# candidate's second header (stream_r1v); chunk windows from the sample's mean and longest
# frame (stream_rw_h); then re-profile the stream workloads on the final K2
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job13_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_job13_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_options.py -x -q --timeout 120 --timeout-method thread -k "stream" > gpurun_out/r04_job13_opts.log 2>&1
rc=$?; tail -3 gpurun_out/r04_job13_opts.log; [ $rc -eq 0 ] || exit 1
O="stream_r1v=0,stream_rw_h=0|stream_r1v=1,stream_rw_h=0|stream_r1v=0,stream_rw_h=1|stream_r1v=1,stream_rw_h=1"
bash tools/ab_opt.sh r04_r1v "--op stream --config cfg3 --steps 10 --warmup 3" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_r1v "--op stream --config cfg3 --graph --steps 10 --warmup 3" "$O" 1 || exit 1
bash tools/gpu_profile_all.sh r04 stream_cfg3 stream_cfg3_graph stream_cfg2 || exit 1
