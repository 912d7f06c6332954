# round 4: stream tests after the walk changes; chunk-size A/B on cfg3 (stream_rw_cmax 21/22/23)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job14_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_job14_tests.log; [ $rc -eq 0 ] || exit 1
O="stream_rw_cmax=23|stream_rw_cmax=22|stream_rw_cmax=21"
bash tools/ab_opt.sh r04_cmax "--op stream --config cfg3 --steps 10 --warmup 3" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_cmax "--op stream --config cfg3 --graph --steps 10 --warmup 3" "$O" 2 || exit 1
