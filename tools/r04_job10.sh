# round-4: R3 group owner walks — parity (stream, graph, options), then same-box A/B
set -o pipefail
T=${1:-r04p}
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_stream.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_stream.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_options.py -k "stream" -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_options.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_options.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_opt.sh ${T}_own "--op stream --config cfg3 --steps 10 --warmup 3" "stream_own=0|stream_own=1" 3 || exit 1
bash tools/ab_opt.sh ${T}_owng "--op stream --config cfg3 --graph --steps 10 --warmup 3" "stream_own=0|stream_own=1" 2 || exit 1
