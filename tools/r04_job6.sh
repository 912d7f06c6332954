# round-4: piece_xg (metadata lines in one XCD's L2) parity + same-box A/B + PMC
set -o pipefail
T=${1:-r04k}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "window_mappings or random_streams or golden or cfg4_shape" -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_parity.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_parity.log; [ $rc -eq 0 ] || exit 1
WSFRAME_AMD_OPTIONS=piece_xg=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "piece and (random_streams or golden or full_size or unordered)" -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_parity_xg.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_parity_xg.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_opt.sh ${T}_xg2 "--steps 20 --warmup 5" "piece_xg=0|piece_xg=1" 3 || exit 1
bash tools/ab_opt.sh ${T}_xg2l "--steps 100 --warmup 20" "piece_xg=0|piece_xg=1" 2 || exit 1
bash tools/ab_opt.sh ${T}_xg3 "--config cfg3 --steps 20 --warmup 5" "piece_xg=0|piece_xg=1" 2 || exit 1
export TMPDIR=/tmp
WSFRAME_AMD_OPTIONS=piece_xg=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_xg_fetch -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-e2e --no-xor-stream > gpurun_out/${T}_xg_fetch.log 2>&1 || exit 1
