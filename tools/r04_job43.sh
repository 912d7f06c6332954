# round 4 (temporary knob): K2's first k2pf/1000 of blocks launched first with cached loads, then the rest
set -o pipefail
WSFRAME_AMD_OPTIONS=k2pf=100 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job43_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04_job43_tests.log; [ $rc -eq 0 ] || exit 1
O="k2pf=0|k2pf=60|k2pf=120|k2pf=250"
bash tools/ab_opt.sh r04_k2pf2 "--steps 100 --warmup 20" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_k2pf2 "--config cfg3 --steps 20 --warmup 5" "$O" 1 || exit 1
