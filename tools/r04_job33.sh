# round 4 (temporary knob): encode E3 stores: 0 global nt (kept so far), 1 buffer sc0|nt, 2 buffer nt
set -o pipefail
WSFRAME_AMD_OPTIONS=e3aux=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job33_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_job33_tests.log; [ $rc -eq 0 ] || exit 1
O="e3aux=0|e3aux=1|e3aux=2"
bash tools/ab_opt.sh r04_e3aux "--op encode --steps 100 --warmup 20" "$O" 3 || exit 1
