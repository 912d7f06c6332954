# round 4 (temporary knob): K2 payload loads as buffer loads with sc1|nt (k2ld 1) or sc0|nt (2) vs global nt (0)
set -o pipefail
WSFRAME_AMD_OPTIONS=k2ld=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job31_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_job31_tests.log; [ $rc -eq 0 ] || exit 1
O="k2ld=0|k2ld=1|k2ld=2"
bash tools/ab_opt.sh r04_k2ld2 "--steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_k2ld2 "--config cfg3 --steps 20 --warmup 5" "$O" 2 || exit 1
