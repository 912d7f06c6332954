# round 4 (temporary knob): K2's whole-chunk stores as sc1|nt buffer stores (k2_sc1 1) vs nt global stores
set -o pipefail
WSFRAME_AMD_OPTIONS=k2_sc1=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job27_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_job27_tests.log; [ $rc -eq 0 ] || exit 1
O="k2_sc1=0|k2_sc1=1"
bash tools/ab_opt.sh r04_k2sc1 "--steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_k2sc1 "--steps 20 --warmup 5" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_k2sc1 "--config cfg3 --steps 20 --warmup 5" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_k2sc1 "--op stream --config cfg3 --steps 10 --warmup 3" "$O" 2 || exit 1
