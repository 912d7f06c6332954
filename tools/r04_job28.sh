# round 4 (temporary knob): encode E3, segfuse and fused-reassembly payload stores as sc1|nt buffer stores
set -o pipefail
WSFRAME_AMD_OPTIONS=st_sc1=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_reasm.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job28_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_job28_tests.log; [ $rc -eq 0 ] || exit 1
O="st_sc1=0|st_sc1=1"
bash tools/ab_opt.sh r04_stsc1 "--op encode --steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_stsc1 "--config cfg5 --steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_stsc1 "--op reasm --config cfg5 --steps 100 --warmup 20" "$O" 3 || exit 1
