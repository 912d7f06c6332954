# round 4 (temporary knob): segfuse / fused-reassembly LDS-DMA fill policy: 0 nt, 1 sc1|nt, 2 sc0|nt
set -o pipefail
WSFRAME_AMD_OPTIONS=fill=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_reasm.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "reasm or reassemble or segfuse or cfg5 or path" > gpurun_out/r04_job32_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_job32_tests.log; [ $rc -eq 0 ] || exit 1
O="fill=0|fill=1|fill=2"
bash tools/ab_opt.sh r04_fill "--config cfg5 --steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_fill "--op reasm --config cfg5 --steps 100 --warmup 20" "$O" 3 || exit 1
