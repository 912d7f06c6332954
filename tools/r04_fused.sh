# round-4: the fused K1+K2 launch — parity first, then an interleaved A/B against K1 + K2
set -o pipefail
T=${1:-r04f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused" -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_parity.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_options.py -k "fused" -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_options.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_options.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_opt.sh ${T}_drv "--steps 20 --warmup 5" "piece_fused=0|piece_fused=1" 3 || exit 1
bash tools/ab_opt.sh ${T}_100 "--steps 100 --warmup 20" "piece_fused=0|piece_fused=1|piece_fused=1,fused_walkers=32|piece_fused=1,fused_walkers=128" 2 || exit 1
