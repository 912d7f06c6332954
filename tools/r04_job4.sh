# round-4: fused launch vs K1 + K2 by walker count (is the fused form walker-bound?); stream + encode
set -o pipefail
T=${1:-r04i}
bash tools/ab_opt.sh ${T}_walkers "--steps 20 --warmup 5" "piece_fused=0|piece_fused=1,fused_walkers=64|piece_fused=1,fused_walkers=256|piece_fused=1,fused_walkers=1024" 2 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_stream.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_more.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_more.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 200 python bench.py --op encode --steps 100 --warmup 20 --no-cpu > gpurun_out/${T}_enc_$i.json 2>/dev/null || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_enc_$i.json; done
for i in 1 2; do timeout -k 10 300 python bench.py --op stream --config cfg3 --steps 10 --warmup 3 --no-cpu > gpurun_out/${T}_stream3_$i.json 2>/dev/null || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_stream3_$i.json; done
