# round-4: fused debug + parity + A/B; encode exact records check
set -o pipefail
T=${1:-r04g}
timeout -k 10 200 python tools/dbg_fused.py > gpurun_out/${T}_dbg.log 2>&1 || { tail -5 gpurun_out/${T}_dbg.log; exit 1; }
cat gpurun_out/${T}_dbg.log | grep -v amdgpu.ids
grep -q "^1 .*bad bytes [1-9]" gpurun_out/${T}_dbg.log && exit 1
bash tools/r04_fused.sh ${T} || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_options.py -k "enc" -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_enc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_enc_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 200 python bench.py --op encode --steps 100 --warmup 20 --no-cpu > gpurun_out/${T}_enc_$i.json 2>/dev/null || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_enc_$i.json; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_stream_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_stream_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 300 python bench.py --op stream --config cfg3 --steps 10 --warmup 3 --no-cpu > gpurun_out/${T}_stream3_$i.json 2>/dev/null || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_stream3_$i.json; done
