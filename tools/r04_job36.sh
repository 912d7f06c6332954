# round 4: the occupancy rule (auto: 7 blocks/CU for segment-dense batches, else 6) vs forced 6
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job36_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_job36_tests.log; [ $rc -eq 0 ] || exit 1
O="piece_lds=0|piece_lds=27136"
bash tools/ab_opt.sh r04_occ_rule "--steps 20 --warmup 5" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_occ_rule "--steps 100 --warmup 20" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_occ_rule "--config cfg3 --steps 20 --warmup 5" "$O" 2 || exit 1
