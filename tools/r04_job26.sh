# round 4: back-to-back streaming rate of one-shot in-place XOR blocks by cache policy (buffer
# loads/stores: nt, plain, sc1, sc1|nt, sc0|nt) at cfg2's and a 5x larger byte count
set -o pipefail
timeout -k 10 300 python tools/calib.py --modes 16,17,18,19,20,26,27 --iters 10 > gpurun_out/r04_calib_policy_4g.json 2>&1 || exit 1
cat gpurun_out/r04_calib_policy_4g.json
timeout -k 10 300 python tools/calib.py --modes 16,18,27,19 --iters 4 --bytes 23000000000 > gpurun_out/r04_calib_policy_23g.json 2>&1 || exit 1
cat gpurun_out/r04_calib_policy_23g.json
