# round 4: one-shot in-place XOR blocks by load/store cache policy (buffer aux bits), back to back
set -o pipefail
timeout -k 10 300 python tools/calib.py --modes 16,27,30,31,32,33,34 --iters 10 > gpurun_out/r04_calib_policy2_4g.json 2>&1 || exit 1
grep kernel gpurun_out/r04_calib_policy2_4g.json
