set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -2 gpurun_out/gpu_tests.log
bash tools/profile.sh gpurun_out/r01_reasm_fused --op reasm --config cfg5
cat gpurun_out/r01_reasm_fused/bench.json
