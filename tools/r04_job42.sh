# round 4: encode edge-chunk stores nontemporal (a build with WS_EDGE_NT=1) vs plain, same box; parity first
set -o pipefail
WSFRAME_AMD_LIB=$PWD/util_amd/libwsframe_amd_edgent.so timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job42_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04_job42_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_lib.sh r04_edgent "--op encode --steps 100 --warmup 20" 3 "base edgent" || exit 1
