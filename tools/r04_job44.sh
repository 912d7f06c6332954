# round 4: R1's window loads nontemporal (a build with WS_R1_NT=1) vs cached, raw stream cfg3; parity first
set -o pipefail
WSFRAME_AMD_LIB=$PWD/util_amd/libwsframe_amd_r1nt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_job44_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04_job44_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_lib.sh r04_r1nt "--op stream --config cfg3 --steps 10 --warmup 3|--op stream --config cfg3 --graph --steps 10 --warmup 3" 3 "base r1nt" || exit 1
