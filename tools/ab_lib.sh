# A/B of builds of libwsframe_amd.so, interleaved on one box:
#   bash tools/ab_lib.sh <tag> "<bench args>|<bench args>|..." [rounds] [libs]
# libs: space-separated names; "new" = util_amd/libwsframe_amd.so, X = util_amd/libwsframe_amd_X.so
# (default "base new")
set -o pipefail
tag=$1; IFS='|' read -ra CASES <<< "$2"; rounds=${3:-3}; libs=${4:-base new}
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for lib in $libs; do
    for c in "${CASES[@]}"; do
      if [ $lib = new ]; then unset WSFRAME_AMD_LIB; else export WSFRAME_AMD_LIB=$PWD/util_amd/libwsframe_amd_$lib.so; fi
      timeout -k 10 180 python bench.py $c --no-cpu --no-e2e --no-xor-stream > gpurun_out/ab_one.json 2>/dev/null || { echo "FAIL $lib $c"; exit 1; }
      python -c "
import json,sys;d=json.load(open('gpurun_out/ab_one.json'));r=d['roofline']
print('$lib', '$c'.strip(), d['ms_per_step'], r['frac'], r.get('kernel_ms_mean'), d['verified'])" | tee -a gpurun_out/ab_$tag.log
    done
  done
done
