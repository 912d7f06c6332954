# A/B of library options (WSFRAME_AMD_OPTIONS), interleaved on one box:
#   bash tools/ab_opt.sh <tag> "<bench args>" "<opts>|<opts>|..." [rounds]
set -o pipefail
tag=$1; args=$2; IFS='|' read -ra OPTS <<< "$3"; rounds=${4:-3}
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for o in "${OPTS[@]}"; do
    WSFRAME_AMD_OPTIONS="$o" timeout -k 10 180 python bench.py $args --no-cpu --no-e2e --no-xor-stream > gpurun_out/ab_one.json 2>/dev/null || { echo "FAIL $o"; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/ab_one.json'));r=d['roofline']
print('$o', '$args', d['ms_per_step'], r['frac'], r.get('kernel_ms_mean'), d['verified'])" | tee -a gpurun_out/ab_$tag.log
  done
done
