# round-4: same-box A/B of the round-3 library (ab_r03/, built from c51ee51) against this one
set -o pipefail
T=${1:-r04l}
one() {  # tag, bench path, args
  timeout -k 10 300 python $2 $3 --no-cpu --no-e2e --no-xor-stream > gpurun_out/ab_one.json 2>/dev/null || { echo "FAIL $1"; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab_one.json'));r=d['roofline']
print('$1', '$3', d['ms_per_step'], r['frac'], r.get('kernel_ms_mean'), d['verified'])" | tee -a gpurun_out/ab_${T}.log
}
for r in 1 2; do
  one r03 ab_r03/bench.py "--config cfg4 --steps 4 --warmup 1"
  one r04 bench.py "--config cfg4 --steps 4 --warmup 1"
done
for r in 1 2; do
  one r03 ab_r03/bench.py "--steps 100 --warmup 20"
  one r04 bench.py "--steps 100 --warmup 20"
  one r03 ab_r03/bench.py "--config cfg3 --steps 20 --warmup 5"
  one r04 bench.py "--config cfg3 --steps 20 --warmup 5"
done
