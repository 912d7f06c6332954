# round-4: cfg4 K2 r03 vs r04 vs K1 variants (own64: a lane writes all its frame's pointers; noearly:
# the walk takes its end round), alternating
set -o pipefail
T=${1:-r04r}
one() {
  timeout -k 10 300 python $2 $3 --no-cpu --no-e2e --no-xor-stream > gpurun_out/ab_one.json 2>/dev/null || { echo "FAIL $1"; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab_one.json'));r=d['roofline']
print('$1', '$3', d['ms_per_step'], r['frac'], r.get('kernel_ms_mean'), d['verified'])" | tee -a gpurun_out/ab_${T}.log
}
A="--config cfg4 --steps 4 --warmup 1"
for r in 1 2; do one r03 ab_r03/bench.py "$A"; one r04 bench.py "$A"; one own64 ab_own64/bench.py "$A"; one noearly ab_noearly/bench.py "$A"; done
