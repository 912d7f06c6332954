# round-4: K1 stores write-through (ab_wt/, WALK_WT=1) vs plain, same box, alternating
set -o pipefail
T=${1:-r04q}
one() {
  timeout -k 10 300 python $2 $3 --no-cpu --no-e2e --no-xor-stream > gpurun_out/ab_one.json 2>/dev/null || { echo "FAIL $1"; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab_one.json'));r=d['roofline']
print('$1', '$3', d['ms_per_step'], r['frac'], r.get('kernel_ms_mean'), d['verified'])" | tee -a gpurun_out/ab_${T}.log
}
for r in 1 2 3; do
  one plain bench.py "--steps 100 --warmup 20"; one wt ab_wt/bench.py "--steps 100 --warmup 20"
done
for r in 1 2; do
  one plain bench.py "--steps 20 --warmup 5"; one wt ab_wt/bench.py "--steps 20 --warmup 5"
  one plain bench.py "--config cfg3 --steps 20 --warmup 5"; one wt ab_wt/bench.py "--config cfg3 --steps 20 --warmup 5"
done
