# GPU box: decode efficiency vs fixed payload length at a fixed wire size (~23.5 GB)
export TMPDIR=/tmp
for pl in "$@"; do
  fr=$(( 23400000000 / (pl + 14) ))
  timeout -k 10 300 python bench.py --config cfg2 --frames $fr --plen $pl --no-cpu --no-e2e --steps 10 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('plen $pl frames $fr', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'])" || exit 1
done
