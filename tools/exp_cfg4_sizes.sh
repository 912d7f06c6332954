export TMPDIR=/tmp
for fr in 65536 131072 262144 358400 524288 1048576; do
  timeout -k 10 300 python bench.py --config cfg4 --frames $fr --no-cpu --no-e2e --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4 frames $fr', d['value'], d['ms_per_step'], d['roofline']['frac'])" || exit 1
done
for fr in 262144 1048576; do
  timeout -k 10 300 python bench.py --config cfg3 --frames $fr --no-cpu --no-e2e --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg3 frames $fr', d['value'], d['ms_per_step'], d['roofline']['frac'])" || exit 1
done
