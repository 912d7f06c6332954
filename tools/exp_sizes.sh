set -e
for spec in "cfg2 1048576" "cfg2 4194304" "cfg2 262144" "cfg3 262144" "cfg3 1048576"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --frames $2 --no-cpu --no-e2e --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2', d['ms_per_step'], d['roofline']['frac'], d['verified'])"
done
