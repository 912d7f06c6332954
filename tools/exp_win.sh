# GPU box: K2 piece windows A/B (option piece_win = log2 windows), interleaved, twice.
#   bash tools/exp_win.sh "cfg2 cfg3" "0 1 2 3"
set -e
export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in $1; do
    for w in $2; do
      WSFRAME_AMD_OPTIONS="piece_win=$w" timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-e2e --inflight 1 --steps 50 2>/dev/null \
        | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg win=$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'])"
    done
  done
done
