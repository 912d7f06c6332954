# GPU box: A/B of library options (WSFRAME_AMD_OPTIONS strings) on bench workloads, interleaved, twice.
#   bash tools/exp_opt.sh "decode:cfg5 reasm:cfg5" "seg_win=0 seg_win=1"
set -e
export TMPDIR=/tmp
for rep in 1 2; do
  for w in $1; do
    op=${w%%:*}; cfg=${w##*:}
    for o in $2; do
      WSFRAME_AMD_OPTIONS="$o" timeout -k 10 300 python bench.py --op $op --config $cfg --no-cpu --no-e2e --inflight 1 --steps 50 2>/dev/null \
        | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$op $cfg $o', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'])"
    done
  done
done
