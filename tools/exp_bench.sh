# GPU box: short benches given as "op:config:options" triples, no tests (A/B sweeps).
#   bash tools/exp_bench.sh "decode:cfg5:nt=0" "decode:cfg5:segfuse_cfg=1" ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  IFS=: read -r op cfg opts <<< "$spec"
  WSFRAME_AMD_OPTIONS="$opts" timeout -k 10 300 python bench.py --op "$op" --config "$cfg" --no-cpu --no-e2e --steps ${STEPS:-50} 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'])" || exit 1
done
