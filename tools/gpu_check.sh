# GPU box: full GPU test suite, then short benches given as "op:config:options" triples.
#   bash tools/gpu_check.sh "decode:cfg5:path=4" "decode:cfg5:path=3" ...
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for spec in "$@"; do
  IFS=: read -r op cfg opts <<< "$spec"
  WSFRAME_AMD_OPTIONS="$opts" timeout -k 10 300 python bench.py --op "$op" --config "$cfg" --no-cpu --no-e2e --steps 20 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'], d['verified'])"
done
