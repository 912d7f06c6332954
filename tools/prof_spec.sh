# GPU box: speculative vs classic piece path on cfg2 (bench lines + rocprofv3 kernel stats).
#   bash tools/prof_spec.sh <outdir>
set -e
export TMPDIR=/tmp
OUT=$1
mkdir -p "$OUT"
R=$(pwd)
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --no-xor-stream > "$OUT/spec.json" 2> "$OUT/spec.err"
WSFRAME_AMD_OPTIONS=piece_spec=0 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --no-xor-stream > "$OUT/classic.json" 2> "$OUT/classic.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/trace" -o run -- python3 "$R/bench.py" --steps 10 --warmup 5 --no-cpu --no-e2e --no-xor-stream > "$OUT/trace.log" 2>&1
