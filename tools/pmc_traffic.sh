# GPU box: FETCH_SIZE / WRITE_SIZE (and L2 hit/miss) per kernel of a short bench run
#   bash tools/pmc_traffic.sh <outdir> <WSFRAME_AMD_OPTIONS> [bench args...]
set -e
export TMPDIR=/tmp
OUT=$1; OPTS=$2; shift 2
mkdir -p "$OUT"
export WSFRAME_AMD_OPTIONS="$OPTS"
R=$(pwd)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$OUT/f" -o run -- python3 "$R/bench.py" --steps 4 --warmup 2 --no-cpu --no-e2e --no-xor-stream "$@" > "$OUT/f.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$OUT/w" -o run -- python3 "$R/bench.py" --steps 4 --warmup 2 --no-cpu --no-e2e --no-xor-stream "$@" > "$OUT/w.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$R/$OUT/h" -o run -- python3 "$R/bench.py" --steps 4 --warmup 2 --no-cpu --no-e2e --no-xor-stream "$@" > "$OUT/h.log" 2>&1
