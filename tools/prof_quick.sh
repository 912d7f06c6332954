# GPU box: kernel stats + FETCH_SIZE/WRITE_SIZE passes of one short bench config.
#   bash tools/prof_quick.sh <outdir> <WSFRAME_AMD_OPTIONS> [bench args...]
set -e
export TMPDIR=/tmp
OUT=$1; OPTS=$2; shift 2
mkdir -p "$OUT"
export WSFRAME_AMD_OPTIONS="$OPTS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e "$@" > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-e2e "$@" > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-e2e "$@" > "$OUT/pmc_write.log" 2>&1
