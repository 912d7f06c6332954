#!/bin/bash
# Run on the GPU box: rocprofv3 kernel stats + the bench line OF THE SAME RUN (so every
# quoted fraction and the kernel averages come from one process), separate PMC passes, and
# an untraced full bench line (CPU baseline, end-to-end) beside them.
#   bash tools/profile.sh <outdir> [bench args...]
# Counters are collected in their own runs (never combined with tracing domains).
set -e
OUT=${1:-gpurun_out/prof}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --no-cpu --no-e2e --no-paths --inflight 1 "$@" > "$OUT/trace_stdout.txt" 2> "$OUT/trace.log"
grep '^{"metric"' "$OUT/trace_stdout.txt" | tail -1 > "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-e2e --no-paths --inflight 1 "$@" > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-e2e --no-paths --inflight 1 "$@" > "$OUT/pmc_write.log" 2>&1
if [ -z "$PROFILE_NO_FULL" ]; then
  timeout -k 10 300 python bench.py --no-paths "$@" > "$OUT/bench_full.json" 2> "$OUT/bench_full.err"
fi
