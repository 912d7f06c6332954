#!/bin/bash
# One parameterised GPU-box job script (replaces the per-round r0x_job*/r0x_final* scripts).
# Every GPU step runs under its own time limit; the first failure ends the job.
#
#   bash tools/gpu_job.sh check <tag>                 smoke + full GPU suite + driver-protocol bench
#   bash tools/gpu_job.sh profile <round> <names...>  tools/gpu_profile_all.sh (trace + PMC per workload)
#   bash tools/gpu_job.sh ab <tag> <reps> "<label>|<bench args>" ...
#                                                     interleaved A/B of bench lines, one log line each
#   bash tools/gpu_job.sh bench <tag> <bench args...> one bench line into gpurun_out/<tag>.json
#
# Environment for a bench line of an A/B arm can be given as "label|ENV=v ENV2=w -- args".
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
mode=$1; shift

bench_line() {  # out.json, args...
  local out=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$out" 2> "${out%.json}.err"
}

case $mode in
  check)
    T=${1:-check}
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
      > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
    tail -1 gpurun_out/${T}_smoke.log
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/${T}_gputest.log 2>&1
    rc=$?; tail -3 gpurun_out/${T}_gputest.log; [ $rc -eq 0 ] || exit 1
    bench_line gpurun_out/${T}_bench.json --steps 20 --warmup 5 || exit 1
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_bench.json
    ;;
  profile)
    R=$1; shift
    bash tools/gpu_profile_all.sh "$R" "$@" || exit 1
    ;;
  ab)
    T=$1; reps=$2; shift 2
    for ((r = 0; r < reps; r++)); do
      for arm in "$@"; do
        label=${arm%%|*}; spec=${arm#*|}
        envs=""; args=$spec
        if [[ $spec == *" -- "* ]]; then envs=${spec%% -- *}; args=${spec#* -- }; fi
        env $envs timeout -k 10 400 python bench.py $args --no-cpu --no-e2e --no-xor-stream --no-paths \
          > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err || { echo "FAIL $label"; tail -5 gpurun_out/ab_one.err; exit 1; }
        python - "$label" "$args" >> gpurun_out/ab_${T}.log <<'EOF'
import json, sys
d = json.load(open('gpurun_out/ab_one.json')); r = d['roofline']
print(sys.argv[1], '|', sys.argv[2], '|', d['ms_per_step'], round(r['frac'], 4),
      r.get('kernel_ms_mean'), d['verified'])
EOF
        tail -1 gpurun_out/ab_${T}.log
      done
    done
    ;;
  bench)
    T=$1; shift
    bench_line gpurun_out/${T}.json "$@" || exit 1
    cut -c1-400 gpurun_out/${T}.json
    ;;
  *)
    echo "usage: $0 check|profile|ab|bench ..." >&2; exit 2 ;;
esac
