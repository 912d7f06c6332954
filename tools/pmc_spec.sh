# GPU box: SQ instruction counters of the decode kernels (one short bench run, default path)
set -e
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
R=$(pwd)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$R/$OUT" -o run -- python3 "$R/bench.py" --steps 4 --warmup 2 --no-cpu --no-e2e --no-xor-stream "$@" > "$OUT/pmc.log" 2>&1
