# TEMPORARY: SQ counters of the speculative kernel's debug variants (cfg2, 6 calls each)
set -e
export TMPDIR=/tmp
OUT=$1
mkdir -p "$OUT"
R=$(pwd)
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$R/$OUT" -o run -- python3 "$R/tools/exp_dbg.py" > "$OUT/pmc.log" 2>&1
