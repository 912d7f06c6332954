# GPU box: refreshed evidence after the two-window K2 / segment order:
# headline cfg2, cfg3, cfg4 (piece path), cfg5 segfuse decode, cfg5 fused reassembly.
set -e
export TMPDIR=/tmp
bash tools/profile.sh gpurun_out/p_piece
bash tools/profile.sh gpurun_out/p_piece_cfg4 --config cfg4 --steps 30
bash tools/profile.sh gpurun_out/p_piece_cfg3 --config cfg3 --steps 30
bash tools/profile.sh gpurun_out/p_segfuse_cfg5 --config cfg5
bash tools/profile.sh gpurun_out/p_reasm_fused --op reasm --config cfg5
for d in piece piece_cfg4 piece_cfg3 segfuse_cfg5 reasm_fused; do echo "== $d"; cut -c1-200 gpurun_out/p_$d/bench.json; done
