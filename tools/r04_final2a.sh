# round-4 final evidence (part 1) on the final code: piece (cfg4 first), cfg2, cfg3, segfuse, reassembly
set -o pipefail
bash tools/gpu_profile_all.sh r04 piece_cfg4 piece piece_cfg3 segfuse_cfg5 reasm_fused || exit 1
