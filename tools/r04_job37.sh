# round 4: fused reassembly geometries (reasm_cfg 0/1/2) now that all use sc1|nt body stores
set -o pipefail
O="reasm_cfg=0|reasm_cfg=1|reasm_cfg=2"
bash tools/ab_opt.sh r04_reasm_cfg "--op reasm --config cfg5 --steps 100 --warmup 20" "$O" 3 || exit 1
