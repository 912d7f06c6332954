# round 4 (temporary knob): K2's first k2_pf/1000 of blocks with plain (cached) payload loads
set -o pipefail
O="k2_pf=0|k2_pf=50|k2_pf=100|k2_pf=200"
bash tools/ab_opt.sh r04_k2pf "--steps 100 --warmup 20" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_k2pf "--config cfg3 --steps 20 --warmup 5" "$O" 2 || exit 1
