# round 4 (temporary knob): K2 with plain payload loads + nontemporal stores (k2_ld 1) vs nt both
set -o pipefail
O="k2_ld=0|k2_ld=1"
bash tools/ab_opt.sh r04_k2ld "--steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_k2ld "--steps 20 --warmup 5" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_k2ld "--config cfg3 --steps 20 --warmup 5" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_k2ld "--op stream --config cfg3 --steps 10 --warmup 3" "$O" 2 || exit 1
