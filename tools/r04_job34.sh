# round 4: K2 occupancy re-check after the sc1|nt stores (piece_lds: 0 = 6 blocks/CU, 23296 = 7, 32512 = 5)
set -o pipefail
O="piece_lds=0|piece_lds=23296|piece_lds=32512"
bash tools/ab_opt.sh r04_occ_sc1 "--steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_occ_sc1 "--config cfg3 --steps 20 --warmup 5" "$O" 2 || exit 1
