# round 4: K2 at 6 vs 7 blocks per CU with the sc1|nt stores, second box: cfg2 (both protocols), cfg4
set -o pipefail
O="piece_lds=0|piece_lds=23296"
bash tools/ab_opt.sh r04_occ_sc1b "--steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_occ_sc1b "--steps 20 --warmup 5" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_occ_sc1b "--config cfg4 --steps 4 --warmup 1" "$O" 1 || exit 1
