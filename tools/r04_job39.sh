# round 4: cfg2 K2 at 7 (rule) vs 8 blocks per CU (piece_lds 19968) with the sc1|nt stores
set -o pipefail
O="piece_lds=0|piece_lds=19968"
bash tools/ab_opt.sh r04_occ8 "--steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_occ8 "--steps 20 --warmup 5" "$O" 2 || exit 1
