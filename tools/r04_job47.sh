# round 4: occupancy from the frame-length hint (rule, piece_lds 0) vs forced 6 (27136), cfg2 at 16/64/8
# frames per segment and cfg3
set -o pipefail
O="piece_lds=0|piece_lds=27136"
bash tools/ab_opt.sh r04_occ_hint "--steps 100 --warmup 20" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_occ_hint "--steps 20 --warmup 5" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_occ_hint "--fps 64 --steps 100 --warmup 20" "$O" 1 || exit 1
bash tools/ab_opt.sh r04_occ_hint "--fps 8 --steps 100 --warmup 20" "$O" 1 || exit 1
bash tools/ab_opt.sh r04_occ_hint "--config cfg3 --steps 20 --warmup 5" "$O" 1 || exit 1
