# round 4: the occupancy rule's threshold: cfg2 frames in 32- and 64-frame segments (1 segment per 8 / 16
# pieces) at forced 6 (27136) vs forced 7 (23296) blocks per CU
set -o pipefail
O="piece_lds=27136|piece_lds=23296"
bash tools/ab_opt.sh r04_occ_thr "--fps 32 --steps 100 --warmup 20" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_occ_thr "--fps 64 --steps 100 --warmup 20" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_occ_thr "--fps 8 --steps 100 --warmup 20" "$O" 2 || exit 1
