# round 4: the raw stream's K2 at 7 blocks/CU (piece_lds 23296) vs the default 6 (one segment)
set -o pipefail
O="piece_lds=0|piece_lds=23296"
bash tools/ab_opt.sh r04_stream_occ "--op stream --config cfg2 --steps 50 --warmup 10" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_stream_occ "--op stream --config cfg3 --steps 10 --warmup 3" "$O" 2 || exit 1
