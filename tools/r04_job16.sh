# round 4 (temporary knob): the chunk window's mean-frame multiple (stream_rw_hm 4 / 2 / 0) x the largest chunk
set -o pipefail
O="stream_rw_hm=4|stream_rw_hm=2|stream_rw_hm=0|stream_rw_hm=0,stream_rw_cmax=21|stream_rw_hm=0,stream_rw_cmax=23"
bash tools/ab_opt.sh r04_hm "--op stream --config cfg3 --steps 10 --warmup 3" "$O" 2 || exit 1
bash tools/ab_opt.sh r04_hm "--op stream --config cfg3 --graph --steps 10 --warmup 3" "$O" 1 || exit 1
