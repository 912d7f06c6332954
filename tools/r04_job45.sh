# round 4: K2 windows (piece_win 0/1/2) re-checked at 7 blocks/CU with the sc1|nt stores (cfg2)
set -o pipefail
bash tools/ab_opt.sh r04_win7 "--steps 100 --warmup 20" "piece_win=1|piece_win=2|piece_win=0" 2 || exit 1
