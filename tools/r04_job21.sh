# round 4 (temporary knob): the headline without K1's stride hint from the previous call
set -o pipefail
O="nohint=0|nohint=1"
bash tools/ab_opt.sh r04_nohint "--steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_nohint "--steps 20 --warmup 5" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_nohint "--config cfg3 --steps 20 --warmup 5" "$O" 2 || exit 1
