# round 4 (temporary knob): K2 stores sc0|sc1|nt (aux19 1) vs sc1|nt (0)
set -o pipefail
O="aux19=0|aux19=1"
bash tools/ab_opt.sh r04_aux19 "--steps 100 --warmup 20" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_aux19 "--config cfg3 --steps 20 --warmup 5" "$O" 2 || exit 1
