# round 4 (temporary knob): the raw stream's K2 with plain payload stores (k2_st 1) vs nontemporal
set -o pipefail
O="k2_st=0|k2_st=1"
bash tools/ab_opt.sh r04_k2st "--op stream --config cfg3 --steps 10 --warmup 3" "$O" 3 || exit 1
bash tools/ab_opt.sh r04_k2st "--op stream --config cfg2 --steps 50 --warmup 10" "$O" 2 || exit 1
