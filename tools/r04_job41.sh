# round 4: K1 alphabet speculation on/off on cfg3 with the final K2 (sc1 stores, occupancy rule)
set -o pipefail
bash tools/ab_opt.sh r04_alpha_final "--config cfg3 --steps 20 --warmup 5" "scan_alpha=1|scan_alpha=0" 3 || exit 1
