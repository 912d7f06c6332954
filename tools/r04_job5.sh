# round-4: alphabet speculation in the segment walk, same-box A/B (cfg3 and cfg2)
set -o pipefail
T=${1:-r04j}
bash tools/ab_opt.sh ${T}_alpha3 "--config cfg3 --steps 20 --warmup 5" "scan_alpha=0|scan_alpha=1" 3 || exit 1
bash tools/ab_opt.sh ${T}_alpha2 "--steps 20 --warmup 5" "scan_alpha=0|scan_alpha=1" 3 || exit 1
