# round 4: descriptor stores nontemporal (a build with WS_DESC_NT=1) vs plain, same box
set -o pipefail
bash tools/ab_lib.sh r04_descnt "--steps 100 --warmup 20|--config cfg3 --steps 20 --warmup 5" 3 "base descnt" || exit 1
