# GPU box: cfg4-size decode vs rx segment size and K2 store mode
export TMPDIR=/tmp
run() { WSFRAME_AMD_OPTIONS="$2" timeout -k 10 300 python bench.py --config cfg4 --frames 358400 $1 --no-cpu --no-e2e --steps 10 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'])"; }
run "--fps 1" "" && run "--fps 4" "" && run "--fps 16" "" && run "--fps 64" "" && run "--fps 16" "piece_whole=0" && run "--fps 16" "piece_whole=1" && run "--fps 16" "nt=0" && run "--fps 16" "nt=2"
