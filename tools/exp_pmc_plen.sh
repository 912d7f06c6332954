# GPU box: K2 counters (L2 hits/misses, HBM requests, wave cycles) for fixed payload lengths
# at ~23.5 GB of wire — the 12000 B vs 14000 B step of DESIGN.md §4. One pass per group.
#   bash tools/exp_pmc_plen.sh 12000 14000
export TMPDIR=/tmp
for pl in "$@"; do
  fr=$(( 23400000000 / (pl + 14) ))
  i=0
  for ctrs in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES"; do
    i=$((i + 1))
    rm -rf /tmp/pp$i
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d /tmp/pp$i -o run -- python3 bench.py --config cfg2 --frames $fr --plen $pl --steps 2 --warmup 1 --no-cpu --no-e2e > /tmp/pp.log 2>&1 || { tail -5 /tmp/pp.log; exit 1; }
  done
  python - "$pl" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob('/tmp/pp*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if "ws_piece_unmask" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("plen", sys.argv[1], "  ".join("%s %.4g" % (k, sum(v) / len(v)) for k, v in sorted(acc.items())))
PY
done
