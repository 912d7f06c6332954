# GPU box: K2 HBM traffic (FETCH_SIZE x2 + WRITE_SIZE, per launch) for "config:frames[:plen]"
# workloads, each counter in its own pass (MI355X_MICROARCH.md HBM section)
export TMPDIR=/tmp
for spec in "$@"; do
  IFS=: read -r cfg fr pl <<< "$spec"
  extra=""; [ -n "$pl" ] && extra="--plen $pl"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    rm -rf /tmp/pm_$ctr
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d /tmp/pm_$ctr -o run -- python3 bench.py --config $cfg --frames $fr $extra --steps 2 --warmup 1 --no-cpu --no-e2e > /tmp/pm.log 2>&1 || exit 1
  done
  python - "$spec" <<'PY'
import csv, glob, sys
def avg(ctr):
    f = glob.glob('/tmp/pm_%s/**/*counter_collection.csv' % ctr, recursive=True)[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
         if "ws_piece_unmask" in r["Kernel_Name"] and r["Counter_Name"] == ctr]
    return sum(v) / len(v) * 1024, len(v)
fe, n = avg("FETCH_SIZE")
wr, _ = avg("WRITE_SIZE")
print(sys.argv[1], "K2 launches %d  read %.3f GB (FETCH x2)  write %.3f GB" % (n, 2 * fe / 1e9, wr / 1e9))
PY
done
