# GPU box: per-kernel times (rocprofv3 kernel trace) of the decode for "config:frames" pairs
export TMPDIR=/tmp
for spec in "$@"; do
  cfg=${spec%%:*}; fr=${spec##*:}
  rm -rf /tmp/pk
  timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/pk -o run -- python bench.py --config $cfg --frames $fr --no-cpu --no-e2e --steps 10 --warmup 3 > /tmp/pk.log 2>&1 || exit 1
  python - "$spec" <<'PY'
import sqlite3, glob, sys
db = glob.glob('/tmp/pk/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
out = []
for r in c.execute("select name, count(*), avg(end-start)/1e3, min(end-start)/1e3 from kernels where name like '%ws_piece%' or name like '%ws_walker%' group by name"):
    out.append("%s n%d avg %.1f min %.1f us" % (r[0][:28], r[1], r[2], r[3]))
print(sys.argv[1], " | ".join(out))
PY
done
