# GPU box: spec-kernel A/B for the chunk-parallel stream walk (chunk size x phase-B on/off).
#   bash tools/exp_stream_spec.sh "22:0" "22:128" ...   (log2 chunk : debug flags)
export TMPDIR=/tmp; mkdir -p gpurun_out
for cfg in "$@"; do
  cm=${cfg%%:*}; dbg=${cfg##*:}
  rm -rf /tmp/pab
  WSFRAME_AMD_OPTIONS="stream_rw_cmax=$cm,debug=$dbg" timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/pab -o run -- python bench.py --op stream --config cfg3 --no-cpu --no-e2e --steps 3 --warmup 1 > /tmp/pab.log 2>&1
  rc=$?; [ $rc -le 1 ] || exit 1     # 1: the A/B run's own verification (phase B off) fails
  python - "$cfg" <<'PY'
import sqlite3, glob, sys
db = glob.glob('/tmp/pab/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
out = []
for k in ("ws_rw_cand", "ws_rw_spec", "ws_rw_own", "ws_rw_emit", "void ws_piece_unmask"):
    r = list(c.execute("select count(*), avg(end-start)/1e3 from kernels where name like ?", (k + "%",)))[0]
    out.append("%s %d x %.1f us" % (k, r[0], r[1] or 0))
print(sys.argv[1], " | ".join(out))
PY
done
