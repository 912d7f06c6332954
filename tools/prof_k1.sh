# GPU box: rocprofv3 kernel stats of the decode for several WSFRAME_AMD_OPTIONS settings
set -e
export TMPDIR=/tmp
i=0
for o in "$@"; do
  WSFRAME_AMD_OPTIONS="$o" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k1_$i -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e > gpurun_out/k1_$i.log 2>&1 || [ $? -eq 1 ]   # 1 = verification mismatch (expected under "debug"); anything else stops
  echo "$o" > gpurun_out/k1_$i/opts.txt
  i=$((i+1))
done
