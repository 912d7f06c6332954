# GPU box: committed evidence for this round — bench line + rocprofv3 kernel stats + PMC
# passes for the headline decode (cfg2), decode of small segments (cfg5, segfuse), fused
# reassembly (cfg5) and client encode (cfg2). Summaries: tools/prof_summary.py (on the CPU side).
set -e
export TMPDIR=/tmp
R=${1:-r01}
bash tools/profile.sh gpurun_out/${R}_piece
bash tools/profile.sh gpurun_out/${R}_segfuse_cfg5 --config cfg5
bash tools/profile.sh gpurun_out/${R}_reasm_fused --op reasm --config cfg5
bash tools/profile.sh gpurun_out/${R}_encode_cfg2 --op encode
bash tools/profile.sh gpurun_out/${R}_stream_cfg3 --op stream --config cfg3
for d in piece segfuse_cfg5 reasm_fused encode_cfg2 stream_cfg3; do echo "== $d"; cut -c1-300 gpurun_out/${R}_$d/bench.json; done
