# GPU box: committed evidence for this round — bench line + rocprofv3 kernel stats + PMC
# passes per workload (tools/profile.sh). Summaries: tools/prof_all_summary.sh (CPU side).
#   bash tools/gpu_profile_all.sh r02 [names...]
set -e
export TMPDIR=/tmp
R=${1:-r03}; shift || true
# the driver's protocol (20 timed calls after 5 warm-up calls) unless PROFILE_STEPS says otherwise:
# the bench line's `paths` entries are cross-checked against these profiles
P=${PROFILE_STEPS:-"--steps 20 --warmup 5"}
ALL="piece piece_cfg3 piece_cfg4 segfuse_cfg5 reasm_fused encode_cfg2 stream_cfg2 stream_cfg3 stream_cfg3_graph"
for n in ${@:-$ALL}; do
  case $n in
    piece)        bash tools/profile.sh gpurun_out/${R}_piece $P ;;
    piece_cfg3)   bash tools/profile.sh gpurun_out/${R}_piece_cfg3 --config cfg3 --no-cpu --no-e2e $P ;;
    piece_cfg4)   bash tools/profile.sh gpurun_out/${R}_piece_cfg4 --config cfg4 --steps 10 --warmup 2 ;;
    segfuse_cfg5) bash tools/profile.sh gpurun_out/${R}_segfuse_cfg5 --config cfg5 --no-cpu --no-e2e $P ;;
    reasm_fused)  bash tools/profile.sh gpurun_out/${R}_reasm_fused --op reasm --config cfg5 --readcache 1048576 $P ;;
    encode_cfg2)  bash tools/profile.sh gpurun_out/${R}_encode_cfg2 --op encode $P ;;
    stream_cfg2)  bash tools/profile.sh gpurun_out/${R}_stream_cfg2 --op stream --config cfg2 $P ;;
    stream_cfg3)  bash tools/profile.sh gpurun_out/${R}_stream_cfg3 --op stream --config cfg3 $P ;;
    stream_cfg3_graph) bash tools/profile.sh gpurun_out/${R}_stream_cfg3_graph --op stream --config cfg3 --graph $P ;;
  esac
  echo "== $n"; cut -c1-200 gpurun_out/${R}_$n/bench.json
done
