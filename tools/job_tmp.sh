set -o pipefail
A="--op stream --config cfg3 --steps 20 --warmup 5"
O=WSFRAME_AMD_OPTIONS
bash tools/gpu_job.sh ab split3 2 "s16|$O=stream_split=16 -- $A" "s16p1|$O=stream_split=16,stream_side_prio=1 -- $A" "s24p1|$O=stream_split=24,stream_side_prio=1 -- $A" "s32p1|$O=stream_split=32,stream_side_prio=1 -- $A" "s16p2|$O=stream_split=16,stream_side_prio=2 -- $A" "s24|$O=stream_split=24 -- $A" "s0|$O=stream_split=0 -- $A"
