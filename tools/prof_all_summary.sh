# CPU side: profiles/<R>_* summaries from gpurun_out/<R>_* (tools/gpu_profile_all.sh)
#   bash tools/prof_all_summary.sh r02
set -e
R=${1:-r03}
K2=ws_piece_unmask_kernel
S() { if [ -d gpurun_out/${R}_$1 ]; then python tools/prof_summary.py gpurun_out/${R}_$1 ${R}_$1 --kernel $2 $3 > /dev/null && echo "${R}_$1"; fi; }
S piece $K2,ws_piece_scan_kernel
S piece_cfg3 $K2,ws_piece_scan_kernel
S piece_cfg4 $K2,ws_piece_scan_kernel
S segfuse_cfg5 ws_segfuse_kernel
S reasm_fused ws_reasm_seg_kernel
S encode_cfg2 ws_enc_copy_kernel,ws_enc_front_kernel,ws_enc_tsum_kernel,ws_enc_tscan_kernel,ws_enc_edge_kernel,ws_enc_ptr_kernel
S stream_cfg2 $K2,ws_stream_pass_kernel,ws_stream_resolve_kernel
# (round 6: the eager cfg3 stream's unmask runs as three launches beside the split walk (captured calls too); its walk
# kernels run partly on the side stream, overlapping the first launch: their sum exceeds the step)
S stream_cfg3 $K2,ws_stream_pass_kernel,ws_stream_resolve_kernel,ws_rw_plan_kernel,ws_rw_own_kernel,ws_rw_cand_kernel,ws_rw_spec_kernel,ws_rw_plink_kernel,ws_rw_pscan_kernel,ws_rw_link_kernel,ws_rw_emit_kernel,ws_rw_chunk_kernel,ws_stream_finish_kernel "--launches-per-step 3"
S stream_cfg3_graph $K2,ws_stream_pass_kernel,ws_stream_resolve_kernel,ws_rw_plan_kernel,ws_rw_own_kernel,ws_rw_cand_kernel,ws_rw_spec_kernel,ws_rw_plink_kernel,ws_rw_pscan_kernel,ws_rw_link_kernel,ws_rw_emit_kernel "--launches-per-step 3"
