# experiment only: the product sources built with 8 KiB pieces (WS_PIECE_U=2) + exp_k1k2.hip
# into tools/libexp_k1k2_u2.so
set -e
cd "$(dirname "$0")/.."
O=build/obj_u2; mkdir -p $O
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -fvisibility=hidden -mllvm -amdgpu-atomic-optimizer-strategy=None -DWS_PIECE_U=${U:-2} -DWS_PIECE_SHIFT=${S:-13} ${XDEF}"
for f in ws_api ws_hostpath ws_segfuse ws_piece ws_stream ws_reasm ws_encode ws_walker; do
  /opt/rocm/bin/hipcc $F -c util_amd/csrc/$f.hip -o $O/$f.o &
done
/opt/rocm/bin/hipcc $F -c tools/exp_k1k2.hip -o $O/exp_k1k2.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/obj/ws_host.o build/obj/ws_channel.o $O/*.o -o tools/libexp_k1k2_${NAME:-u${U:-2}}.so
