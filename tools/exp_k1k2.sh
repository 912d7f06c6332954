# build tools/libexp_k1k2.so (experiment only): the product's objects + tools/exp_k1k2.hip
set -e
cd "$(dirname "$0")/.."
make -C util_amd/csrc -s
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -fvisibility=hidden -mllvm -amdgpu-atomic-optimizer-strategy=None"
/opt/rocm/bin/hipcc $F -c tools/exp_k1k2.hip -o build/obj/exp_k1k2.o
/opt/rocm/bin/hipcc $F -DWS_K1_VARIANTS -c util_amd/csrc/ws_piece.hip -o build/obj/ws_piece_var.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/obj/ws_host.o build/obj/ws_channel.o build/obj/ws_api.o \
  build/obj/ws_hostpath.o build/obj/ws_segfuse.o build/obj/ws_piece_var.o build/obj/ws_stream.o \
  build/obj/ws_reasm.o build/obj/ws_encode.o build/obj/ws_walker.o build/obj/exp_k1k2.o -o tools/libexp_k1k2.so
