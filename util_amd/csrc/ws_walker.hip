// ws_walker.hip — variant "walker": one wavefront walks one rx segment and
// unmasks each frame as it goes (net_reactor.c:515-526 loop, fused).
//
// Kept as option path=1 and as the unmask kernel's fallback for batches with no pieces (the
// default is the piece path, ws_piece.hip: K1 walks, K2 unmasks 16 KiB pieces): every frame is a
// dependent round (header -> payload loads -> stores) inside one long-lived wave,
// and on CDNA vmcnt retires loads and stores in issue order, so each frame's loads
// also wait for the previous frame's stores. Measured ~5.2 TB/s on cfg2 vs ~6 TB/s
// for one-round waves.
#include "ws_walk.h"

#define WALK_WAVES 4
#define WALK_BLOCK (64 * WALK_WAVES)

// one wave per segment, grid-stride; 4 chunks per lane per batch, nontemporal loads and stores
// (a dynamic dequeue, 2 or 8 chunks per lane, plain loads/stores: measured no faster, round 1)
__global__ __launch_bounds__(WALK_BLOCK) void ws_walker_kernel(
    unsigned char* __restrict__ buf, const u64* __restrict__ seg_off, const u64* __restrict__ seg_len, u32 nseg,
    u32 max_frames, const u64* __restrict__ desc_base, WebsocketFrameDesc_t* __restrict__ desc,
    WebsocketSegResult_t* __restrict__ res, const u32* __restrict__ gate, u32 gate_gen) {
    // gated fallback (ws_piece.hip): run only if the piece path found the segments unordered
    if (gate && *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(gate)) != gate_gen) return;
    const u32 lane = threadIdx.x & 63;
    const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u32 nwaves = gridDim.x * WALK_WAVES;
    for (u32 s = blockIdx.x * WALK_WAVES + wave; s < nseg; s += nwaves)
        walk_segment<4, 1>(buf, s, seg_off, seg_len, max_frames, desc_base, desc, res, lane);
}

int ws_launch_walker(const WsLaunch& L, const u32* gate, u32 gate_gen) {
    u32 blocks = (L.nseg + WALK_WAVES - 1) / WALK_WAVES;
    const u32 cap = (u32)(L.cus > 0 ? L.cus : 256) * (gate ? 1u : 64u);   // a gated fallback: one block per CU
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(ws_walker_kernel, dim3(blocks), dim3(WALK_BLOCK), 0, L.stream, L.buf, L.seg_off, L.seg_len,
                       L.nseg, L.max_frames, L.desc_base, L.desc, L.res, gate, gate_gen);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_walker_kernel launch", e);
}
