// ws_walker.hip — variant "walker": one wavefront walks one rx segment and
// unmasks each frame as it goes (net_reactor.c:515-526 loop, fused).
//
// Kept as an A/B variant of the split design (ws_split.hip): every frame is a
// dependent round (header -> payload loads -> stores) inside one long-lived wave,
// and on CDNA vmcnt retires loads and stores in issue order, so each frame's loads
// also wait for the previous frame's stores. Measured ~5.2 TB/s on cfg2 vs ~6 TB/s
// for one-round waves.
#include "ws_walk.h"

#define WALK_WAVES 4
#define WALK_BLOCK (64 * WALK_WAVES)

__device__ __forceinline__ u32 dequeue_issue(u32* ctr, u32 lane) {
    u32 v = 0;
    if (lane == 0) v = atomicAdd(ctr, 1u);
    return v;
}

template <int U, int NT, bool DYN>
__global__ __launch_bounds__(WALK_BLOCK) void ws_walker_kernel(
    unsigned char* __restrict__ buf, const u64* __restrict__ seg_off, const u64* __restrict__ seg_len, u32 nseg,
    u32 max_frames, const u64* __restrict__ desc_base, WebsocketFrameDesc_t* __restrict__ desc,
    WebsocketSegResult_t* __restrict__ res, u32* __restrict__ ctr, const u32* __restrict__ gate, u32 gate_gen) {
    // gated fallback (ws_piece.hip): run only if the piece path found the segments unordered
    if (gate && *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(gate)) != gate_gen) return;
    const u32 lane = threadIdx.x & 63;
    const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u32 nwaves = gridDim.x * WALK_WAVES;
    u32 s = DYN ? __builtin_amdgcn_readfirstlane(dequeue_issue(ctr, lane)) : blockIdx.x * WALK_WAVES + wave;

    while (s < nseg) {
        const u32 s_next_v = DYN ? dequeue_issue(ctr, lane) : s + nwaves;
        walk_segment<U, NT>(buf, s, seg_off, seg_len, max_frames, desc_base, desc, res, lane);
        s = DYN ? __builtin_amdgcn_readfirstlane(s_next_v) : s_next_v;
    }
}

typedef void (*walker_t)(unsigned char*, const u64*, const u64*, u32, u32, const u64*, WebsocketFrameDesc_t*,
                         WebsocketSegResult_t*, u32*, const u32*, u32);

template <int U>
static walker_t pick(int nt, int dyn) {
    if (dyn) return nt == 1 ? ws_walker_kernel<U, 1, true> : (nt == 2 ? ws_walker_kernel<U, 2, true> : ws_walker_kernel<U, 0, true>);
    return nt == 1 ? ws_walker_kernel<U, 1, false> : (nt == 2 ? ws_walker_kernel<U, 2, false> : ws_walker_kernel<U, 0, false>);
}

int ws_launch_walker(const WsLaunch& L, int unroll, int nt, int dyn, int blocks_per_cu, u32* ctr, const u32* gate,
                     u32 gate_gen) {
    walker_t k = unroll == 8 ? pick<8>(nt, dyn) : (unroll == 2 ? pick<2>(nt, dyn) : pick<4>(nt, dyn));
    int per_cu = blocks_per_cu;
    if (per_cu <= 0) {
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(k), WALK_BLOCK, 0) !=
                hipSuccess || occ <= 0)
            occ = 4;
        per_cu = occ;
    }
    u32 blocks = (L.nseg + WALK_WAVES - 1) / WALK_WAVES;
    const u32 cap = (u32)L.cus * (u32)per_cu;
    if (blocks > cap) blocks = cap;
    hipError_t e;
    if (dyn && (e = hipMemsetAsync(ctr, 0, 16, L.stream)) != hipSuccess) return ws_set_err("hipMemsetAsync(counter)", e);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(WALK_BLOCK), 0, L.stream, L.buf, L.seg_off, L.seg_len, L.nseg,
                       L.max_frames, L.desc_base, L.desc, L.res, ctr, gate, gate_gen);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_walker_kernel launch", e);
}
