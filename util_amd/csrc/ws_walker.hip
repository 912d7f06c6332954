// ws_walker.hip — variant "walker": one wavefront walks one rx segment and
// unmasks each frame as it goes (net_reactor.c:515-526 loop, fused).
//
// Kept as an A/B variant of the split design (ws_split.hip): every frame is a
// dependent round (header -> payload loads -> stores) inside one long-lived wave,
// and on CDNA vmcnt retires loads and stores in issue order, so each frame's loads
// also wait for the previous frame's stores. Measured ~5.2 TB/s on cfg2 vs ~6 TB/s
// for one-round waves.
#include "ws_common.h"

#define WALK_WAVES 4
#define WALK_BLOCK (64 * WALK_WAVES)

struct HdrWords { u32 w0, w1, w2, w3, w4; };

// The 5 aligned dwords covering header bytes [p, p+14), by scalar loads (lgkmcnt,
// so waiting for them never waits on this wave's payload stores). Unconditional:
// WEBSOCKET_BATCH_PAD guarantees readable bytes after every segment.
__device__ __forceinline__ HdrWords load_header(const unsigned char* p) {
    const cu32* sq = reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    HdrWords h;
    h.w0 = sq[0]; h.w1 = sq[1]; h.w2 = sq[2]; h.w3 = sq[3]; h.w4 = sq[4];
    return h;
}

// Unmask payload bytes [P0, P1) with LE key K in place, by one wave. The <=15
// unaligned bytes at each end go through lanes 0-31 one byte each (loaded first,
// stored last); the 16-B-aligned interior in branch-free batches of 64*U chunks
// (lanes past the end re-load/re-store the last chunk with the identical value).
template <int U, int NT>
__device__ __forceinline__ void unmask_payload(unsigned char* P0, unsigned char* P1, u32 K, u32 lane) {
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(P0), a1 = reinterpret_cast<uintptr_t>(P1);
    const uintptr_t A = (a0 + 15) & ~(uintptr_t)15, B = a1 & ~(uintptr_t)15;
    const uintptr_t head_end = A < a1 ? A : a1;
    const uintptr_t tail_beg = A > B ? A : B;
    uintptr_t x = 0;
    bool act = false;
    if (lane < 16) { x = a0 + lane; act = x < head_end; }
    else if (lane < 32) { x = tail_beg + (lane - 16); act = x < a1; }
    gu8* const px = reinterpret_cast<gu8*>(x);
    const u32 eb = *reinterpret_cast<const gu8*>(act ? x : a0);
    if (A < B) {
        const u32 R = rotl32(K, 8u * (u32)(a0 & 3));
        gu32x4* pb = reinterpret_cast<gu32x4*>(A);
        const u64 n = (u64)(B - A) >> 4;
        for (u64 base = 0; base < n; base += 64 * U, pb += 64 * U) {
            const u64 left = n - base;
            const u32 lim = left < (u64)(64 * U) ? (u32)left - 1u : (u32)(64 * U - 1);
            u32 c[U];
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                c[u] = min((u32)(u * 64) + lane, lim);
                v[u] = ld16<NT>(pb + c[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) st16<NT>(v[u] ^ R, pb + c[u]);
        }
    }
    if (act) *px = (unsigned char)(eb ^ (K >> (8u * (u32)((x - a0) & 3))));
}

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
        const u64 so = seg_off[s], sl = seg_len[s];
        const u64 dbase = desc_base ? desc_base[s] : (u64)s * max_frames;
        unsigned char* const seg = buf + so;
        u64 off = 0;
        u32 nf = 0;
        int status = WEBSOCKET_SEG_OK;
        HdrWords hw = load_header(seg);
        while (off < sl) {
            if (nf >= max_frames) { status = WEBSOCKET_SEG_MAX_FRAMES; break; }
            const u64 avail = sl - off;
            if (avail < 2) break;                                           // websocketframe.c:121
            unsigned char* const p = seg + off;
            const u64 lo = (u64)hw.w0 | ((u64)hw.w1 << 32);
            const u64 mi = (u64)hw.w2 | ((u64)hw.w3 << 32);
            const u64 hi = (u64)hw.w4;
            const u32 sh = 8u * (u32)(reinterpret_cast<uintptr_t>(p) & 3);
            const WsHdr h = ws_parse(sh ? (lo >> sh) | (mi << (64 - sh)) : lo,
                                     sh ? (mi >> sh) | (hi << (64 - sh)) : mi, avail);
            if (h.kind == WS_PARSE_INCOMPLETE) break;
            if (h.kind == WS_PARSE_WRAP) { status = WEBSOCKET_SEG_ERR_LEN_WRAP; break; }
            const HdrWords hwn = load_header(h.ret > 0 && off + (u32)h.ret < sl ? p + (u32)h.ret : p);
            if (h.masked) unmask_payload<U, NT>(p + h.hdr, p + h.hdr + h.plen, h.key, lane);
            if (h.ret == 0) break;                                          // (int) truncated to 0
            if (lane == 0) ws_store_desc(desc + dbase + nf, so + off, h);
            ++nf;
            if (h.ret < 0) { status = WEBSOCKET_SEG_ERR_DECODE; break; }    // net_reactor.c:518-520
            off += (u32)h.ret;                                              // net_reactor.c:525
            hw = hwn;
        }
        if (lane == 0) ws_store_res(res + s, off, nf, status);
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
