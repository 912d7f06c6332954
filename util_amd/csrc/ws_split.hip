// ws_split.hip — default decode path: walk, then one-round unmask.
//
// K1 ws_walk_kernel: ONE LANE per rx segment runs the reactor loop
//   (net_reactor.c:515-526) over websocketframeDecode's header logic
//   (websocketframe.c:112-165, ws_parse), writing every descriptor, the segment
//   result, each masked frame's key and the number of payload "work items".
//   Only header bytes are touched; all segments walk concurrently, so the serial
//   header chain costs ~frames-per-segment dependent loads for the whole batch.
// K2 ws_unmask_kernel: ONE BLOCK per segment. It loads the whole segment region
//   (16-B-aligned chunks, unconditional loads so they issue back to back), loads
//   the segment's frame table into LDS meanwhile, builds each chunk's 32-bit
//   rotated key (binary search of the frame table), XORs and stores payload bytes
//   only (each chunk by its one owning lane): full chunks with one 16-B store, chunks that straddle a frame edge with
//   byte stores of exactly the payload bytes (headers, gaps and other segments
//   are never written). A segment that fits one round (T*U chunks, 72 KiB at
//   512x9) is one load round + one store round per wave and the block exits: on
//   CDNA vmcnt retires loads and stores in issue order, so never making a wave
//   load after its own stores is what keeps HBM busy.
#include "ws_common.h"

#define WALK_T 256

__global__ __launch_bounds__(WALK_T) void ws_walk_kernel(const unsigned char* __restrict__ buf,
                                                         const u64* __restrict__ seg_off,
                                                         const u64* __restrict__ seg_len, u32 nseg, u32 max_frames,
                                                         const u64* __restrict__ desc_base,
                                                         WebsocketFrameDesc_t* __restrict__ desc,
                                                         WebsocketSegResult_t* __restrict__ res,
                                                         u32* __restrict__ keys, u32* __restrict__ nwork) {
    const u32 s = blockIdx.x * WALK_T + threadIdx.x;
    if (s >= nseg) return;
    const u64 so = seg_off[s], sl = seg_len[s];
    const u64 dbase = desc_base ? desc_base[s] : (u64)s * max_frames;
    const u64 kbase = (u64)s * max_frames;
    u64 off = 0;
    u32 nf = 0, extra = 0;
    int status = WEBSOCKET_SEG_OK;
    // 32 bytes from floor16(p) cover header bytes [p, p+14) (WEBSOCKET_BATCH_PAD). The next
    // header's loads are issued before this frame's descriptor stores, so waiting for them
    // never waits for the stores (vmcnt is in issue order).
    uintptr_t p = reinterpret_cast<uintptr_t>(buf + so);
    u32x4 x0 = reinterpret_cast<const gu32x4*>(p & ~(uintptr_t)15)[0];
    u32x4 x1 = reinterpret_cast<const gu32x4*>(p & ~(uintptr_t)15)[1];
    while (off < sl) {
        if (nf >= max_frames) { status = WEBSOCKET_SEG_MAX_FRAMES; break; }
        const u64 avail = sl - off;
        if (avail < 2) break;                                                // websocketframe.c:121
        u64 h0, h1;
        ws_hdr_from32(x0, x1, (u32)(p & 15), h0, h1);
        const WsHdr h = ws_parse(h0, h1, avail);
        if (h.kind == WS_PARSE_INCOMPLETE) break;
        if (h.kind == WS_PARSE_WRAP) { status = WEBSOCKET_SEG_ERR_LEN_WRAP; break; }
        // prefetch the next header (harmless re-load of this one if the loop will stop)
        const uintptr_t pn = h.ret > 0 && off + (u32)h.ret < sl ? p + (u32)h.ret : p;
        const gu32x4* qn = reinterpret_cast<const gu32x4*>(pn & ~(uintptr_t)15);
        x0 = qn[0];
        x1 = qn[1];
        // slot nf: a real descriptor, or (ret == 0) scratch holding the work item only
        ws_store_desc(desc + dbase + nf, so + off, h);
        if (h.masked) *gptr<u32>(keys + kbase + nf) = h.key;
        if (h.ret == 0) { extra = 1; break; }                                // (int) truncated to 0: unmasked,
        ++nf;                                                                // no descriptor, loop breaks
        if (h.ret < 0) { status = WEBSOCKET_SEG_ERR_DECODE; break; }         // net_reactor.c:518-520
        off += (u32)h.ret;                                                   // net_reactor.c:525
        p = pn;
    }
    ws_store_res(res + s, off, nf, status);
    *gptr<u32>(nwork + s) = nf + extra;
}

template <int T, int U, int NT>
__global__ __launch_bounds__(T) void ws_unmask_kernel(unsigned char* __restrict__ buf, const u64* __restrict__ seg_off,
                                                      const u64* __restrict__ seg_len, u32 max_frames,
                                                      const u64* __restrict__ desc_base,
                                                      const WebsocketFrameDesc_t* __restrict__ desc,
                                                      const u32* __restrict__ keys, const u32* __restrict__ nwork) {
    constexpr u32 FW = T - 1;              // items per window (+1 thread reads the next item's start)
    constexpr int RB = T * U * 16;         // bytes per round
    __shared__ Item tab[T];
    __shared__ u64 s_cap;
    const u32 s = blockIdx.x;
    const u32 tid = threadIdx.x;
    const u32 nw = nwork[s];
    if (nw == 0) return;
    const u64 so = seg_off[s], sl = seg_len[s];
    const u64 dbase = desc_base ? desc_base[s] : (u64)s * max_frames;
    const u64 kbase = (u64)s * max_frames;
    const uintptr_t seg_abs = reinterpret_cast<uintptr_t>(buf + so);
    const uintptr_t origin = seg_abs & ~(uintptr_t)15;
    const u64 org_off = so - (u64)(seg_abs - origin);                       // buffer offset of the origin
    const u64 nchunks = (u64)(((seg_abs + sl + 15) & ~(uintptr_t)15) - origin) >> 4;
    gu32x4* const base = reinterpret_cast<gu32x4*>(origin);

    u32 f0 = 0, cnt = 0;
    u64 ip0 = 0, ip1 = 0;   // this thread's window item, relative to the origin
    u32 irk = 0;
    bool have = false, loaded = false;
    for (u64 c0 = 0; c0 < nchunks;) {
        const u32 left = nw - f0;
        const bool all = left <= FW;
        const bool reload = !loaded || !all;
        // ---- 1. raw window item loads (descriptor + key together), decoded later
        u32x4 q0 = {0, 0, 0, 0}, q1 = {0, 0, 0, 0};
        u32 kraw = 0;
        if (reload) {
            cnt = all ? left : FW;
            have = tid <= cnt && f0 + tid < nw;
            if (have) {
                const gu32x4* d = gptr<u32x4>(desc + dbase + f0 + tid);
                q0 = d[0];
                q1 = d[1];
                kraw = *gptr<u32>(keys + kbase + f0 + tid);
            }
        }
        u64 c1 = c0 + (u64)(T * U) < nchunks ? c0 + (u64)(T * U) : nchunks;
        auto decode = [&]() {
            const u64 fo = (u64)q0.x | ((u64)q0.y << 32), dof = (u64)q0.z | ((u64)q0.w << 32);
            const u64 dl = (u64)q1.x | ((u64)q1.y << 32);
            if (have && ((q1.w >> 16) & 1u) && dl) {
                ip0 = dof - org_off;
                ip1 = ip0 + dl;
                irk = rotl32(kraw, 8u * (u32)(ip0 & 3));
            } else {
                ip0 = ip1 = have ? fo - org_off : ~0ULL;
                irk = 0;
            }
        };
        if (reload && !all) {  // windowed: the round must end before the next window's first item
            decode();
            if (tid == cnt) s_cap = ip0;
            __syncthreads();
            const u64 capc = s_cap >> 4;
            if (capc < c1) c1 = capc;
        }
        // ---- 2. payload loads: unconditional, clamped to the round's last chunk
        const u32 lim = (u32)(c1 - 1 - c0);
        gu32x4* const rb = base + c0;
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld16<NT>(rb + min(tid + (u32)(u * T), lim));
        if (reload && all) decode();   // window decoded while the payload loads are in flight
        loaded = true;
        // ---- 3. this round's table (32-bit offsets relative to the round start)
        if (tid < cnt) {
            const long long r0 = (long long)(c0 << 4);
            long long a = (long long)ip0 - r0, b = (long long)ip1 - r0;
            a = a < -16 ? -16 : (a > RB + 16 ? RB + 16 : a);
            b = b < -16 ? -16 : (b > RB + 16 ? RB + 16 : b);
            Item it;
            it.p0 = (int)a; it.p1 = (int)b; it.rkey = irk; it.pad = 0;
            tab[tid] = it;
        }
        __syncthreads();
        // ---- 4. per chunk: XOR with its item's key, store payload bytes only
        ws_xor_round<T, U, NT>(v, rb, lim, tab, cnt, tid);
        c0 = c1;
        if (c0 < nchunks) {
            // window: drop the items that end at or before the new round start
            if (!all) f0 += (u32)__syncthreads_count(tid < cnt && ip1 <= (c0 << 4));
            __syncthreads();  // every thread done reading `tab` before it is rewritten
        }
    }
}

template <int T, int U>
static int launch_unmask(const WsLaunch& L, int nt, const u32* keys, const u32* nwork) {
    if (nt == 1)
        hipLaunchKernelGGL((ws_unmask_kernel<T, U, 1>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, keys, nwork);
    else if (nt == 2)
        hipLaunchKernelGGL((ws_unmask_kernel<T, U, 2>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, keys, nwork);
    else
        hipLaunchKernelGGL((ws_unmask_kernel<T, U, 0>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, keys, nwork);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_unmask_kernel launch", e);
}

// variant: 0 -> 512 threads x 9 chunks (72 KiB rounds), 1 -> 1024 x 5, 2 -> 256 x 17, 3 -> 512 x 4
int ws_launch_split(const WsLaunch& L, int variant, int nt, u32* keys, u32* nwork) {
    hipLaunchKernelGGL(ws_walk_kernel, dim3((L.nseg + WALK_T - 1) / WALK_T), dim3(WALK_T), 0, L.stream, L.buf,
                       L.seg_off, L.seg_len, L.nseg, L.max_frames, L.desc_base, L.desc, L.res, keys, nwork);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ws_set_err("ws_walk_kernel launch", e);
    switch (variant) {
    case 1: return launch_unmask<1024, 5>(L, nt, keys, nwork);
    case 2: return launch_unmask<256, 17>(L, nt, keys, nwork);
    case 3: return launch_unmask<512, 4>(L, nt, keys, nwork);
    default: return launch_unmask<512, 9>(L, nt, keys, nwork);
    }
}
