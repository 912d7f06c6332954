// ws_walk.h — one wavefront walks one rx segment (net_reactor.c:515-526) and unmasks
// each frame as it goes: the walker variant (ws_walker.hip) and the piece path's
// fallback for unordered batches (ws_piece.hip) share it.
#pragma once
#include "ws_common.h"

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

// One wavefront runs the reactor loop over segment s and unmasks as it goes.
template <int U, int NT>
__device__ __forceinline__ void walk_segment(unsigned char* __restrict__ buf, u32 s, const u64* __restrict__ seg_off,
                                             const u64* __restrict__ seg_len, u32 max_frames,
                                             const u64* __restrict__ desc_base, WebsocketFrameDesc_t* __restrict__ desc,
                                             WebsocketSegResult_t* __restrict__ res, u32 lane) {
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
}
