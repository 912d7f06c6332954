// ws_reasm.hip — fused decode + fragmented-message reassembly (SURVEY §8a row a6,
// §8f rank 1). The reactor-side behaviour: every decoded frame's
// unmasked body joins the connection's pending message; a frame with FIN set closes
// it, and the message body handed to the application is the concatenation of its
// frames' bodies (a FIN frame with nothing pending is a message by itself). The
// reference pays an unmask in place, a copy into a cached packet and a merge copy
// (≈3x the bytes); here every body byte is read once from the wire and written once,
// unmasked, into a contiguous per-connection output region.
//
// R1 ws_piece_scan_kernel (ws_piece.hip): the reactor-loop walk — descriptors,
//    segment results, per-frame payload items.
// R2 ws_reasm_layout_kernel: one thread per segment turns its descriptors into body
//    placements (output offset = running sum of the bodies before it) and message
//    descriptors, and carries the open/closed state across batches.
// R3 ws_reasm_gather_kernel: one wavefront per frame body: 16-B-aligned output chunks
//    from one unaligned 16-B wire load each, XOR with the key rotated to the output
//    phase; the <=15 bytes at each body edge by byte ops (bodies are adjacent, so two
//    waves may share an output chunk but never a byte).
// The wire buffer is only read.
//
// Fragment-cache limit (websocketframeBatchReassembleDeviceEx): the stream hook refuses to
// cache a body that would take the connection's cached bytes past readcache_max_size
// (check_cache_overflow, net_channel_ex.c:45-53, applied at :129-135 to every frame that is
// cached: one arriving while a message is pending, or a non-FIN one); the channel is then
// detached with NET_REACTOR_CACHE_READ_OVERFLOW_ERR and the frame is not consumed. Both paths
// stop the segment there with WEBSOCKET_SEG_ERR_CACHE_OVERFLOW (descriptor written, not
// consumed, no body). Cached bytes are counted in u32 as the reference's
// StreamTransportCtx_t.cache_recv_bytes (transport_ctx.c:179-201) and carried across batches.
#include "ws_common.h"

// check_cache_overflow (net_channel_ex.c:45-53) on u32 counts
__device__ __forceinline__ bool ws_cache_overflow(u32 already, u32 add, u32 max_limit) {
    if (max_limit == 0) return false;
    if (max_limit < add) return true;
    return already > max_limit - add;
}

#define RLAY_T 256
#define RGAT_T 256
#define RGAT_U 4

struct GatherRec {       // 32 B per body, slot s*max_frames + body index
    u64 src;             // first payload byte, origin-relative in the wire buffer
    u64 dst;             // first body byte, origin-relative in the output buffer
    u64 len;
    u32 key;             // XOR key rotated to the output byte phase: byte (y & 3) for output byte y
    u32 pad;
};

// R2 with LG lanes per segment: lane j takes frame k0 + j of each round of LG frames;
// body offsets are a group prefix sum, message boundaries come from the group's FIN mask.
#define RLAY_G 16
__global__ __launch_bounds__(RLAY_T) void ws_reasm_layout_kernel(
    const unsigned char* __restrict__ buf, u32 nseg, u32 max_frames, const u64* __restrict__ seg_off,
    const u64* __restrict__ seg_len, const WebsocketFrameDesc_t* __restrict__ desc, WebsocketSegResult_t* __restrict__ res,
    const u32x4* __restrict__ items, const unsigned char* __restrict__ out, const u64* __restrict__ out_off,
    WebsocketMsgDesc_t* __restrict__ msg, u32* __restrict__ nmsg, unsigned char* __restrict__ open_io,
    GatherRec* __restrict__ recs, u32* __restrict__ nbody, u32 cache_max, u32* __restrict__ cached_io) {
    constexpr u32 G = RLAY_G;
    const u32 lane = threadIdx.x & 63, gl = lane % G, gb = lane - gl;
    const u32 s = (blockIdx.x * RLAY_T + threadIdx.x) / G;
    const bool active = s < nseg;
    const u32 sc = active ? s : nseg - 1;
    const u64 lead_o = reinterpret_cast<uintptr_t>(out) & 15;
    const u64 so = seg_off[sc], sl = seg_len[sc];
    const u64 ob = out_off ? out_off[sc] : so;                              // output region start (d_out-relative)
    const u64 base = (u64)sc * max_frames;
    const u32 nf = active ? res[sc].n_frames : 0u;
    const int status0 = res[sc].status;
    u32 open = active && open_io ? open_io[sc] : 0u, cont = open;
    u32 cached = open && cached_io ? cached_io[sc] : 0u;                     // bytes of the pending message
    u32 nm = 0, nb = 0, first = 0;                                           // group-uniform state
    u64 q = 0, q0 = 0;
    bool stop = false, overflow = false;
    int cstop_frame = -1;                                                    // frame refused by the cache limit
    const u64 gmask = (1ull << G) - 1;
    (void)buf;
    for (u32 k0 = 0; __ballot(active && !stop && k0 < nf); k0 += G) {
        const u32 k = k0 + gl;
        const bool in = active && !stop && k < nf;
        WebsocketFrameDesc_t d = {};
        u32x4 it = {0, 0, 0, 0};
        if (in) { d = desc[base + k]; it = items[base + k]; }
        // frames with a body: consecutive from k0 up to the first ret <= 0 (the error frame)
        const u64 badm = (__ballot(in && d.ret <= 0) >> gb) & gmask;
        const u64 inm = (__ballot(in) >> gb) & gmask;
        const u32 nbody_r = badm ? (u32)__builtin_ctzll(badm) : (u32)__builtin_popcountll(inm);
        const bool body = gl < nbody_r;
        const u64 len = body ? d.datalen : 0;
        // inclusive prefix sum of the body lengths within the group
        u64 incl = len;
#pragma unroll
        for (u32 o = 1; o < G; o <<= 1) {
            const u64 t = __shfl_up(incl, o, G);
            if (gl >= o) incl += t;
        }
        const u64 qs = q + incl - len;                                       // this body's output offset
        // bodies must fit the segment's region (only the (int) return quirk can break this)
        const u64 ovm = (__ballot(body && len > sl - qs) >> gb) & gmask;   // qs <= sl before the first overflow
        u32 ntake = ovm ? (u32)__builtin_ctzll(ovm) : nbody_r;
        // the fragment cache's limit: pending before frame k = frame k-1 was not FIN (lane 0: the
        // carried state); cached bytes before k = the current message's bodies before k (u32)
        const u32 blen = (u32)len;
        u32 cincl = blen;
#pragma unroll
        for (u32 o = 1; o < G; o <<= 1) {
            const u32 t = (u32)__shfl_up((int)cincl, o, G);
            if (gl >= o) cincl += t;
        }
        const bool finb = body && d.is_fin;
        const u64 fin_all = (__ballot(finb) >> gb) & gmask;
        const u64 fin_below = fin_all & ((1ull << gl) - 1);
        const u32 lastf = fin_below ? 63 - __builtin_clzll(fin_below) : 0;
        const u32 cincl_lastf = (u32)__shfl((int)cincl, (int)(gb + lastf), 64);
        const u32 cbefore = fin_below ? cincl - blen - cincl_lastf : cached + cincl - blen;
        const bool pend = gl == 0 ? open != 0 : !((fin_all >> (gl - 1)) & 1ull);
        const u64 ccm = (__ballot(body && (pend || !d.is_fin) && ws_cache_overflow(cbefore, blen, cache_max)) >> gb) & gmask;
        const u32 cst = ccm ? (u32)__builtin_ctzll(ccm) : 64u;
        if (cst < ntake) {
            ntake = cst;
            cstop_frame = (int)(k0 + cst);
        }
        if (gl < ntake) {
            const u64 p0 = ((u64)it.x | ((u64)it.y << 32)) & 0xFFFFFFFFFFFFull;
            const u32 rk = (u32)(((u64)it.x | ((u64)it.y << 32)) >> 48) | ((u32)(((u64)it.z | ((u64)it.w << 32)) >> 48) << 16);
            const u32 sh = 8u * (u32)(p0 & 3);
            const u32 key = sh ? (rk >> sh) | (rk << (32 - sh)) : rk;       // the frame's key (wire order)
            const u64 dst = ob + qs + lead_o;
            GatherRec r;
            r.src = p0; r.dst = dst; r.len = len; r.key = d.masked ? rotl32(key, 8u * (u32)(dst & 3)) : 0u; r.pad = 0;
            recs[base + nb + gl] = r;
        }
        // messages closed by FIN frames among the taken ones
        const u64 finm = (__ballot(gl < ntake && d.is_fin) >> gb) & gmask;
        const u64 below = finm & ((1ull << gl) - 1);                         // earlier FINs in this round
        const u32 prevl = below ? 63 - __builtin_clzll(below) : gl;
        const u64 incl_prev = __shfl(incl, (int)(gb + prevl), 64);          // all lanes active here
        if (gl < ntake && d.is_fin) {
            const u32 mfirst = below ? k0 + prevl + 1 : first;
            const u64 prevq = below ? q + incl_prev : q0;
            WebsocketMsgDesc_t m;
            m.out_off = ob + prevq; m.len = qs + len - prevq; m.first_frame = mfirst; m.n_frames = k + 1 - mfirst;
            m.complete = 1; m.continued = below ? 0u : cont;
            msg[base + nm + (u32)__builtin_popcountll(below)] = m;
        }
        const u64 tot_l = __shfl(incl, (int)(gb + (ntake ? ntake - 1 : 0)), 64);
        const u32 last = finm ? 63 - __builtin_clzll(finm) : 0;             // last FIN of the round
        const u64 incl_last = __shfl(incl, (int)(gb + last), 64);
        const u64 tot = ntake ? tot_l : 0;
        const u32 ctot = (u32)__shfl((int)cincl, (int)(gb + (ntake ? ntake - 1 : 0)), 64);
        const u32 clast = (u32)__shfl((int)cincl, (int)(gb + last), 64);
        if (ntake) cached = finm ? (ntake > last + 1 ? ctot - clast : 0u) : cached + ctot;
        if (finm) {
            q0 = q + incl_last;
            first = k0 + last + 1;
            cont = 0;
            open = ntake > last + 1 ? 1u : 0u;
            nm += (u32)__builtin_popcountll(finm);
        } else if (ntake) {
            open = 1;
        }
        q += tot;
        nb += ntake;
        if (ntake < G || k0 + G >= nf) stop = true;                          // error frame, overflow or end
        if (ovm && cstop_frame < 0) overflow = true;
        if (!active) stop = true;
    }
    if (!active || gl != 0) return;
    if (open && nb > first) {                                                // still open at the segment end
        WebsocketMsgDesc_t m;
        m.out_off = ob + q0; m.len = q - q0; m.first_frame = first; m.n_frames = nb - first;
        m.complete = 0; m.continued = cont;
        msg[base + nm++] = m;
    }
    if (cstop_frame >= 0) {                                                  // not consumed; the channel detaches
        const WebsocketFrameDesc_t dc = desc[base + (u32)cstop_frame];
        ws_store_res(res + s, dc.frame_off - so, (u32)cstop_frame + 1, WEBSOCKET_SEG_ERR_CACHE_OVERFLOW);
    } else if (overflow) {
        res[s].status = WEBSOCKET_SEG_ERR_OUT_SPACE;
    }
    (void)status0;
    nmsg[s] = nm;
    nbody[s] = nb;
    if (open_io) open_io[s] = (unsigned char)open;
    if (cached_io) cached_io[s] = open ? cached : 0u;
}

typedef u32x4 __attribute__((aligned(1))) u32x4u;

__device__ __forceinline__ u64 rl64(u64 v, u32 i) {          // 64-bit readlane
    return (u64)(u32)__builtin_amdgcn_readlane((int)(u32)v, (int)i) |
           ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), (int)i) << 32);
}

template <int NT>
__global__ __launch_bounds__(RGAT_T) void ws_reasm_gather_kernel(const unsigned char* __restrict__ buf,
                                                                 unsigned char* __restrict__ out, u32 max_frames,
                                                                 u64 nslots, const GatherRec* __restrict__ recs,
                                                                 const u32* __restrict__ nbody) {
    const u32 lane = threadIdx.x & 63;
    const u64 nw = (u64)gridDim.x * (RGAT_T / 64);
    const uintptr_t borg = reinterpret_cast<uintptr_t>(buf) & ~(uintptr_t)15;
    const uintptr_t oorg = reinterpret_cast<uintptr_t>(out) & ~(uintptr_t)15;
    for (u64 slot = (u64)blockIdx.x * (RGAT_T / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); slot < nslots;
         slot += nw) {
        const u32 s = (u32)(slot / max_frames), k = (u32)(slot - (u64)s * max_frames);
        if (k >= *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(nbody + s))) continue;
        const __attribute__((address_space(4))) u32* rq =
            reinterpret_cast<const __attribute__((address_space(4))) u32*>(reinterpret_cast<uintptr_t>(recs + slot));
        const u64 src = (u64)rq[0] | ((u64)rq[1] << 32), dst = (u64)rq[2] | ((u64)rq[3] << 32);
        const u64 len = (u64)rq[4] | ((u64)rq[5] << 32);
        const u32 key = rq[6];
        if (!len) continue;
        const u64 d1 = dst + len;
        const u64 A = (dst + 15) & ~15ull, B = d1 & ~15ull;
        // edge bytes: lanes 0-15 the head [dst, min(A, d1)), lanes 16-31 the tail [max(A, B), d1)
        u64 y = 0;
        bool act = false;
        if (lane < 16) { y = dst + lane; act = y < (A < d1 ? A : d1); }
        else if (lane < 32) { y = (A > B ? A : B) + (lane - 16); act = y < d1; }
        const u32 eb = *reinterpret_cast<const gu8*>(borg + src + (act ? y - dst : 0));
        // interior: 16-B output chunks [A, B)
        if (A < B) {
            const u64 nch = (B - A) >> 4;
            for (u64 c0 = 0; c0 < nch; c0 += 64 * RGAT_U) {
                u32x4 v[RGAT_U];
#pragma unroll
                for (int u = 0; u < RGAT_U; ++u) {
                    if (u && c0 + (u64)u * 64 >= nch) break;                 // wave-uniform: no empty rows
                    const u64 c = c0 + (u64)(u * 64 + lane);
                    const u64 cc = c < nch ? c : nch - 1;
                    v[u] = *reinterpret_cast<const WS_GLOBAL u32x4u*>(borg + src + (A + (cc << 4) - dst));
                }
#pragma unroll
                for (int u = 0; u < RGAT_U; ++u) {
                    const u64 c = c0 + (u64)(u * 64 + lane);
                    if (c < nch) st16<NT>(v[u] ^ key, reinterpret_cast<gu32x4*>(oorg + A + (c << 4)));
                }
            }
        }
        if (act) *reinterpret_cast<gu8*>(oorg + y) = (unsigned char)(eb ^ (key >> (8u * (u32)(y & 3))));
    }
}

// ---------------------------------------------------------------------------------------------
// Fused path: ONE workgroup per rx segment, the whole decode + reassembly of the segment
// in one kernel. The segment's wire bytes stream through LDS in windows (one window for
// segments up to 17 KiB: cfg5's 16.5 KiB messages are one-shot blocks — load once,
// store once, exit, the pattern that reaches the part's streaming ceiling):
//   1. LDS-DMA (global_load_lds_dwordx4): every wave issues its 1 KiB slices of the
//      window at once, clamped to the segment's readable bytes (segment +
//      WEBSOCKET_BATCH_PAD), no registers involved;
//   2. wave 0 walks the reactor loop (net_reactor.c:515-526) over the headers in LDS by
//      stride speculation (64 candidate frames per round, the stride seeded by the
//      first header, as ws_piece_scan_kernel), writes the descriptors, places each body
//      at the running sum of the bodies before it and emits the message descriptors
//      (the delivery rule of SURVEY §8a a6);
//   3. wave w copies bodies w, w+4, ... of the window: every 16-B-aligned output chunk
//      inside a body is one unaligned 16-B LDS read (two aligned reads + funnel shift),
//      XOR with the key rotated to the output phase, one 16-B store; the <= 15 bytes at
//      each body/window edge go one per lane (lanes 0-15 head, 16-31 tail).
// Frames longer than a window (or a header past it) continue in the next window; the
// walk state and the body table (max_frames <= RSEG_TB bodies) persist across windows.
// Each wire byte is read from HBM once (+ 1 KiB of look-ahead per extra window), each
// body byte written once.
#define RSEG_T 256
// window = L LDS-DMA wave instructions of 1 KiB: (L-1) KiB owned + 1 KiB look-ahead;
// L = 18 is ~20 KB of LDS: 8 workgroups (32 waves) per CU ("reasm_cfg" A/B: ws_reasm_cfg)
#define RSEG_TB 64                                 // body table entries = max max_frames of this path

typedef __attribute__((address_space(3))) void lds_void;

struct BodyL {           // body table entry (LDS; its key, rotated to the absolute output phase
    u64 x0;              // (0 for unmasked frames), in a separate array to keep LDS at 20 KB)
    u64 dst;             // first payload byte in window coordinates (segment offset + lead),
    u64 len;             // first body byte region-relative, body length
};

// Interior copy of one body from the LDS window: output chunks c = lane, lane + 64, ... < nch
// at dst + 16c take the 16 source bytes at window byte o0 + 16c, XOR key. The source phase
// o0 & 15 is the same for every chunk of the body (wave-uniform), so the 16 bytes are four
// v_alignbyte_b32 of dwords picked at compile time (SD = (o0 >> 2) & 3, one loop per SD),
// not a per-lane 64-bit funnel shift.
// Stores: sc1|nt through a descriptor over the body (cfg5 1.403-1.406 -> 1.392-1.399 ms against
// nt global stores, profiles/r04_store_sc1nt_ab.log).
template <int SD>
__device__ __forceinline__ void reasm_copy(const u32x4* win, u32 o0, u32 nch, u32 key, u64 dst, u32 lane) {
    const u32 sb = o0 & 3u;
    const __amdgpu_buffer_rsrc_t wrs = ws_rsrc((uintptr_t)dst, nch * 16u);
    for (u32 c = lane; c < nch; c += 64) {
        const u32 i = (o0 >> 4) + c;
        const u32x4 a = win[i], b = win[i + 1];
        const u32 d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        u32x4 w;
        w.x = __builtin_amdgcn_alignbyte(d[SD + 1], d[SD + 0], sb) ^ key;
        w.y = __builtin_amdgcn_alignbyte(d[SD + 2], d[SD + 1], sb) ^ key;
        w.z = __builtin_amdgcn_alignbyte(d[SD + 3], d[SD + 2], sb) ^ key;
        w.w = __builtin_amdgcn_alignbyte(d[SD + 4], d[SD + 3], sb) ^ key;
        st16_sc1nt(w, wrs, c << 4);
    }
}

template <int RSEG_L, int MINW>
__global__ __launch_bounds__(RSEG_T) __attribute__((amdgpu_waves_per_eu(MINW, 8))) void ws_reasm_seg_kernel(
    const unsigned char* __restrict__ buf, u32 max_frames, const u64* __restrict__ seg_off,
    const u64* __restrict__ seg_len, WebsocketFrameDesc_t* __restrict__ desc, WebsocketSegResult_t* __restrict__ res,
    unsigned char* __restrict__ out, const u64* __restrict__ out_off, WebsocketMsgDesc_t* __restrict__ msg,
    u32* __restrict__ nmsg, unsigned char* __restrict__ open_io, u32 merge, u32 nseg, u32 wsh, u32 ppw, u32 cache_max,
    u32* __restrict__ cached_io) {
    constexpr u32 RSEG_C = (RSEG_L - 1) * 64;         // chunks owned per window
    __shared__ __attribute__((aligned(16))) u32x4 win[RSEG_L * 64];
    __shared__ BodyL tab[RSEG_TB];
    __shared__ u32 tkey[RSEG_TB];
    __shared__ u64 sh_next;                        // next window's first chunk, ~0 = done
    __shared__ u32 sh_blo, sh_bhi;                 // bodies with bytes in this window [blo, bhi], blo > bhi: none
    const u32 s = ws_winn(blockIdx.x, wsh, ppw), tid = threadIdx.x, lane = tid & 63;
    if (s >= nseg) return;                         // the last window's spare blocks
    const u32 wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool w0 = wv == 0;
    const u64 so = seg_off[s], sl = seg_len[s];
    const uintptr_t segp = reinterpret_cast<uintptr_t>(buf + so);
    const u64 lead = segp & 15;
    const gu32x4* const gseg = reinterpret_cast<const gu32x4*>(segp & ~(uintptr_t)15);
    const u64 cmax = (sl + lead + WEBSOCKET_BATCH_PAD - 1) >> 4;     // last readable chunk
    const u64 ob = out_off ? out_off[s] : so;
    const uintptr_t obase = reinterpret_cast<uintptr_t>(out) + ob;   // absolute region start
    const u64 base = (u64)s * max_frames;
    const unsigned char* const wb = reinterpret_cast<const unsigned char*>(win);
    // wave-0 walk state (wave-uniform)
    u64 off = 0, g = 0, q = 0, q0 = 0;
    u32 nf = 0, nb = 0, nm = 0, first = 0;
    int status = WEBSOCKET_SEG_OK;
    bool walking = true, bodies_on = true, overflow = false;
    u32 open = w0 && open_io ? open_io[s] : 0u, cont = open;
    u32 cached = open && cached_io ? cached_io[s] : 0u;             // bytes of the pending message (u32)
    u64 wc = 0;                                                      // window's first chunk
    for (;;) {
        const u64 W0 = wc << 4, W1 = W0 + (u64)RSEG_C * 16;
        // ---- 1. LDS-DMA of the window (slices past the readable end are skipped)
        for (u32 i = wv; i < RSEG_L; i += RSEG_T / 64) {
            const u64 c0 = wc + (u64)i * 64;
            if (c0 > cmax) break;
            const u64 c = c0 + lane < cmax ? c0 + lane : cmax;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const WS_GLOBAL void*>(gseg + c),
                                             (lds_void*)(&win[i * 64]), 16, 0, 2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // ---- 2. wave 0: headers starting in [W0, W1)
        if (w0) {
            while (walking) {
                const WsRound r = ws_lds_round(win, W0, W1, lead, sl, off, g, nf, max_frames, lane);
                const WsHdr& h = r.h;
                const u64 pos = r.pos, X = pos + lead;
                const u32 mm = r.mm, code_m = r.code_m, ntake = r.ntake;
                if (lane < ntake && h.ret != 0) ws_store_desc(desc + base + nf + lane, so + pos, h);
                // bodies: consumed frames with ret > 0 (the a6 delivery rule), each at the
                // running sum of the bodies before it; none after an overflow
                const u32 nbr = bodies_on ? mm + (code_m == 1 ? 1u : 0u) : 0u;
                if (nbr) {
                    const bool body = lane < nbr;
                    const u64 len = body ? h.plen : 0;
                    u64 incl = len;
#pragma unroll
                    for (u32 d = 1; d < 64; d <<= 1) {
                        const u64 t = __shfl_up(incl, d, 64);
                        if (lane >= d) incl += t;
                    }
                    const u64 qs = q + incl - len;
                    // bodies must fit the segment's region (qs <= sl for every lane before the first overflow)
                    const u64 ovm = __ballot(body && len > sl - qs);
                    u32 ntb = ovm ? (u32)__builtin_ctzll(ovm) : nbr;
                    // the fragment cache's limit (see the file header): pending before lane i =
                    // frame i-1 not FIN (lane 0: carried), cached bytes = the message's bodies so far
                    const u32 blen = (u32)len;
                    u32 cincl = blen;
#pragma unroll
                    for (u32 d = 1; d < 64; d <<= 1) {
                        const u32 t = (u32)__shfl_up((int)cincl, d, 64);
                        if (lane >= d) cincl += t;
                    }
                    const bool finl = h.b0 >> 7;
                    const u64 fin_all = __ballot(body && finl);
                    const u64 fin_below = fin_all & ((1ull << lane) - 1);
                    const u32 lastf = fin_below ? 63 - __builtin_clzll(fin_below) : 0;
                    const u32 cincl_lastf = (u32)__shfl((int)cincl, (int)lastf, 64);
                    const u32 cbefore = fin_below ? cincl - blen - cincl_lastf : cached + cincl - blen;
                    const bool pend = lane == 0 ? open != 0 : !((fin_all >> (lane - 1)) & 1ull);
                    const u64 ccm = __ballot(body && (pend || !finl) && ws_cache_overflow(cbefore, blen, cache_max));
                    const u32 cst = ccm ? (u32)__builtin_ctzll(ccm) : 64u;
                    const bool cref = cst < ntb;                 // refused before any out-of-space body
                    if (cref) ntb = cst;
                    else if (ovm) { bodies_on = false; overflow = true; }
                    if (lane < ntb) {
                        BodyL b;
                        b.x0 = X + h.hdr; b.dst = qs; b.len = len;
                        tab[nb + lane] = b;
                        tkey[nb + lane] = h.masked ? rotl32(h.key, 8u * (u32)((obase + qs) & 3)) : 0u;
                    }
                    // messages closed by FIN frames among the taken bodies (body index == frame index)
                    const bool fin = lane < ntb && (h.b0 >> 7);
                    const u64 finm = __ballot(fin);
                    const u64 below = finm & ((1ull << lane) - 1);
                    const u32 prevl = below ? 63 - __builtin_clzll(below) : lane;
                    const u64 incl_prev = __shfl(incl, (int)prevl, 64);
                    if (fin) {
                        WebsocketMsgDesc_t m;
                        const u32 mfirst = below ? nb + prevl + 1 : first;
                        const u64 prevq = below ? q + incl_prev : q0;
                        m.out_off = ob + prevq; m.len = qs + len - prevq; m.first_frame = mfirst;
                        m.n_frames = nb + lane + 1 - mfirst; m.complete = 1; m.continued = below ? 0u : cont;
                        msg[base + nm + (u32)__builtin_popcountll(below)] = m;
                    }
                    const u64 tot = __shfl(incl, (int)(ntb ? ntb - 1 : 0), 64);
                    const u32 last = finm ? 63 - __builtin_clzll(finm) : 0;
                    const u64 incl_last = __shfl(incl, (int)last, 64);
                    if (finm) {
                        q0 = q + incl_last;
                        first = nb + last + 1;
                        cont = 0;
                        open = ntb > last + 1 ? 1u : 0u;
                        nm += (u32)__builtin_popcountll(finm);
                    } else if (ntb) {
                        open = 1;
                    }
                    const u32 ctot = (u32)__shfl((int)cincl, (int)(ntb ? ntb - 1 : 0), 64);
                    const u32 clast = (u32)__shfl((int)cincl, (int)last, 64);
                    if (ntb) cached = finm ? (ntb > last + 1 ? ctot - clast : 0u) : cached + ctot;
                    q += ntb ? tot : 0;
                    nb += ntb;
                    if (cref) {                              // refused: not consumed, the walk ends there
                        off = __shfl(pos, (int)cst, 64);
                        nf += cst + 1;
                        status = WEBSOCKET_SEG_ERR_CACHE_OVERFLOW;
                        walking = false;
                        break;
                    }
                }
                if (!ws_round_advance(r, off, g, nf, status, walking)) break;
            }
            // bodies with bytes in [W0, W1), and where the next window starts
            const BodyL t = tab[lane];
            const u64 bm = __ballot(lane < nb && t.len && t.x0 < W1 && t.x0 + t.len > W0);
            const u64 lend = nb ? tab[nb - 1].x0 + tab[nb - 1].len : 0;      // only the last body can pend
            if (lane == 0) {
                sh_blo = bm ? (u32)__builtin_ctzll(bm) : 1u;
                sh_bhi = bm ? 63u - (u32)__builtin_clzll(bm) : 0u;
                sh_next = lend > W1 ? W1 >> 4 : (walking ? (off + lead) >> 4 : ~0ull);
            }
        }
        __syncthreads();
        // ---- 3. wave wv: the window's part of bodies blo + wv, blo + wv + 4, ... The body table
        //         goes to registers once (lane i: body i); a body's fields come back by readlane,
        //         so the loop has no LDS round trips besides the data.
        const u32 blo = sh_blo, bhi = sh_bhi;
        const BodyL t = tab[lane];
        const u32 tk = tkey[lane];
        // The output chunk holding the boundary between bodies j-1 and j (off the 16-B grid) is
        // assembled whole by body j's wave when both bodies cover it from this window (one 16-B
        // store instead of byte stores from two waves): bit j of mg.
        u64 mg = 0;
        if (merge) {
            const u64 px0 = __shfl_up(t.x0, 1, 64), pdst = __shfl_up(t.dst, 1, 64), plen = __shfl_up(t.len, 1, 64);
            const u64 da = obase + t.dst, C0 = da & ~15ull;
            const bool ok = lane > blo && lane <= bhi && (da & 15) && t.len && plen >= da - C0 &&
                            px0 + (C0 - obase - pdst) >= W0 && t.len >= C0 + 16 - da && t.x0 + (C0 + 16 - da) <= W1;
            mg = __ballot(ok);
        }
        for (u32 bi = blo + wv; bi <= bhi; bi += RSEG_T / 64) {
            BodyL b;
            b.x0 = rl64(t.x0, bi); b.dst = rl64(t.dst, bi); b.len = rl64(t.len, bi);
            const u32 key = (u32)__builtin_amdgcn_readlane((int)tk, (int)bi);
            if (!b.len) continue;
            const u64 xa = b.x0 > W0 ? b.x0 : W0, xe = b.x0 + b.len < W1 ? b.x0 + b.len : W1;
            const u64 da = obase + b.dst + (xa - b.x0), de = da + (xe - xa);   // absolute output range
            const u64 A = (da + 15) & ~15ull, B = de & ~15ull;
            // interior: 16-B output chunks [A, B), source at xa + (y - da)
            if (A < B) {
                const u32 nch = (u32)((B - A) >> 4);
                const u32 o0 = (u32)(xa - W0 + (A - da));
                switch ((o0 >> 2) & 3u) {
                    case 0: reasm_copy<0>(win, o0, nch, key, A, lane); break;
                    case 1: reasm_copy<1>(win, o0, nch, key, A, lane); break;
                    case 2: reasm_copy<2>(win, o0, nch, key, A, lane); break;
                    default: reasm_copy<3>(win, o0, nch, key, A, lane);
                }
            }
            const bool mh = (mg >> bi) & 1ull, mt = bi < 63 && ((mg >> (bi + 1)) & 1ull);
            if (mh && lane == 0) {                                           // head chunk: bodies bi-1 and bi
                const u64 px0 = rl64(t.x0, bi - 1), pdst = rl64(t.dst, bi - 1);
                const u32 kp = (u32)__builtin_amdgcn_readlane((int)tk, (int)bi - 1);
                const u64 C0 = da & ~15ull;
                const u32 sb = (u32)(da - C0);                               // bytes of body bi-1 in it (1..15)
                // body bi-1's bytes as they sit at chunk positions 0..15, body bi's first 16 bytes
                const u32 op = (u32)(px0 + (C0 - obase - pdst) - W0), oc = (u32)(b.x0 - W0);
                u64 p0, p1, c0, c1;
                ws_hdr_from32(win[op >> 4], win[(op >> 4) + 1], op & 15u, p0, p1);
                ws_hdr_from32(win[oc >> 4], win[(oc >> 4) + 1], oc & 15u, c0, c1);
                // shift body bi's bytes up by sb positions (128-bit left shift by 8*sb bits)
                const u32 sh = 8u * sb;
                const u64 n0 = sh < 64 ? c0 << sh : 0ull;
                const u64 n1 = sh < 64 ? (c1 << sh) | (c0 >> (64 - sh)) : c0 << (sh - 64);
                const u64 m0 = sh < 64 ? (1ull << sh) - 1 : ~0ull;            // byte q < sb: body bi-1
                const u64 m1 = sh > 64 ? (1ull << (sh - 64)) - 1 : 0ull;
                const u64 kp64 = (u64)kp | ((u64)kp << 32), kc64 = (u64)key | ((u64)key << 32);
                const u64 r0 = ((p0 ^ kp64) & m0) | ((n0 ^ kc64) & ~m0);
                const u64 r1 = ((p1 ^ kp64) & m1) | ((n1 ^ kc64) & ~m1);
                u32x4 w;
                w.x = (u32)r0; w.y = (u32)(r0 >> 32); w.z = (u32)r1; w.w = (u32)(r1 >> 32);
                st16<1>(w, reinterpret_cast<gu32x4*>(C0));
            }
            // edges: lanes 0-15 the head [da, min(A, de)), lanes 16-31 the tail [max(A, B), de),
            // except a boundary chunk assembled whole above (head) or by the next body (tail)
            u64 y = 0;
            bool act = false;
            if (lane < 16) { y = da + lane; act = !mh && y < (A < de ? A : de); }
            else if (lane < 32) { y = (A > B ? A : B) + (lane - 16); act = !mt && y < de; }
            if (act) {
                const u32 kb = (key >> (8u * (u32)(y & 3))) & 0xFFu;
                *reinterpret_cast<gu8*>(y) = (unsigned char)(wb[xa - W0 + (y - da)] ^ kb);
            }
        }
        const u64 nxt = sh_next;
        __syncthreads();                                                     // window LDS is reused
        if (nxt == ~0ull) break;
        wc = nxt;
    }
    if (tid != 0) return;
    if (open && nb > first) {                                                // still open at the segment end
        WebsocketMsgDesc_t m;
        m.out_off = ob + q0; m.len = q - q0; m.first_frame = first; m.n_frames = nb - first;
        m.complete = 0; m.continued = cont;
        msg[base + nm++] = m;
    }
    ws_store_res(res + s, off, nf, overflow ? WEBSOCKET_SEG_ERR_OUT_SPACE : status);
    nmsg[s] = nm;
    if (open_io) open_io[s] = (unsigned char)open;
    if (cached_io) cached_io[s] = open ? cached : 0u;
}

// 0 auto, 1 fused segment kernel, 2 scan + layout + gather ("reasm_path")
WsOpt ws_reasm_path{0};
// fused kernel geometry ("reasm_cfg"): 0 17 KiB windows + 8 waves/SIMD (default: 49 SGPRs spill
// to VGPR lanes, yet 1.404-1.411 vs 1.459-1.462 ms on cfg5 once the body copy is alignbyte-based;
// round 1 measured it slower with the funnel-shift copy), 1 17 KiB windows at the compiler's
// occupancy (7 waves/SIMD), 2 19 KiB windows
WsOpt ws_reasm_cfg{0};

extern "C" WSFRAME_AMD_EXPORT int websocketframeBatchReassembleDeviceEx(
    const unsigned char* d_buf, unsigned long long buflen, const u64* d_seg_off, const u64* d_seg_len,
    unsigned int nseg, unsigned int max_frames, WebsocketFrameDesc_t* d_desc, WebsocketSegResult_t* d_res,
    unsigned char* d_out, const u64* d_out_off, WebsocketMsgDesc_t* d_msg, unsigned int* d_nmsg,
    unsigned char* d_open, unsigned int readcache_max_size, unsigned int* d_cached, void* hip_stream) {
    if (nseg == 0) return 0;
    if (!d_buf || !d_seg_off || !d_seg_len || !d_desc || !d_res || !d_out || !d_msg || !d_nmsg || max_frames == 0)
        return ws_set_msg("websocketframeBatchReassembleDevice: invalid argument");
    if ((reinterpret_cast<uintptr_t>(d_desc) | reinterpret_cast<uintptr_t>(d_res) | reinterpret_cast<uintptr_t>(d_msg)) & 15)
        return ws_set_msg("websocketframeBatchReassembleDevice: d_desc/d_res/d_msg not 16-B aligned");
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    // fused segment kernel for many small segments (one-shot blocks); the three-kernel
    // path for few or large segments (its gather spreads one segment over many waves)
    const int rpath = ws_reasm_path, rcfg = ws_reasm_cfg;
    const bool fused = rpath == 1 || (rpath == 0 && max_frames <= RSEG_TB && nseg >= 1024 && buflen <= (u64)nseg << 18);
    if (fused && max_frames <= RSEG_TB) {
        auto k = rcfg == 1 ? ws_reasm_seg_kernel<18, 1> : (rcfg == 2 ? ws_reasm_seg_kernel<20, 1> : ws_reasm_seg_kernel<18, 8>);
        const int swin = ws_seg_win;                                   // one read per call
        const WsWinGrid wg = ws_win_grid(nseg, swin < 0 ? 3 : swin);
        // (body-boundary chunks: one byte-store instruction from 31 lanes; one lane assembling
        // them whole measured slower, cfg5u 1.65 vs 1.50 ms)
        hipLaunchKernelGGL(k, dim3(wg.blocks), dim3(RSEG_T), 0, st, d_buf, max_frames, d_seg_off,
                           d_seg_len, d_desc, d_res, d_out, d_out_off, d_msg, d_nmsg, d_open, 0u, nseg, wg.wsh, wg.ppw,
                           (u32)readcache_max_size, d_cached);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_reasm_seg_kernel launch", e);
    }
    const u64 nslots = (u64)nseg * max_frames;
    const size_t piece = ws_piece_workspace_bytes(buflen, nseg, max_frames);
    const size_t rec_off = (piece + 255) & ~(size_t)255;
    const size_t nb_off = rec_off + nslots * sizeof(GatherRec);
    void* ws = nullptr;
    WsSlot slot;
    int rc = slot.acquire(st);
    if (rc || (rc = slot.workspace(nb_off + (size_t)nseg * 4 + 64, 16, &ws))) return rc;
    unsigned char* w8 = reinterpret_cast<unsigned char*>(ws);
    GatherRec* recs = reinterpret_cast<GatherRec*>(w8 + rec_off);
    u32* nbody = reinterpret_cast<u32*>(w8 + nb_off);
    WsLaunch L;
    L.buf = const_cast<unsigned char*>(d_buf); L.seg_off = d_seg_off; L.seg_len = d_seg_len; L.nseg = nseg;
    L.max_frames = max_frames; L.desc_base = nullptr; L.desc = d_desc; L.res = d_res; L.stream = st;
    L.cus = slot.cus; L.lds_per_cu = slot.lds;
    PieceWs P;
    if ((rc = ws_launch_piece_scan(L, 0, buflen, w8, ws_next_gen(), &P))) return rc;
    hipLaunchKernelGGL(ws_reasm_layout_kernel, dim3((u32)(((u64)nseg * RLAY_G + RLAY_T - 1) / RLAY_T)), dim3(RLAY_T), 0, st, d_buf, nseg,
                       max_frames, d_seg_off, d_seg_len, d_desc, d_res, P.items, d_out, d_out_off, d_msg, d_nmsg,
                       d_open, recs, nbody, (u32)readcache_max_size, d_cached);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ws_set_err("ws_reasm_layout_kernel launch", e);
    const u64 waves = nslots;
    const u64 blocks = (waves + RGAT_T / 64 - 1) / (RGAT_T / 64);
    const u32 grid = (u32)(blocks < (1ull << 20) ? blocks : (1ull << 20));
    hipLaunchKernelGGL((ws_reasm_gather_kernel<1>), dim3(grid), dim3(RGAT_T), 0, st, d_buf, d_out, max_frames, nslots,
                       recs, nbody);
    if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_reasm_gather_kernel launch", e);
    return 0;
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeBatchReassembleDevice(
    const unsigned char* d_buf, unsigned long long buflen, const u64* d_seg_off, const u64* d_seg_len,
    unsigned int nseg, unsigned int max_frames, WebsocketFrameDesc_t* d_desc, WebsocketSegResult_t* d_res,
    unsigned char* d_out, const u64* d_out_off, WebsocketMsgDesc_t* d_msg, unsigned int* d_nmsg,
    unsigned char* d_open, void* hip_stream) {
    return websocketframeBatchReassembleDeviceEx(d_buf, buflen, d_seg_off, d_seg_len, nseg, max_frames, d_desc, d_res,
                                                 d_out, d_out_off, d_msg, d_nmsg, d_open, 0, nullptr, hip_stream);
}
