// ws_segblock.hip — one workgroup per rx segment, one memory round per 64 KiB.
//
// Per round of the segment's 16-B chunks:
//   1. the payload is fetched in one go: into registers (ws_segblock_kernel) or
//      straight into LDS by LDS-DMA (ws_segdma_kernel, no VGPRs held);
//   2. wave 0 walks the frame headers — the reactor loop (net_reactor.c:515-526) over
//      websocketframeDecode's header logic (websocketframe.c:112-165, ws_parse) —
//      with STRIDE SPECULATION: lane k parses the header at off + k*g (g = length of
//      the last frame); lane k's position is the true one iff frames 0..k-1 all had
//      length g, so a run of equal frames is walked in one step (first change found
//      by ballot), descriptors and frame-table entries are written by the lanes in
//      parallel, and the next step speculates with the new length. Header bytes come
//      from HBM (register variant) or from the LDS copy (DMA variant: no extra round
//      trip at all);
//   3. one barrier; every thread XORs its chunks with their frame's rotated key and
//      stores payload bytes only (full chunks one 16-B store, chunks at frame edges
//      exactly the payload bytes); the workgroup exits.
// A wave never loads after its own stores (on CDNA vmcnt retires loads and stores in
// issue order), which is what the one-round-per-wave streaming ceiling needs
// (DESIGN.md §4). Frames spanning rounds stay in an LDS ring.
#include "ws_common.h"

int ws_dbg_flags = 0;  // A/B tooling: bit 0 = skip payload stores (walk + loads only)

template <int FW>
struct SegRing {
    Item tab[FW];        // this round's table (32-bit offsets relative to the round start)
    u64 rp0[FW];         // frame ring: payload ranges relative to the segment origin
    u64 rp1[FW];
    u32 rrk[FW];
    u32 cnt;             // entries in tab
    u32 c1;              // round end (chunks, relative to the round start)
    u32 more;            // another round has payload to unmask
};

struct WalkState {
    u64 off;             // segment offset of the next frame
    u64 g;               // stride guess: length of the last frame walked
    u32 nf, head, tail;
    int status;
    bool wdone;
};

// Segment constants shared by both kernels.
struct SegCtx {
    u64 so, sl, dbase, lead, nchunks;
    uintptr_t seg_abs;
    u32 max_frames;
    WebsocketFrameDesc_t* desc;
};

__device__ __forceinline__ SegCtx seg_ctx(unsigned char* buf, const u64* seg_off, const u64* seg_len, u32 max_frames,
                                          const u64* desc_base, WebsocketFrameDesc_t* desc) {
    SegCtx S;
    const u32 s = blockIdx.x;
    S.so = seg_off[s];
    S.sl = seg_len[s];
    S.dbase = desc_base ? desc_base[s] : (u64)s * max_frames;
    S.seg_abs = reinterpret_cast<uintptr_t>(buf + S.so);
    const uintptr_t origin = S.seg_abs & ~(uintptr_t)15;
    S.lead = (u64)(S.seg_abs - origin);
    S.nchunks = (u64)(((S.seg_abs + S.sl + 15) & ~(uintptr_t)15) - origin) >> 4;
    S.max_frames = max_frames;
    S.desc = desc;
    return S;
}

// One round of the walk, run by all 64 lanes of wave 0. `fetch(prel, x0, x1)` returns
// the 32 bytes at floor16(prel) (origin-relative). Frames starting at or after
// walk_end are left for the next round; if such a frame starts inside this round,
// the round's XOR range ends at its 16-B chunk (only walked frames touch the chunks
// before it). Writes L.cnt / L.c1 / L.more.
template <int FW, typename Fetch>
__device__ __forceinline__ void seg_walk_round(WalkState& W, SegRing<FW>& L, const SegCtx& S, u64 c0, u64 c1full,
                                               u64 walk_end, long long RB, Fetch fetch) {
    const u32 lane = threadIdx.x & 63;
    const long long r0 = (long long)(c0 << 4);
    u64 endx = c1full << 4;                                              // round end (bytes from origin)
    u32 cnt = 0;
    auto clampi = [&](u64 p) -> int {
        const long long a = (long long)p - r0;
        return (int)(a < -16 ? -16 : (a > RB + 16 ? RB + 16 : a));
    };
    // frames carried over from the previous round (still ending past its start)
    while (W.head < W.tail && L.rp1[W.head % FW] <= (c0 << 4)) ++W.head;
    for (u32 i = W.head; i < W.tail; ++i) {
        if (lane == 0) {
            Item it;
            it.p0 = clampi(L.rp0[i % FW]); it.p1 = clampi(L.rp1[i % FW]); it.rkey = L.rrk[i % FW]; it.pad = 0;
            L.tab[cnt] = it;
        }
        ++cnt;
    }
    while (!W.wdone) {
        const u32 room = FW - (W.tail - W.head);
        if (S.lead + W.off >= walk_end || room == 0) {                    // defer / ring full: end the round
            const u64 cap = (S.lead + W.off) & ~(u64)15;
            if (cap < endx) endx = cap;
            break;
        }
        const u32 kmax = room < 64u ? room : 64u;
        const u32 k = lane;
        const u64 pos = W.off + (u64)k * W.g;                             // candidate frame offset
        const bool cand = k < kmax && (k == 0 || W.g > 0);
        const bool eval = cand && pos < S.sl;
        const u64 prel = S.lead + (eval ? pos : 0);
        u32x4 x0, x1;
        fetch(prel, x0, x1);
        u64 h0, h1;
        ws_hdr_from32(x0, x1, (u32)(prel & 15), h0, h1);
        const WsHdr h = ws_parse(h0, h1, eval ? S.sl - pos : 0);
        // per-lane outcome, in the reactor loop's order (net_reactor.c:515-526)
        //   0 consumed, chain continues with stride g   1 consumed, ret != g: step ends
        //   2 consumed, walk ends (ret <= 0)             3 not consumed, walk ends
        //   4 not consumed: round end / beyond kmax
        u32 code = 4;
        int st = WEBSOCKET_SEG_OK;
        if (cand) {
            if (S.lead + pos >= walk_end) code = 4;
            else if (pos >= S.sl) code = 3;
            else if (W.nf + k >= S.max_frames) { code = 3; st = WEBSOCKET_SEG_MAX_FRAMES; }
            else if (S.sl - pos < 2) code = 3;                            // websocketframe.c:121
            else if (h.kind == WS_PARSE_INCOMPLETE) code = 3;
            else if (h.kind == WS_PARSE_WRAP) { code = 3; st = WEBSOCKET_SEG_ERR_LEN_WRAP; }
            else if (h.ret == 0) code = 2;                                // (int) truncated to 0
            else if (h.ret < 0) { code = 2; st = WEBSOCKET_SEG_ERR_DECODE; }
            else code = (u64)(u32)h.ret == W.g ? 0u : 1u;
        }
        const u64 stop_mask = __ballot(code != 0);
        const u32 m = stop_mask ? (u32)__builtin_ctzll(stop_mask) : 64u;  // first non-continuing lane
        const u32 code_m = m < 64 ? (u32)__builtin_amdgcn_readlane((int)code, (int)m) : 4u;
        const u32 ntake = m + ((code_m == 1 || code_m == 2) ? 1u : 0u);
        // consume lanes [0, ntake): frame-table entries, ring, descriptors — in parallel
        if (k < ntake) {
            const u64 fpos = S.lead + pos;
            u64 p0 = fpos, p1 = fpos;
            u32 rk = 0;
            if (h.masked && h.plen) {
                p0 = fpos + h.hdr;
                p1 = p0 + h.plen;
                rk = rotl32(h.key, 8u * (u32)(p0 & 3));
            }
            Item it;
            it.p0 = clampi(p0); it.p1 = clampi(p1); it.rkey = rk; it.pad = 0;
            L.tab[cnt + k] = it;
            const u32 ri = (W.tail + k) % FW;
            L.rp0[ri] = p0; L.rp1[ri] = p1; L.rrk[ri] = rk;
            if (h.ret != 0) ws_store_desc(S.desc + S.dbase + W.nf + k, S.so + pos, h);
        }
        cnt += ntake;
        W.tail += ntake;
        if (m == 64) {                                                    // whole step continued
            W.nf += 64;
            W.off += 64 * W.g;
            continue;
        }
        const u64 pos_m = W.off + (u64)m * W.g;
        const int ret_m = __builtin_amdgcn_readlane(h.ret, (int)m);
        const int st_m = __builtin_amdgcn_readlane(st, (int)m);
        W.nf += m;
        W.off = pos_m;
        if (code_m == 4) continue;                                        // the loop top decides
        if (code_m == 1) {                                                // consumed, new stride
            W.nf += 1;
            W.off = pos_m + (u32)ret_m;
            W.g = (u32)ret_m;
            continue;
        }
        if (code_m == 2 && ret_m != 0) W.nf += 1;                         // ret < 0 keeps its descriptor
        W.status = st_m;                                                  // codes 2 and 3: walk ends
        W.wdone = true;
        break;
    }
    // another round is needed if the walk continues or a frame extends past this round
    bool more = !W.wdone;
    for (u32 i = W.head; i < W.tail && !more; ++i) more = L.rp1[i % FW] > endx;
    if (lane == 0) {
        L.cnt = cnt;
        L.c1 = (u32)((endx >> 4) - c0);
        L.more = more;
    }
}

// ---------------------------------------------------------------------------------------------
// variant A: payload in registers (U chunks per thread), headers fetched from HBM

template <int T, int U, int NT>
__global__ __launch_bounds__(T) void ws_segblock_kernel(unsigned char* __restrict__ buf,
                                                        const u64* __restrict__ seg_off,
                                                        const u64* __restrict__ seg_len, u32 max_frames,
                                                        const u64* __restrict__ desc_base,
                                                        WebsocketFrameDesc_t* __restrict__ desc,
                                                        WebsocketSegResult_t* __restrict__ res, int dbg) {
    constexpr int FW = 256;
    constexpr long long RB = (long long)T * U * 16;
    __shared__ SegRing<FW> L;
    const u32 tid = threadIdx.x;
    const bool walker = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;
    const SegCtx S = seg_ctx(buf, seg_off, seg_len, max_frames, desc_base, desc);
    gu32x4* const base = reinterpret_cast<gu32x4*>(S.seg_abs - S.lead);
    WalkState W = {0, 0, 0, 0, 0, WEBSOCKET_SEG_OK, false};

    for (u64 c0 = 0; c0 < S.nchunks;) {
        const u64 c1full = c0 + (u64)(T * U) < S.nchunks ? c0 + (u64)(T * U) : S.nchunks;
        const u32 lim0 = (u32)(c1full - 1 - c0);
        gu32x4* const rb = base + c0;
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld16<NT>(rb + min(tid + (u32)(u * T), lim0));
        if (walker)
            seg_walk_round<FW>(W, L, S, c0, c1full, c1full << 4, RB, [&](u64 prel, u32x4& x0, u32x4& x1) {
                const gu32x4* q = base + (prel >> 4);
                x0 = q[0];
                x1 = q[1];
            });
        __syncthreads();
        const u32 cnt = L.cnt, c1r = L.c1;
        const bool more = L.more;
        if (c1r && !(dbg & 1)) ws_xor_round<T, U, NT>(v, rb, c1r - 1, L.tab, cnt, tid);
        if (dbg & 1) {
#pragma unroll
            for (int u = 0; u < U; ++u) asm volatile("" ::"v"(v[u].x));
        }
        c0 += c1r;
        if (!more) break;
        __syncthreads();  // tab is rewritten next round
    }
    if (walker && tid == 0) ws_store_res(res + blockIdx.x, W.off, W.nf, W.status);
}

// ---------------------------------------------------------------------------------------------
// variant B: payload staged in LDS by LDS-DMA (RC chunks per round), headers read from LDS

typedef __attribute__((address_space(3))) void lds_void;

template <int T, int RC, int NT>
__global__ __launch_bounds__(T) void ws_segdma_kernel(unsigned char* __restrict__ buf, const u64* __restrict__ seg_off,
                                                      const u64* __restrict__ seg_len, u32 max_frames,
                                                      const u64* __restrict__ desc_base,
                                                      WebsocketFrameDesc_t* __restrict__ desc,
                                                      WebsocketSegResult_t* __restrict__ res, int dbg) {
    constexpr int FW = 128;
    constexpr u32 NW = T / 64;
    constexpr long long RB = (long long)RC * 16;
    static_assert(RC % 64 == 0, "rounds are whole LDS-DMA wave instructions");
    __shared__ __attribute__((aligned(16))) u32x4 lbuf[RC + 2];    // +2: 32-B header window at the end
    __shared__ SegRing<FW> L;
    const u32 tid = threadIdx.x, lane = tid & 63;
    const u32 wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool walker = wv == 0;
    const SegCtx S = seg_ctx(buf, seg_off, seg_len, max_frames, desc_base, desc);
    gu32x4* const base = reinterpret_cast<gu32x4*>(S.seg_abs - S.lead);
    WalkState W = {0, 0, 0, 0, 0, WEBSOCKET_SEG_OK, false};

    for (u64 c0 = 0; c0 < S.nchunks;) {
        const u64 c1full = c0 + (u64)RC < S.nchunks ? c0 + (u64)RC : S.nchunks;
        const u32 nrc = (u32)(c1full - c0);
        gu32x4* const rb = base + c0;
        // ---- 1. LDS-DMA: wave w stages 1 KiB pieces w, w+NW, ... (lane-linear: chunk i*64+lane)
        for (u32 i = wv; i * 64 < nrc; i += NW) {
            const u32 c = min(i * 64 + lane, nrc - 1);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const WS_GLOBAL void*>(rb + c),
                                             (lds_void*)(&lbuf[i * 64]), 16, 0, NT == 1 ? 2 : 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // ---- 2. wave 0 walks from the LDS copy; a header whose 32-B window could pass the
        //         staged data (not the last round) waits for the next round
        if (walker) {
            const u64 endx = c1full << 4;
            const u64 walk_end = c1full == S.nchunks ? endx : endx - 32;
            seg_walk_round<FW>(W, L, S, c0, c1full, walk_end, RB, [&](u64 prel, u32x4& x0, u32x4& x1) {
                u32 i = (u32)((prel >> 4) - c0);
                i = i > (u32)RC ? (u32)RC : i;
                x0 = lbuf[i];
                x1 = lbuf[i + 1];
            });
        }
        __syncthreads();
        const u32 cnt = L.cnt, c1r = L.c1;
        const bool more = L.more;
        // ---- 3. XOR from LDS, store payload bytes (wave-uniform item cursor per 64-chunk slot)
        if (!(dbg & 1)) {
            u32 icur = 0;
            for (u32 lw = 64u * wv; lw < c1r; lw += T) {
                while (icur < cnt && L.tab[icur].p1 <= (int)(lw * 16)) ++icur;
                const u32 lc = lw + lane;
                if (lc >= c1r) continue;
                const int x = (int)(lc * 16);
                u32 j = icur;
                Item it = L.tab[j < cnt ? j : 0];
                while (j < cnt && it.p1 <= x) { ++j; it = L.tab[j < cnt ? j : 0]; }
                if (j >= cnt || it.p0 >= x + 16) continue;
                const u32x4 v = lbuf[lc];
                gu32x4* const pc = rb + lc;
                if (it.p0 <= x && it.p1 >= x + 16) {
                    st16<NT>(v ^ it.rkey, pc);
                    continue;
                }
                ws_store_partial<NT>(v, pc, L.tab, j, cnt, x);
            }
        }
        c0 += c1r;
        if (!more) break;
        __syncthreads();  // lbuf and tab are rewritten next round
    }
    if (walker && tid == 0) ws_store_res(res + blockIdx.x, W.off, W.nf, W.status);
}

template <int T, int U>
static int launch_segblock(const WsLaunch& L, int nt) {
    if (nt == 1)
        hipLaunchKernelGGL((ws_segblock_kernel<T, U, 1>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, L.res, ws_dbg_flags);
    else
        hipLaunchKernelGGL((ws_segblock_kernel<T, U, 0>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, L.res, ws_dbg_flags);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_segblock_kernel launch", e);
}

template <int T, int RC>
static int launch_segdma(const WsLaunch& L, int nt) {
    if (nt == 1)
        hipLaunchKernelGGL((ws_segdma_kernel<T, RC, 1>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, L.res, ws_dbg_flags);
    else
        hipLaunchKernelGGL((ws_segdma_kernel<T, RC, 0>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, L.res, ws_dbg_flags);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_segdma_kernel launch", e);
}

// cfg 0-4: register payload (threads x chunks): 256x17, 512x9, 1024x5, 256x8, 512x4
// cfg 10-13: LDS-DMA payload (threads x round chunks): 512x4480 (70 KiB, 2 blocks/CU),
//            256x4480, 1024x4480, 512x2944 (46 KiB, 3 blocks/CU)
int ws_launch_segblock(const WsLaunch& L, int cfg, int nt) {
    switch (cfg) {
    case 1: return launch_segblock<512, 9>(L, nt);
    case 2: return launch_segblock<1024, 5>(L, nt);
    case 3: return launch_segblock<256, 8>(L, nt);
    case 4: return launch_segblock<512, 4>(L, nt);
    case 10: return launch_segdma<512, 4480>(L, nt);
    case 11: return launch_segdma<256, 4480>(L, nt);
    case 12: return launch_segdma<1024, 4480>(L, nt);
    case 13: return launch_segdma<512, 2944>(L, nt);
    default: return launch_segblock<256, 17>(L, nt);
    }
}
