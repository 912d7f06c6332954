// ws_segblock.hip — default decode path: one workgroup per rx segment.
//
// Per round of T*U 16-B chunks of the segment (one round covers a 64 KiB inbuf):
//   1. every thread issues its U payload loads at once (the chunk addresses need
//      only seg_off/seg_len, not the frames);
//   2. meanwhile wave 0 walks the frame headers in order — the reactor loop
//      (net_reactor.c:515-526) over websocketframeDecode's header logic
//      (websocketframe.c:112-165, ws_parse) — with SCALAR loads (counted by
//      lgkmcnt, so they never wait on the vector payload loads; they hit lines
//      those loads are already bringing in), writes each descriptor, and appends
//      each frame's payload range + rotated key to an LDS frame ring;
//   3. one barrier; every thread XORs its chunks with their frame's key and stores
//      payload bytes only (ws_xor_round), and the workgroup exits.
// So each wave does one load round and one store round per 64 KiB segment (on CDNA
// vmcnt retires loads and stores in issue order: a wave that loads after its own
// stores waits for them), the serial header walk hides under the payload-load
// latency, and there is no second kernel or workspace. Larger segments take more
// rounds; frames spanning rounds stay in the ring.
#include "ws_common.h"

int ws_dbg_flags = 0;  // debug builds of the A/B tools: bit 0 = skip payload stores

template <int FW>
struct SegLds {
    Item tab[FW];        // this round's table (32-bit offsets relative to the round start)
    u64 rp0[FW];         // frame ring: payload ranges relative to the segment origin
    u64 rp1[FW];
    u32 rrk[FW];
    u32 cnt;             // entries in tab
    u32 c1;              // round end (chunks, relative to the round start)
    u32 more;            // another round has payload to unmask
};

template <int T, int U, int NT>
__global__ __launch_bounds__(T) void ws_segblock_kernel(unsigned char* __restrict__ buf,
                                                        const u64* __restrict__ seg_off,
                                                        const u64* __restrict__ seg_len, u32 max_frames,
                                                        const u64* __restrict__ desc_base,
                                                        WebsocketFrameDesc_t* __restrict__ desc,
                                                        WebsocketSegResult_t* __restrict__ res, int dbg) {
    constexpr u32 FW = 256;                // ring / table capacity (frames per round)
    constexpr long long RB = (long long)T * U * 16;
    __shared__ SegLds<FW> L;
    const u32 s = blockIdx.x;
    const u32 tid = threadIdx.x;
    const bool walker = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;
    const u64 so = seg_off[s], sl = seg_len[s];
    const u64 dbase = desc_base ? desc_base[s] : (u64)s * max_frames;
    const uintptr_t seg_abs = reinterpret_cast<uintptr_t>(buf + so);
    const uintptr_t origin = seg_abs & ~(uintptr_t)15;
    const u64 lead = (u64)(seg_abs - origin);                              // segment start - origin
    const u64 nchunks = (u64)(((seg_abs + sl + 15) & ~(uintptr_t)15) - origin) >> 4;
    gu32x4* const base = reinterpret_cast<gu32x4*>(origin);

    // walk state (wave-uniform, used by wave 0)
    u64 off = 0;
    u32 nf = 0, head = 0, tail = 0;
    u64 g = 0;                 // stride guess: length of the last frame walked
    int status = WEBSOCKET_SEG_OK;
    bool wdone = false;

    for (u64 c0 = 0; c0 < nchunks;) {
        const u64 c1full = c0 + (u64)(T * U) < nchunks ? c0 + (u64)(T * U) : nchunks;
        // ---- 1. payload loads: unconditional, clamped to the round's last chunk
        const u32 lim0 = (u32)(c1full - 1 - c0);
        gu32x4* const rb = base + c0;
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld16<NT>(rb + min(tid + (u32)(u * T), lim0));
        // ---- 2. wave 0: walk headers, build this round's frame table
        if (walker) {
            const long long r0 = (long long)(c0 << 4);
            u64 endx = c1full << 4;                                          // round end (bytes from origin)
            u32 cnt = 0;
            auto put = [&](u64 p0, u64 p1, u32 rk) {
                long long a = (long long)p0 - r0, b = (long long)p1 - r0;
                a = a < -16 ? -16 : (a > RB + 16 ? RB + 16 : a);
                b = b < -16 ? -16 : (b > RB + 16 ? RB + 16 : b);
                if (tid == 0) {
                    Item it;
                    it.p0 = (int)a; it.p1 = (int)b; it.rkey = rk; it.pad = 0;
                    L.tab[cnt] = it;
                }
                ++cnt;
            };
            // frames carried over from the previous round (still ending past its start)
            while (head < tail && L.rp1[head % FW] <= (c0 << 4)) ++head;
            for (u32 i = head; i < tail; ++i) put(L.rp0[i % FW], L.rp1[i % FW], L.rrk[i % FW]);
            // Speculative walk: lane k parses the header at off + k*g (g = length of the last
            // frame walked). Lane k's position is the true frame position iff frames 0..k-1
            // all had ret == g, so every frame up to the first length change (ballot) is
            // walked in one round trip; that frame is itself correctly placed and consumed,
            // and the next batch speculates with its length.
            const u32 lane = tid & 63;
            while (!wdone) {
                const u32 room = FW - (tail - head);
                if (lead + off >= endx) break;                               // next round's frame
                if (room == 0) {                                             // ring full: end the round
                    const u64 cap = (lead + off) & ~(u64)15;                 // chunks before it only touch
                    if (cap < endx) endx = cap;                              // frames already in the ring
                    break;
                }
                const u32 kmax = room < 64u ? room : 64u;
                const u32 k = lane;
                const u64 pos = off + (u64)k * g;                            // candidate frame offset
                // per-lane outcome, in the reactor loop's order (net_reactor.c:515-526)
                //   0 consumed, chain continues with stride g   1 consumed, ret != g: batch ends
                //   2 consumed, walk ends (ret <= 0)             3 not consumed, walk ends
                //   4 not consumed: round end / beyond kmax
                // branch-free: every lane loads the 32 bytes at floor16 of its candidate
                // (a harmless re-read of the segment start when the candidate is invalid)
                const bool eval = k < kmax && (k == 0 || g > 0) && pos < sl;
                const uintptr_t pp = seg_abs + (eval ? pos : 0);
                const gu32x4* q = reinterpret_cast<const gu32x4*>(pp & ~(uintptr_t)15);
                const u32x4 x0 = q[0], x1 = q[1];
                u64 h0, h1;
                ws_hdr_from32(x0, x1, (u32)(pp & 15), h0, h1);
                const WsHdr h = ws_parse(h0, h1, eval ? sl - pos : 0);
                // per-lane outcome, in the reactor loop's order (net_reactor.c:515-526)
                //   0 consumed, chain continues with stride g   1 consumed, ret != g: batch ends
                //   2 consumed, walk ends (ret <= 0)             3 not consumed, walk ends
                //   4 not consumed: round end / beyond kmax
                u32 code = 4;
                int st = WEBSOCKET_SEG_OK;
                if (k < kmax && (k == 0 || g > 0)) {
                    if (lead + pos >= endx) code = 4;
                    else if (pos >= sl) code = 3;
                    else if (nf + k >= max_frames) { code = 3; st = WEBSOCKET_SEG_MAX_FRAMES; }
                    else if (sl - pos < 2) code = 3;                           // websocketframe.c:121
                    else if (h.kind == WS_PARSE_INCOMPLETE) code = 3;
                    else if (h.kind == WS_PARSE_WRAP) { code = 3; st = WEBSOCKET_SEG_ERR_LEN_WRAP; }
                    else if (h.ret == 0) code = 2;                             // (int) truncated to 0
                    else if (h.ret < 0) { code = 2; st = WEBSOCKET_SEG_ERR_DECODE; }
                    else code = (u64)(u32)h.ret == g ? 0u : 1u;
                }
                const u64 stop_mask = __ballot(code != 0);
                const u32 m = stop_mask ? (u32)__builtin_ctzll(stop_mask) : 64u;   // first non-continuing lane
                const u32 code_m = m < 64 ? (u32)__builtin_amdgcn_readlane((int)code, (int)m) : 4u;
                const bool take_m = code_m == 1 || code_m == 2;
                const u32 ntake = m + (take_m ? 1u : 0u);
                // consume lanes [0, ntake): items, ring, descriptors — in parallel
                if (k < ntake) {
                    const u64 fpos = lead + pos;
                    u64 p0 = fpos, p1 = fpos;
                    u32 rk = 0;
                    if (h.masked && h.plen) {
                        p0 = fpos + h.hdr;
                        p1 = p0 + h.plen;
                        rk = rotl32(h.key, 8u * (u32)(p0 & 3));
                    }
                    long long a0 = (long long)p0 - r0, a1 = (long long)p1 - r0;
                    a0 = a0 < -16 ? -16 : (a0 > RB + 16 ? RB + 16 : a0);
                    a1 = a1 < -16 ? -16 : (a1 > RB + 16 ? RB + 16 : a1);
                    Item it;
                    it.p0 = (int)a0; it.p1 = (int)a1; it.rkey = rk; it.pad = 0;
                    L.tab[cnt + k] = it;
                    const u32 ri = (tail + k) % FW;
                    L.rp0[ri] = p0; L.rp1[ri] = p1; L.rrk[ri] = rk;
                    if (h.ret != 0) ws_store_desc(desc + dbase + nf + k, so + pos, h);
                }
                cnt += ntake;
                tail += ntake;
                if (m == 64) {                                               // whole batch continued
                    nf += 64;
                    off += 64 * g;
                    continue;
                }
                const u64 pos_m = off + (u64)m * g;
                const int ret_m = __builtin_amdgcn_readlane(h.ret, (int)m);
                const int st_m = __builtin_amdgcn_readlane(st, (int)m);
                nf += m;
                off = pos_m;
                if (code_m == 4) continue;                                   // round end / batch limit:
                                                                             // the loop top decides
                if (code_m == 1) {                                           // consumed, new stride
                    nf += 1;
                    off = pos_m + (u32)ret_m;
                    g = (u32)ret_m;
                    continue;
                }
                if (code_m == 2 && ret_m != 0) nf += 1;                      // ret < 0 keeps its descriptor
                status = st_m;                                               // codes 2 and 3: walk ends
                wdone = true;
                break;
            }
            // another round is needed if the walk continues or a frame extends past this round
            bool more = !wdone;
            for (u32 i = head; i < tail && !more; ++i) more = L.rp1[i % FW] > endx;
            if (tid == 0) {
                L.cnt = cnt;
                L.c1 = (u32)((endx >> 4) - c0);
                L.more = more;
            }
        }
        __syncthreads();
        const u32 cnt = L.cnt;
        const u32 c1r = L.c1;
        const bool more = L.more;
        // ---- 3. XOR + store this round's chunks [0, c1r)
        if (c1r && !(dbg & 1)) ws_xor_round<T, U, NT>(v, rb, c1r - 1, L.tab, cnt, tid);
        if (dbg & 1) {
#pragma unroll
            for (int u = 0; u < U; ++u) asm volatile("" ::"v"(v[u].x));
        }
        c0 += c1r;
        if (!more) break;
        __syncthreads();  // tab is rewritten next round
    }
    if (walker && tid == 0) ws_store_res(res + s, off, nf, status);
}

template <int T, int U>
static int launch_segblock(const WsLaunch& L, int nt) {
    if (nt == 1)
        hipLaunchKernelGGL((ws_segblock_kernel<T, U, 1>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, L.res, ws_dbg_flags);
    else if (nt == 2)
        hipLaunchKernelGGL((ws_segblock_kernel<T, U, 2>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, L.res, ws_dbg_flags);
    else
        hipLaunchKernelGGL((ws_segblock_kernel<T, U, 0>), dim3(L.nseg), dim3(T), 0, L.stream, L.buf, L.seg_off,
                           L.seg_len, L.max_frames, L.desc_base, L.desc, L.res, ws_dbg_flags);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_segblock_kernel launch", e);
}

// cfg: 0 -> 256 threads x 17 chunks (68 KiB rounds), 1 -> 512 x 9 (72 KiB), 2 -> 1024 x 5 (80 KiB),
//      3 -> 256 x 8 (32 KiB), 4 -> 512 x 4 (32 KiB)
int ws_launch_segblock(const WsLaunch& L, int cfg, int nt) {
    switch (cfg) {
    case 1: return launch_segblock<512, 9>(L, nt);
    case 2: return launch_segblock<1024, 5>(L, nt);
    case 3: return launch_segblock<256, 8>(L, nt);
    case 4: return launch_segblock<512, 4>(L, nt);
    default: return launch_segblock<256, 17>(L, nt);
    }
}
