// ws_segfuse.hip — decode path 4: ONE workgroup per rx segment, walk + unmask fused
// in one kernel, for batches of many small segments (many connections, a few KiB each;
// cfg5's 16.5 KiB segments of 1 KiB frames).
//
// The piece path (ws_piece.hip) needs a scan kernel whose cost is one header-line
// fetch per frame; for 1 KiB frames that is 1/8 of the wire read a second time. Here
// the segment's bytes stream through LDS in windows (one window up to 17 KiB: a
// one-shot block — load once, store once, exit):
//   1. LDS-DMA (global_load_lds_dwordx4) of the window: every wave issues its 1 KiB
//      slices at once, clamped to the segment's readable bytes (segment +
//      WEBSOCKET_BATCH_PAD), no registers involved;
//   2. wave 0 walks the reactor loop (net_reactor.c:515-526) over the headers in LDS
//      (ws_lds_round: 64 candidate frames per round by stride speculation), writes the
//      descriptors and the segment's frame table (payload range + key of every
//      consumed masked frame — websocketframe.c:153-158 also unmasks a frame whose
//      (int) return is <= 0);
//   3. all waves XOR the window's chunks: the frame table sits in registers (lane i,
//      frame i), a 1 KiB row's frames come from one ballot, per-lane byte masks (key
//      rotated to the chunk phase) by readlane, one 16-B store per chunk
//      that holds payload bytes — header bytes of a chunk inside the segment are
//      stored back unchanged; a chunk shared with a neighbouring segment gets exact
//      byte stores.
// Frames longer than a window continue in the next one; the walk state and the frame
// table (max_frames <= SF_TB) persist across windows.
#include "ws_common.h"

// window = SF_L LDS-DMA wave instructions of 1 KiB: (SF_L-1) KiB owned + 1 KiB look-ahead;
// SF_L = 18 is ~20 KB of LDS: 8 workgroups (32 waves) per CU ("segfuse_cfg" A/B)
#define SF_TB 64                                    // frame table entries = max max_frames of this path

typedef __attribute__((address_space(3))) void lds_void;

struct FrameL {         // masked payload of a consumed frame (LDS)
    u64 x0;             // first payload byte, window coordinates (segment offset + lead)
    u64 x1;             // one past the last
    u32 rkey;           // key rotated to the 16-B chunk phase: byte (x & 3) applies to byte x
    u32 pad;
};

template <int NT, int SF_L, int SF_T>
__global__ __launch_bounds__(SF_T) void ws_segfuse_kernel(unsigned char* __restrict__ buf,
                                                          const u64* __restrict__ seg_off,
                                                          const u64* __restrict__ seg_len, u32 max_frames,
                                                          const u64* __restrict__ desc_base,
                                                          WebsocketFrameDesc_t* __restrict__ desc,
                                                          WebsocketSegResult_t* __restrict__ res, u32 nseg, u32 wsh, u32 ppw) {
    constexpr u32 SF_C = (SF_L - 1) * 64;             // chunks owned per window
    __shared__ __attribute__((aligned(16))) u32x4 win[SF_L * 64];
    __shared__ FrameL tab[SF_TB];
    __shared__ u64 sh_next;                         // next window's first chunk, ~0 = done
    __shared__ u32 sh_flo, sh_fhi;                  // frames with bytes in this window [flo, fhi)
    const u32 s = ws_winn(blockIdx.x, wsh, ppw), tid = threadIdx.x, lane = tid & 63;
    if (s >= nseg) return;                          // the last window's spare blocks
    const u32 wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u64 so = seg_off[s], sl = seg_len[s];
    const uintptr_t segp = reinterpret_cast<uintptr_t>(buf + so);
    const u64 lead = segp & 15, xend = lead + sl;                    // segment bytes: X in [lead, xend)
    gu32x4* const gseg = reinterpret_cast<gu32x4*>(segp & ~(uintptr_t)15);
    const u64 cmax = (sl + lead + WEBSOCKET_BATCH_PAD - 1) >> 4;     // last readable chunk
    const u64 dbase = desc_base ? desc_base[s] : (u64)s * max_frames;
    // wave-0 walk state (wave-uniform)
    u64 off = 0, g = 0;
    u32 nf = 0, nt = 0;
    int status = WEBSOCKET_SEG_OK;
    bool walking = true;
    u64 wc = 0;                                                      // window's first chunk
    for (;;) {
        const u64 W0 = wc << 4, W1 = W0 + (u64)SF_C * 16;
        // ---- 1. LDS-DMA of the window (slices past the readable end are skipped)
        for (u32 i = wv; i < SF_L; i += SF_T / 64) {
            const u64 c0 = wc + (u64)i * 64;
            if (c0 > cmax) break;
            const u64 c = c0 + lane < cmax ? c0 + lane : cmax;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const WS_GLOBAL void*>(gseg + c),
                                             (lds_void*)(&win[i * 64]), 16, 0, NT == 1 || NT == 4 ? 2 : 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // ---- 2. wave 0: headers starting in [W0, W1)
        if (wv == 0) {
            while (walking) {
                const WsRound r = ws_lds_round(win, W0, W1, lead, sl, off, g, nf, max_frames, lane);
                const bool took = lane < r.ntake;
                if (took && r.h.ret != 0) ws_store_desc(desc + dbase + nf + lane, so + r.pos, r.h);
                // every consumed masked frame is unmasked, whatever its (int) return
                const bool mk = took && r.h.masked && r.h.plen;
                const u64 mkm = __ballot(mk);
                if (mk) {
                    FrameL f;
                    f.x0 = r.pos + lead + r.h.hdr;
                    f.x1 = f.x0 + r.h.plen;
                    f.rkey = rotl32(r.h.key, 8u * (u32)(f.x0 & 3));
                    f.pad = 0;
                    tab[nt + (u32)__builtin_popcountll(mkm & ((1ull << lane) - 1))] = f;
                }
                nt += (u32)__builtin_popcountll(mkm);
                if (!ws_round_advance(r, off, g, nf, status, walking)) break;
            }
            // frames with bytes in [W0, W1) (the table is in address order), next window
            const FrameL t = tab[lane];
            const u64 fm = __ballot(lane < nt && t.x0 < W1 && t.x1 > W0);
            const u64 lend = nt ? tab[nt - 1].x1 : 0;                    // only the last frame can pend
            if (lane == 0) {
                sh_flo = fm ? (u32)__builtin_ctzll(fm) : 0u;
                sh_fhi = fm ? 64u - (u32)__builtin_clzll(fm) : 0u;
                sh_next = lend > W1 ? W1 >> 4 : (walking ? (off + lead) >> 4 : ~0ull);
            }
        }
        __syncthreads();
        // ---- 3. XOR + store: wave wv, row u = chunks [u*T + 64*wv, +64) of the window. The
        //         frame table goes to registers once (lane i: frame i, window-relative range
        //         clamped to [-16, window + 16]); a row's frames come from one ballot and are
        //         read back by readlane, so the loop has no LDS round trips.
        constexpr int WB = SF_C * 16;
        const u32 flo = sh_flo, fhi = sh_fhi;
        const FrameL f = tab[lane];
        const long long fa = (long long)(f.x0 - W0), fb = (long long)(f.x1 - W0);
        const int A = (int)(fa < -16 ? -16 : (fa > WB + 16 ? WB + 16 : fa));
        const int B = (int)(fb < -16 ? -16 : (fb > WB + 16 ? WB + 16 : fb));
        const bool fv = lane >= flo && lane < fhi;
        const int xseg0 = (int)(lead > W0 ? lead - W0 : 0);                // segment bytes in the window:
        const int xseg1 = (int)(xend - W0 < (u64)WB ? xend - W0 : (u64)WB); // [xseg0, xseg1)
#pragma unroll
        for (u32 u = 0; u < SF_C / SF_T + 1; ++u) {
            const u32 cb = u * SF_T + 64 * wv;                          // wave-uniform first chunk
            if (cb >= SF_C) break;
            const int r0 = (int)(cb << 4), r1 = r0 + 1024;
            u64 hm = __ballot(fv && A < r1 && B > r0);
            if (!hm) continue;
            const int x = r0 + (int)(lane << 4);
            u32 m0 = 0, m1 = 0, m2 = 0, m3 = 0, cov = 0;
            while (hm) {
                const int i = __builtin_ctzll(hm);
                hm &= hm - 1;
                const int a = __builtin_amdgcn_readlane(A, i), b = __builtin_amdgcn_readlane(B, i);
                const u32 key = (u32)__builtin_amdgcn_readlane((int)f.rkey, i);
                const int lo = a > x ? a - x : 0, hi = b < x + 16 ? b - x : 16;
                if (hi <= lo) continue;
                ws_or_masks(key, lo, hi, m0, m1, m2, m3, cov);
            }
            if (!cov) continue;
            u32x4 w = win[cb + lane];
            w.x ^= m0; w.y ^= m1; w.z ^= m2; w.w ^= m3;
            gu32x4* const pc = gseg + (wc + cb + lane);
            if (x >= xseg0 && x + 16 <= xseg1) {                         // whole chunk inside the segment
                // NT 4: sc1|nt through a descriptor over the wave's 1 KiB row (cfg5 1.386-1.388 ->
                // 1.368-1.373 ms against nt stores, profiles/r04_store_sc1nt_ab.log)
                if constexpr (NT == 4) st16_sc1nt(w, ws_rsrc(reinterpret_cast<uintptr_t>(gseg + (wc + cb)), 1024), lane * 16);
                else st16<NT>(w, pc);
            } else {
                ws_store_bytes(reinterpret_cast<gu8*>(pc), w, cov);
            }
        }
        const u64 nxt = sh_next;
        __syncthreads();                                                     // window LDS is reused
        if (nxt == ~0ull) break;
        wc = nxt;
    }
    if (tid == 0) ws_store_res(res + s, off, nf, status);
}

// 256 threads, 17 KiB windows (8 workgroups per CU). Measured and dropped (round 2): 19 KiB
// windows, 1024 x 65 KiB and 512 x 33 KiB blocks, fewer blocks per CU through unused LDS
// (5 per CU 20 % slower), plain (not nontemporal) loads and stores.
int ws_launch_segfuse(const WsLaunch& L) {
    if (L.max_frames > SF_TB) return ws_set_msg("segfuse path: max_frames > 64");
    const int swin = ws_seg_win;                                         // one read per call
    const WsWinGrid wg = ws_win_grid(L.nseg, swin < 0 ? 2 : swin);
    hipLaunchKernelGGL((ws_segfuse_kernel<4, 18, 256>), dim3(wg.blocks), dim3(256), 0, L.stream, L.buf,
                       L.seg_off, L.seg_len, L.max_frames, L.desc_base, L.desc, L.res, L.nseg, wg.wsh, wg.ppw);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_segfuse_kernel launch", e);
}

// the decode's auto choice between this path and the piece path: many small segments
bool ws_segfuse_fits(u64 span, u32 nseg, u32 max_frames) {
    return max_frames <= SF_TB && nseg >= 1024 && span <= (u64)nseg * ((17u << 10) - 64);
}
