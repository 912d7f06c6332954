// ws_spec.hip — decode path 5 "spec": the reactor loop's chain (net_reactor.c:515-526) is
// PREDICTED per rx segment instead of walked before the unmask, and every unmask block
// checks the prediction on the headers of its own 16 KiB piece (which it has loaded anyway).
//
// Prediction (the regular case — a connection sending equal frames, BASELINE cfg2/cfg4):
// segment s's frames all have the wire length g of its first frame, so frame k starts at
// so + k*g for k < K = min(max_frames, sl / g), and the loop stops at so + K*g (end of the
// segment, max_frames, or an incomplete tail there).
//
// S0 ws_spec_prep_kernel — one thread per segment: the batch-order check (as K1: segments
//    ascending, inside [lo, hi)), the first header -> g, the predicted segment result, and for
//    every 4 KiB region of the batch its first and last segment. Segments shorter than 4 KiB,
//    and those whose first frame cannot seed a prediction, go straight to the repair list, so
//    a region meets at most two predicted segments (its first and its last).
// S1 ws_spec_unmask_kernel — one-shot 256-thread block per 16 KiB piece (two windows, as K2):
//    payload loads first; meanwhile (scalar loads only: lgkmcnt, never behind the payload's
//    vmcnt) the piece's segment records and the header of the frame reaching into the piece
//    from before. Then the piece goes to LDS (+32 B halo), one thread per predicted frame
//    parses its header (websocketframe.c:121-164, ws_parse), writes the descriptor of frames
//    starting in the piece and checks them: every frame must be complete with exactly
//    g = hdr + datalen bytes, and the stop position must parse incomplete. The unmask then
//    applies T_pred: frame k's payload [pos_k + hdr_k, pos_k + g) XOR key_k for every
//    predicted frame whose own header is a complete masked frame of exactly g bytes.
//    A failed check lists the segment for repair (deduplicated per call).
//
// Repair list without resets (so that a captured graph replays correctly): `cnt` only grows;
// S2 leaves `next` = cnt for the following call, whose S0 copies it to `start`; the call's tag
// is start + 1 (never the zeroed workspace's 0); S0 and S1 append at cnt (list is a ring of
// nseg, each call appends <= nseg distinct segments); S2 repairs [start, cnt). brk[s] == tag
// marks s as listed in this call: a tag is written only by a listing, which advances cnt, so
// the next call's tag differs. The disorder word is tagged the same way (S2 advances cnt
// after an out-of-order batch).
// S2 ws_spec_repair_kernel — one wavefront per listed segment: T_pred is an involution
//    computed from bytes it never modifies (the predicted header bytes), so applying it once
//    more restores the wire; then the exact reactor walk (ws_walk.h) decodes the segment.
//    If S0 found the batch out of order, S1 stored nothing and S2 walks every segment.
// Every path result is bit-identical to the reference loop; only the speed depends on the
// prediction. The host falls back to K1+K2 (ws_piece.hip) when the previous call on the
// stream had to repair many segments.
#include "ws_walk.h"

#define SPEC_T 256
#define SPEC_U 4
#define SPEC_SHIFT 14                 // 16 KiB pieces
#define SPEC_RSHIFT 12                // 4 KiB regions: one wavefront each
#define SPEC_GMIN 128                 // smallest predicted stride: <= 34 frames touch one wave's 4 KiB
#define SPEC_NONE 0xFFFFFFFFu

struct SpecRec {                      // per segment, written by S0 (32 B)
    u64 so, sl;
    u32 g;                            // predicted frame wire length; 0: no prediction (S2 walks it)
    u32 K;                            // predicted frames
    u32 stop;                         // 1: the frame at so + K*g must parse incomplete
    u32 pad;
};

typedef __attribute__((address_space(4))) const u64 cu64;
typedef __attribute__((address_space(4))) const u32x4 cu32x4;

struct SpecCtl {                      // workspace head (zeroed when the workspace is allocated)
    u32 disorder;                     // == the call's tag: segments out of order / out of range
    u32 start;                        // cnt when the call began (its tag: start + 1)
    u32 cnt;                          // repair-list appends, ever
    u32 next;                         // the next call's start (written by S2)
};

// list segment s for repair once per call (brk[s] holds the tag of the call that listed it)
__device__ __forceinline__ void spec_list(u32* brk, SpecCtl* ctl, u32* list, u32 nseg, u32 s, u32 tag, u32 undo) {
    if (atomicExch(brk + s, tag) != tag) {
        const u32 i = atomicAdd(&ctl->cnt, 1u);
        list[i % nseg] = s | (undo << 31);
    }
}

__global__ __launch_bounds__(256) void ws_spec_prep_kernel(const unsigned char* __restrict__ buf,
                                                           const u64* __restrict__ seg_off,
                                                           const u64* __restrict__ seg_len, u32 nseg,
                                                           u32 max_frames, SpecRec* __restrict__ rec,
                                                           WebsocketSegResult_t* __restrict__ res,
                                                           u32* __restrict__ rtab, u64 rbase, u64 nreg,
                                                           SpecCtl* __restrict__ ctl, u32* __restrict__ brk,
                                                           u32* __restrict__ list, u64 lo, u64 hi) {
    const u32 s = blockIdx.x * 256 + threadIdx.x;
    if (s >= nseg) return;
    const u32 start = *reinterpret_cast<const volatile u32*>(&ctl->next);  // written by the previous S2
    const u32 tag = start + 1;
    if (s == 0) ctl->start = start;
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    const u64 so = seg_off[s], sl = seg_len[s];
    const u64 prev_end = s ? seg_off[s - 1] + seg_len[s - 1] : 0;
    // out of order, or outside the declared range: S1 stores nothing, S2 walks the batch
    if (prev_end > so || so < lo || so > hi || sl > hi - so) ctl->disorder = tag;
    // region tables (origin-relative 4 KiB regions [rbase, rbase + nreg)):
    //   first[R] = s for regions whose first byte lies in [end of segment s-1, end of segment s)
    //   last[R]  = s for regions whose last byte lies in [start of segment s, start of segment s+1)
    {
        u32* const first = rtab;
        u32* const last = rtab + nreg;
        const u64 a = s ? prev_end + lead0 : 0, b = so + lead0 + sl;
        u64 p = (a + (1ull << SPEC_RSHIFT) - 1) >> SPEC_RSHIFT;
        for (p = p > rbase ? p : rbase; (p << SPEC_RSHIFT) < b && p < rbase + nreg; ++p)
            *gptr<u32>(first + (p - rbase)) = s;
        if (s == nseg - 1)
            for (; p < rbase + nreg; ++p) *gptr<u32>(first + (p - rbase)) = SPEC_NONE;
        const u64 c = so + lead0, d = s + 1 < nseg ? seg_off[s + 1] + lead0 : (hi + lead0 + (1ull << SPEC_RSHIFT));
        // regions R with (R+1)*4096 - 1 in [c, d): R in [ceil((c + 1) / 4096) - 1, ...)
        u64 q = (c + 1 + (1ull << SPEC_RSHIFT) - 1) >> SPEC_RSHIFT;
        q = q ? q - 1 : 0;
        for (q = q > rbase ? q : rbase; ((q + 1) << SPEC_RSHIFT) - 1 < d && q < rbase + nreg; ++q)
            *gptr<u32>(last + (q - rbase)) = s;
        if (s == 0) {                                                    // regions ending before segment 0
            for (u64 t = rbase; t < rbase + nreg && ((t + 1) << SPEC_RSHIFT) - 1 < c; ++t)
                *gptr<u32>(last + (t - rbase)) = SPEC_NONE;
        }
    }
    // the first frame seeds the prediction
    const uintptr_t pa = reinterpret_cast<uintptr_t>(buf + so);
    const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
    u64 h0, h1;
    ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
    const WsHdr h = ws_parse(h0, h1, sl);
    SpecRec r;
    r.so = so; r.sl = sl; r.g = 0; r.K = 0; r.stop = 0; r.pad = 0;
    if (sl < 2 || h.kind == WS_PARSE_INCOMPLETE) {
        ws_store_res(res + s, 0, 0, WEBSOCKET_SEG_OK);                   // the loop stops at once
    } else if (h.kind == WS_PARSE_FRAME && h.ret >= SPEC_GMIN && (u64)h.hdr + h.plen == (u64)(u32)h.ret &&
               sl >= (1ull << SPEC_RSHIFT)) {
        const u32 g = (u32)h.ret;
        const u64 kmax = sl / g;
        const u32 K = kmax < (u64)max_frames ? (u32)kmax : max_frames;
        const u64 consumed = (u64)K * g;
        r.g = g; r.K = K;
        r.stop = K < max_frames && consumed < sl ? 1u : 0u;
        ws_store_res(res + s, consumed, K,
                     K == max_frames && consumed < sl ? WEBSOCKET_SEG_MAX_FRAMES : WEBSOCKET_SEG_OK);
    } else {
        spec_list(brk, ctl, list, nseg, s, tag, 0u);                     // no prediction: S2 walks it
    }
    const u64 w0 = so, w1 = sl, w2 = (u64)r.g | ((u64)r.K << 32), w3 = (u64)r.stop;
    gu32x4* rp = gptr<u32x4>(rec + s);
    u32x4 a, b;
    a.x = (u32)w0; a.y = (u32)(w0 >> 32); a.z = (u32)w1; a.w = (u32)(w1 >> 32);
    b.x = (u32)w2; b.y = (u32)(w2 >> 32); b.z = (u32)w3; b.w = 0;
    rp[0] = a;
    rp[1] = b;
}

// header bytes [p, p+16) (p buf-relative) from 5 scalar dwords at floor4(p)
struct SHdr { u32 w0, w1, w2, w3, w4; };
__device__ __forceinline__ SHdr spec_sload(const unsigned char* p) {
    const cu32* sq = reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    SHdr h;
    h.w0 = sq[0]; h.w1 = sq[1]; h.w2 = sq[2]; h.w3 = sq[3]; h.w4 = sq[4];
    return h;
}
__device__ __forceinline__ void spec_hdr(const SHdr& hw, u32 o, u64& h0, u64& h1) {
    const u64 lo = (u64)hw.w0 | ((u64)hw.w1 << 32), mi = (u64)hw.w2 | ((u64)hw.w3 << 32), hi = hw.w4;
    const u32 sh = 8u * (o & 3);
    h0 = sh ? (lo >> sh) | (mi << (64 - sh)) : lo;
    h1 = sh ? (mi >> sh) | (hi << (64 - sh)) : mi;
}

// T_pred's decision for predicted frame k (header parsed with the loop's avail): XOR its
// payload iff the header is a complete masked frame of exactly g bytes
__device__ __forceinline__ bool spec_xor(const WsHdr& h, u32 g) {
    return h.kind == WS_PARSE_FRAME && (u64)h.hdr + h.plen == (u64)g && h.masked;
}
__device__ __forceinline__ bool spec_ok(const WsHdr& h, u32 g) {
    return h.kind == WS_PARSE_FRAME && (u64)h.hdr + h.plen == (u64)g;
}

// One wavefront's share of a predicted segment: the frames touching the wave's 4 KiB
// [W0, W1) (buf-relative), and where the stop position is checked.
struct SpecSpan {
    u32 ka, nfr, nfx;                  // first frame, frames, frames + the stop check (lanes)
};
__device__ __forceinline__ SpecSpan spec_span(const SpecRec& r, long long W0, long long W1) {
    SpecSpan sp;
    sp.ka = 0; sp.nfr = 0; sp.nfx = 0;
    if (!r.g) return sp;
    const long long so = (long long)r.so, lastb = so + (long long)r.K * r.g;   // end of the predicted frames
    if (W0 > so) {
        const u64 k = (u64)(W0 - so) / r.g;                              // the frame holding W0
        sp.ka = (u32)(k < r.K ? k : r.K);
    }
    const long long bend = W1 < lastb ? W1 : lastb;
    if (sp.ka < r.K && bend > so + (long long)sp.ka * r.g) {
        const u32 kb = (u32)((u64)(bend - 1 - so) / r.g);
        sp.nfr = kb - sp.ka + 1;
    }
    sp.nfx = sp.nfr + (r.stop == 1 && lastb >= W0 && lastb < W1 ? 1u : 0u);
    return sp;
}

__device__ __forceinline__ SpecRec spec_rec(const SpecRec* rec, u32 s) {
    const cu32x4* rp = reinterpret_cast<const cu32x4*>(reinterpret_cast<uintptr_t>(rec + s));
    const u32x4 a = rp[0], b = rp[1];
    SpecRec r;
    r.so = (u64)a.x | ((u64)a.y << 32); r.sl = (u64)a.z | ((u64)a.w << 32);
    r.g = b.x; r.K = b.y; r.stop = b.z; r.pad = 0;
    return r;
}

// One lane's frame: parse, check (frames starting in [W0, W1) are this wave's), descriptor,
// T_pred's payload range (wave-relative, clamped) and key rotated for 16-B chunks.
struct SpecLane { int a, b; u32 rkey; bool bad; };
__device__ __forceinline__ SpecLane spec_lane(long long pos, u64 avail, u32 g, bool stopchk, const u32x4 x0,
                                              const u32x4 x1, long long W0, long long W1, u64 lead0,
                                              WebsocketFrameDesc_t* d) {
    constexpr long long RW = 64 * SPEC_U * 16;
    u64 h0, h1;
    ws_hdr_from32(x0, x1, (u32)(((u64)pos + lead0) & 15), h0, h1);
    const WsHdr h = ws_parse(h0, h1, avail);
    SpecLane L;
    L.a = L.b = 0; L.rkey = 0; L.bad = false;
    if (stopchk) {                                                       // the loop must stop here
        L.bad = h.kind != WS_PARSE_INCOMPLETE;
        return L;
    }
    if (pos >= W0 && pos < W1) {                                         // this wave's frame
        L.bad = !spec_ok(h, g);
        if (!L.bad) ws_store_desc(d, (u64)pos, h);
    }
    const bool x = spec_xor(h, g);
    const long long q0 = pos + h.hdr - W0, q1 = x ? pos + (long long)g - W0 : q0;
    L.a = (int)(q0 < -16 ? -16 : (q0 > RW + 16 ? RW + 16 : q0));
    L.b = (int)(q1 < -16 ? -16 : (q1 > RW + 16 ? RW + 16 : q1));
    L.rkey = rotl32(h.key, 8u * (u32)(((u64)(pos + h.hdr) + lead0) & 3));
    return L;
}

// accumulate the XOR masks of lanes in `hm` (payload ranges a..b, wave-relative) into the
// wave's 4 chunks per lane
__device__ __forceinline__ void spec_masks(u64 hm, int a, int b, u32 rkey, int xl, u32 (&m)[SPEC_U][4],
                                           u32 (&cov)[SPEC_U]) {
    while (hm) {
        const int i = __builtin_ctzll(hm);
        hm &= hm - 1;
        const int ia = __builtin_amdgcn_readlane(a, i), ib = __builtin_amdgcn_readlane(b, i);
        const u32 key = (u32)__builtin_amdgcn_readlane((int)rkey, i);
#pragma unroll
        for (int u = 0; u < SPEC_U; ++u) {
            const int x = u * 1024 + xl;
            const int lo = ia > x ? ia - x : 0, hi = ib < x + 16 ? ib - x : 16;
            if (hi <= lo) continue;
            const u32 bits = (0xFFFFu >> (16 - hi)) & (0xFFFFu << lo);
            cov[u] |= bits;
            m[u][0] |= key & nib_to_bytemask(bits & 15u);
            m[u][1] |= key & nib_to_bytemask((bits >> 4) & 15u);
            m[u][2] |= key & nib_to_bytemask((bits >> 8) & 15u);
            m[u][3] |= key & nib_to_bytemask(bits >> 12);
        }
    }
}

__device__ __forceinline__ void spec_segcov(const SpecRec& r, long long W0, int xl, u32 (&segcov)[SPEC_U]) {
    constexpr long long RW = 64 * SPEC_U * 16;
    const long long sa = (long long)r.so - W0, sb = sa + (long long)r.sl;
    const int SA = (int)(sa < -16 ? -16 : (sa > RW + 16 ? RW + 16 : sa));
    const int SB = (int)(sb < -16 ? -16 : (sb > RW + 16 ? RW + 16 : sb));
#pragma unroll
    for (int u = 0; u < SPEC_U; ++u) {
        const int x = u * 1024 + xl;
        const int lo = SA > x ? (SA - x < 16 ? SA - x : 16) : 0;
        const int hi = SB > x ? (SB - x < 16 ? SB - x : 16) : 0;
        if (hi > lo) segcov[u] |= (0xFFFFu >> (16 - hi)) & (0xFFFFu << lo);
    }
}

// S1: one-shot 256-thread block per 16 KiB piece; every wavefront works alone on its 4 KiB
// region (no LDS, no barrier): payload loads; by scalar loads the region's first and last
// segment and their records (every segment between them is shorter than the region: S0 listed
// it for S2); then, behind the payload in the same load queue, the 32-B header windows of the
// predicted frames touching the region (lane t: frame t; <= 34 frames of >= 128 B, + the two
// stop checks); masks from the lanes' parsed headers (ballot + readlane, as K2's items); stores.
template <int NT>
__global__ __launch_bounds__(SPEC_T) void ws_spec_unmask_kernel(
    unsigned char* __restrict__ buf, const u64* __restrict__ desc_base, WebsocketFrameDesc_t* __restrict__ desc,
    u32 nseg, u32 max_frames, const SpecRec* __restrict__ rec, const u32* __restrict__ rtab, u64 rbase, u64 nreg,
    SpecCtl* __restrict__ ctl, u32* __restrict__ brk, u32* __restrict__ list, u64 pbase, u64 c_lo, u64 c_hi,
    u32 wshift, u64 ppw, u64 npieces) {
    constexpr long long RW = 64 * SPEC_U * 16;
    const u32 tid = threadIdx.x, lane = tid & 63;
    const u32 wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 bx = blockIdx.x;
    const u64 pw = (u64)(bx & ((1u << wshift) - 1u)) * ppw + (bx >> wshift);      // windows side by side
    const bool pvalid = pw < npieces;
    const u64 pidx = pvalid ? pw : npieces - 1;
    const u64 pc0 = (pbase + pidx) << (SPEC_SHIFT - 4);
    const u64 wc0 = pc0 + (u64)wv * (64 * SPEC_U);
    gu32x4* const base = reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(buf) & ~(uintptr_t)15);
    // ---- 1. payload loads (clamped to the batch's chunks)
    u32x4 v[SPEC_U];
#pragma unroll
    for (int u = 0; u < SPEC_U; ++u) {
        const u64 c = wc0 + (u64)(u * 64 + lane);
        v[u] = ld16<NT>(base + (c < c_lo ? c_lo : (c < c_hi ? c : c_hi - 1)));
    }
    // ---- 2. scalar: the region's first and last segment, their records
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    const u64 reg = wc0 >> (SPEC_RSHIFT - 4);                            // origin-relative region index
    const long long W0 = (long long)(wc0 << 4) - (long long)lead0;        // this wave's 4 KiB, buf-relative
    const long long W1 = W0 + RW;
    const u32 tag = *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(&ctl->start)) + 1;
    const u32 dis = *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(&ctl->disorder)) == tag;
    const bool rvalid = pvalid && !dis && reg >= rbase && reg < rbase + nreg;
    const u32 sa = rvalid ? *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(rtab + (reg - rbase))) : SPEC_NONE;
    const u32 sb = rvalid ? *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(rtab + nreg + (reg - rbase))) : SPEC_NONE;
    SpecRec r0, r1;
    r0.so = r1.so = 0; r0.sl = r1.sl = 0; r0.g = r1.g = 0; r0.K = r1.K = 0; r0.stop = r1.stop = 0; r0.pad = r1.pad = 0;
    const bool havea = sa < nseg, haveb = sb < nseg && sb != sa;
    if (havea) r0 = spec_rec(rec, sa);
    if (haveb) r1 = spec_rec(rec, sb);
    // a segment ending at or before W0 (the region may lie in a gap) takes no part
    const bool ina = havea && (long long)r0.so < W1 && (long long)(r0.so + r0.sl) > W0;
    const bool inb = haveb && (long long)r1.so < W1 && (long long)(r1.so + r1.sl) > W0;
    const SpecSpan p0 = ina ? spec_span(r0, W0, W1) : SpecSpan{0, 0, 0};
    const SpecSpan p1 = inb ? spec_span(r1, W0, W1) : SpecSpan{0, 0, 0};
    // ---- 3. header windows of the frames touching this 4 KiB: lane t < p0.nfx segment a, then b
    const u32 n01 = p0.nfx + p1.nfx;                                     // <= 36: frames >= 128 B are disjoint
    const bool ls0 = lane < p0.nfx, ls1 = !ls0 && lane < n01;
    const u32 kk = ls0 ? p0.ka + lane : (ls1 ? p1.ka + (lane - p0.nfx) : 0u);
    const u64 hp = ls0 ? r0.so + (u64)kk * r0.g : (ls1 ? r1.so + (u64)kk * r1.g : (u64)(W0 > 0 ? W0 : 0));
    const gu32x4* hq = reinterpret_cast<const gu32x4*>((reinterpret_cast<uintptr_t>(buf) + hp) & ~(uintptr_t)15);
    const u32x4 x0 = hq[0], x1 = hq[1];                                  // + WEBSOCKET_BATCH_PAD: readable
    u32 m[SPEC_U][4], cov[SPEC_U], segcov[SPEC_U];
#pragma unroll
    for (int u = 0; u < SPEC_U; ++u) { m[u][0] = m[u][1] = m[u][2] = m[u][3] = 0; cov[u] = 0; segcov[u] = 0; }
    const int xl = (int)lane * 16;
    if (ina) spec_segcov(r0, W0, xl, segcov);
    if (inb) spec_segcov(r1, W0, xl, segcov);
    // ---- 4. parse, check, descriptors, masks
    {
        const u32 s = ls0 ? sa : sb;
        const bool stopchk = ls0 ? lane == p0.nfr : (ls1 && lane - p0.nfx == p1.nfr);
        const u64 avail = ls0 ? r0.sl - (u64)kk * r0.g : r1.sl - (u64)kk * r1.g;
        const u32 g = ls0 ? r0.g : r1.g;
        SpecLane L;
        L.a = L.b = 0; L.rkey = 0; L.bad = false;
        if (ls0 || ls1) {
            const u64 dbase = desc_base ? desc_base[s] : (u64)s * max_frames;
            L = spec_lane((long long)hp, avail, g, stopchk, x0, x1, W0, W1, lead0, desc + dbase + kk);
        }
        if (L.bad) spec_list(brk, ctl, list, nseg, s, tag, 1u);            // S2: undo T_pred, then walk
        spec_masks(__ballot((ls0 || ls1) && !stopchk && L.a < L.b && L.b > 0 && L.a < (int)RW), L.a, L.b, L.rkey, xl,
                   m, cov);
    }
    // ---- 5. stores: chunks inside segments whole (unchanged bytes written back), others exact
    if (pvalid && !dis) {
#pragma unroll
        for (int u = 0; u < SPEC_U; ++u) {
            const u64 c = wc0 + (u64)(u * 64 + lane);
            if (!cov[u] || c < c_lo || c >= c_hi) continue;
            u32x4 w = v[u];
            w.x ^= m[u][0]; w.y ^= m[u][1]; w.z ^= m[u][2]; w.w ^= m[u][3];
            if (cov[u] == 0xFFFFu || segcov[u] == 0xFFFFu) st16<NT>(w, base + c);
            else ws_store_bytes(reinterpret_cast<gu8*>(base + c), w, cov[u]);
        }
    }
}

// S2: one wavefront per listed segment (or per segment when the batch is out of order)
template <int NT>
__global__ __launch_bounds__(256) void ws_spec_repair_kernel(
    unsigned char* __restrict__ buf, const u64* __restrict__ seg_off, const u64* __restrict__ seg_len, u32 nseg,
    u32 max_frames, const u64* __restrict__ desc_base, WebsocketFrameDesc_t* __restrict__ desc,
    WebsocketSegResult_t* __restrict__ res, const SpecRec* __restrict__ rec, SpecCtl* __restrict__ ctl,
    const u32* __restrict__ list, u32* __restrict__ host_cnt) {
    const u32 lane = threadIdx.x & 63;
    const u32 w = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    const u32 start = *reinterpret_cast<const volatile u32*>(&ctl->start), tag = start + 1;
    const u32 dis = *reinterpret_cast<const volatile u32*>(&ctl->disorder) == tag;
    const u32 cnt = *reinterpret_cast<const volatile u32*>(&ctl->cnt);   // nothing appends during S2
    const u32 n = cnt - start;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (host_cnt) *reinterpret_cast<volatile u32*>(host_cnt) = dis ? nseg : n;
        // the next call's start; after an out-of-order batch one more, so its tag differs
        ctl->next = cnt + dis;
        if (dis) ctl->cnt = cnt + 1;
    }
    if (dis) {                                                           // S1 stored nothing
        for (u32 s = w; s < nseg; s += nw)
            walk_segment<4, NT>(buf, s, seg_off, seg_len, max_frames, desc_base, desc, res, lane);
        return;
    }
    for (u32 i = w; i < n && i < nseg; i += nw) {
        const u32 e = list[(start + i) % nseg], s = e & 0x7FFFFFFFu;
        if (s >= nseg) continue;                                         // (never: defensive)
        if (e >> 31) {                                                    // undo T_pred
            const SpecRec r = rec[s];
            for (u32 k = 0; k < r.K; ++k) {
                const u64 pos = r.so + (u64)k * r.g;
                const uintptr_t pa = reinterpret_cast<uintptr_t>(buf + pos);
                const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
                u64 h0, h1;
                ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
                const WsHdr h = ws_parse(h0, h1, r.sl - (u64)k * r.g);
                if (spec_xor(h, r.g)) unmask_payload<4, NT>(buf + pos + h.hdr, buf + pos + r.g, h.key, lane);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");             // restored bytes in L2 first
        }
        walk_segment_vload<4, NT>(buf, s, seg_off, seg_len, max_frames, desc_base, desc, res, lane);
    }
}

// ---------------------------------------------------------------------------------------------
// host side
size_t ws_spec_workspace_bytes(u64 span, u32 nseg) {
    const u64 nreg = (span + 15) / (1ull << SPEC_RSHIFT) + 2;
    size_t b = 256;                                                      // SpecCtl
    b = (b + nreg * 8 + 255) & ~(size_t)255;                             // region first/last tables
    b += (size_t)nseg * sizeof(SpecRec);                                 // records
    b += (size_t)nseg * 8;                                               // brk + list
    return b + 256;
}

// S0 + S1 + S2 over a batch whose segments lie in [lo, hi) of L.buf. `ws` is the stream's
// path 5 workspace (zeroed whole when allocated, used by nothing else); host_cnt (optional,
// device view of host-mapped memory): S2 stores how many segments it repaired, which the
// host reads to choose the next call's path.
int ws_launch_spec(const WsLaunch& L, u64 lo, u64 hi, int nt, unsigned char* ws, u32* host_cnt) {
    const u64 lead0 = reinterpret_cast<uintptr_t>(L.buf) & 15;
    const u64 lo_org = lo + lead0, hi_org = hi + lead0;
    const u64 npieces = hi_org > lo_org ? ((hi_org - 1) >> SPEC_SHIFT) - (lo_org >> SPEC_SHIFT) + 1 : 0;
    const u64 pbase = lo_org >> SPEC_SHIFT;
    const u64 c_lo = lo_org >> 4, c_hi = (hi_org + 15) >> 4;
    const u64 nreg = hi_org > lo_org ? ((hi_org - 1) >> SPEC_RSHIFT) - (lo_org >> SPEC_RSHIFT) + 1 : 0;
    const u64 rbase = lo_org >> SPEC_RSHIFT;
    SpecCtl* ctl = reinterpret_cast<SpecCtl*>(ws);
    size_t b = 256;
    u32* rtab = reinterpret_cast<u32*>(ws + b);
    b = (b + nreg * 8 + 255) & ~(size_t)255;
    SpecRec* rec = reinterpret_cast<SpecRec*>(ws + b);
    b += (size_t)L.nseg * sizeof(SpecRec);
    u32* brk = reinterpret_cast<u32*>(ws + b);
    u32* list = brk + L.nseg;
    hipLaunchKernelGGL(ws_spec_prep_kernel, dim3((L.nseg + 255) / 256), dim3(256), 0, L.stream, L.buf, L.seg_off,
                       L.seg_len, L.nseg, L.max_frames, rec, L.res, rtab, rbase, nreg, ctl, brk, list, lo, hi);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ws_set_err("ws_spec_prep_kernel launch", e);
    if (npieces) {
        const u32 wshift = npieces >= 512 ? 1u : 0u;                     // two windows half a batch apart (K2)
        const u64 ppw = (npieces + (1ull << wshift) - 1) >> wshift;
        auto k = nt == 1 ? ws_spec_unmask_kernel<1> : ws_spec_unmask_kernel<0>;
        hipLaunchKernelGGL(k, dim3((u32)(ppw << wshift)), dim3(SPEC_T), 0, L.stream, L.buf, L.desc_base, L.desc, L.nseg,
                           L.max_frames, rec, rtab, rbase, nreg, ctl, brk, list, pbase, c_lo, c_hi, wshift, ppw,
                           npieces);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_spec_unmask_kernel launch", e);
    }
    auto kr = nt == 1 ? ws_spec_repair_kernel<1> : ws_spec_repair_kernel<0>;
    const u32 rblocks = L.nseg < 1024 * 4 ? (L.nseg + 3) / 4 : 1024;
    hipLaunchKernelGGL(kr, dim3(rblocks), dim3(256), 0, L.stream, L.buf, L.seg_off, L.seg_len, L.nseg, L.max_frames,
                       L.desc_base, L.desc, L.res, rec, ctl, list, host_cnt);
    if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_spec_repair_kernel launch", e);
    return 0;
}
