// ws_spec.hip — decode path 3, speculative form: the unmask kernel finds its own frames.
//
// The classic piece path (ws_piece.hip) runs K1, a walk over every frame header
// (net_reactor.c:515-526 over websocketframe.c:112-165), and only then K2, the one-shot
// unmask over 16 KiB pieces. K1's ~1 M scattered header lines (40 µs on cfg2) sit on the
// critical path in front of K2. Here there is no K1:
//
// S1 ws_piece_spec_kernel — one 256-thread block per 16 KiB piece (K2's block shape,
//   windows and stores). Each wave issues its payload loads, then finds the segments
//   under its 4 KiB range (an interpolation guess checked by two scalar loads) and
//   predicts every segment as frames of ONE wire length g back to back from its start —
//   g is the host's hint: the first frame length the previous call on the stream saw.
//   Per predicted frame k at so + k*g the wave checks the header against the header
//   signature of a complete frame of length g (host-computed: for each length form and
//   MASK bit, the expected byte 1 / extended length, websocketframe.c:126-150) — a
//   scalar load and a few compares — and XORs the payload of every frame that matches
//   with its key. The wave holding a header verifies it for the segment (a mismatch,
//   or after the last predicted frame a header that is not incomplete, flags the
//   segment: one atomicOr, the first flagger lists it) and writes its descriptor; the
//   wave holding the segment's first byte writes the predicted segment result. The first
//   `nchk` waves also check the segment table (ascending, inside [lo, hi)); the last of
//   them publishes the verdict into replicated words, which every wave polls (relaxed,
//   bounded) before its stores: an unordered batch stores nothing, a wave that gives up
//   waiting stores nothing, tags its range and flags its segments (results never depend
//   on dispatch order, only speed does).
// S2 ws_piece_spec_fix_kernel — tiny unless something was flagged: unordered batch ->
//   every segment walked exactly; flagged segments -> the speculative XOR undone (XOR is
//   an involution; the same rule over the same header bytes) on the ranges that stored,
//   then walked exactly (net_reactor.c:515-526 over websocketframeDecode).
//
// Why the speculation is race-free: for predicted frame k at pos = so + k*g the rule is
// "the header matches the signature of form (byte 1) and MASK: XOR [pos + hdr, pos + g)
// with its key". A form whose header would be longer than g never matches (decided from
// byte 1 alone); otherwise every byte the rule reads lies in [pos, pos + hdr) — outside
// every XOR range — so all waves (and S2's undo) read the original bytes whatever has
// been stored. A matching header is a complete frame of total length g (websocketframe.c
// :149 with avail >= g; g < 2^31, no wrap), so the rule is the reference's unmask
// (:153-158) and the descriptor its out-params.
//
// State (per workspace slot, parity-double-buffered, see ws_api.hip): head words
// {ctr, nmis, tmo} and the verdict words rest at zero; S2 of call i zeroes those of call
// i + 1 and clears the flags it consumed. Not used inside HIP graph captures.
#include "ws_walk.h"

#define SPEC_T 256
#define SPEC_U WS_PIECE_U
#define SPEC_SHIFT WS_PIECE_SHIFT
#define SPEC_FAST_G 2048                    // fast path: at most 3 frames touch a wave's range
#define SPEC_RANGE_SHIFT (SPEC_SHIFT - 2)   // one wave's range: 64 lanes x SPEC_U x 16 B = 4 KiB
static_assert((1 << SPEC_RANGE_SHIFT) == 64 * SPEC_U * 16, "wave range");
// bounded wait for the checkers (s_sleep 2 + a load each): option "spec_spins" (0 = give up
// unless the first poll finds them done: exercises the repair path in tests)
WsOpt ws_spec_spins{2048};

enum { SPEC_CTR = 0, SPEC_NMIS = 1, SPEC_TMO = 2, SPEC_HEAD_WORDS = 4 };
// the checkers' verdict, published by the last checker into SPEC_REPL words SPEC_REPL_STRIDE
// bytes apart (every wave polls one of them: one word polled by a million waves is a memory
// hot spot): 0 not yet, 1 ordered, 2 unordered
#define SPEC_REPL 64
#define SPEC_REPL_STRIDE 1024

// The header signature of a complete frame of wire length g (host-computed, by value): per
// MASK bit m, what byte 1 and the extended length must hold (websocketframe.c:126-150).
struct SpecSig {
    u32 g;
    u32 b1[2];        // 7-bit form: byte 1 exactly (0x100: g does not fit this form)
    u32 e16[2];       // 16-bit form: bytes 2-3 read little-endian (0x10000: impossible)
    u32 ok64[2];      // the 64-bit form is possible (g >= 10 + 4m)
    float rg;         // 1.0f / g
    float gs;         // segments per 256 bytes of the batch (the table guess)
    u64 e64[2];       // 64-bit form: bytes 2-9 read little-endian
    // g >= SPEC_FAST_G: the masked frame in its shortest form (16- or 64-bit length) as masked
    // compares of the header's first three dwords; the key at dword 1 (16-bit) or bytes 10-13
    u32 fm[3], fe[3];
    u32 f64, fhdr;
};

static SpecSig spec_sig(u32 g) {
    SpecSig S;
    S.g = g;
    S.rg = 1.0f / (float)g;
    for (u32 m = 0; m < 2; ++m) {
        const u32 h7 = 2 + 4 * m, h16 = 4 + 4 * m, h64 = 10 + 4 * m;
        S.b1[m] = g >= h7 && g - h7 < 126 ? ((m << 7) | (g - h7)) : 0x100u;
        S.e16[m] = g >= h16 && g - h16 <= 0xFFFF ? (((g - h16) >> 8) | (((g - h16) & 0xFFu) << 8)) : 0x10000u;
        S.ok64[m] = g >= h64;
        S.e64[m] = g >= h64 ? __builtin_bswap64((u64)(g - h64)) : 0;
    }
    S.f64 = g - 8 > 0xFFFFu;
    S.fhdr = S.f64 ? 14 : 8;
    const u64 len = g - S.fhdr;
    S.fm[0] = 0xFFFFFF00u;
    if (!S.f64) {
        S.fe[0] = 0xFE00u | (u32)((len >> 8) & 0xFF) << 16 | (u32)(len & 0xFF) << 24;
        S.fm[1] = S.fe[1] = S.fm[2] = S.fe[2] = 0;
    } else {
        const u64 be = __builtin_bswap64(len);          // bytes 2-9 in wire order
        S.fe[0] = 0xFF00u | (u32)(be & 0xFFFF) << 16;
        S.fm[1] = 0xFFFFFFFFu;
        S.fe[1] = (u32)(be >> 16);
        S.fm[2] = 0xFFFFu;
        S.fe[2] = (u32)(be >> 48);
    }
    return S;
}

// The frame at a predicted position: header bytes 0..15 as w0, w1 (little-endian, uniform).
// true: a complete frame of length g — hdr, masked, key (wire order) set.
__device__ __forceinline__ bool spec_match(u64 w0, u64 w1, const SpecSig& S, u32& hdr, u32& masked, u32& key) {
    const u32 b1 = (u32)(w0 >> 8) & 0xFFu, m = b1 >> 7, p7 = b1 & 0x7Fu;
    masked = m;
    if (p7 < 126) {
        hdr = 2 + 4 * m;
        key = (u32)(w0 >> 16);
        return b1 == S.b1[m];
    }
    if (p7 == 126) {
        hdr = 4 + 4 * m;
        key = (u32)(w0 >> 32);
        return ((u32)(w0 >> 16) & 0xFFFFu) == S.e16[m];
    }
    hdr = 10 + 4 * m;
    key = (u32)(w1 >> 16);
    return S.ok64[m] && ((w0 >> 16) | (w1 << 48)) == S.e64[m];
}

__device__ __forceinline__ u32 ld_agent(u32* p) {
    return __hip_atomic_load(gptr<u32>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// P = the number of segments whose offset is <= a, for ascending offsets (the segment
// holding byte a, if any, is P - 1): a 64-entry window around the guess, then 64-ary
// narrowing. Bounded on any input.
__device__ __forceinline__ u32 spec_count_le(const u64* __restrict__ seg_off, u32 nseg, u64 a, u32 guess, u32 lane) {
    u32 lo = 0, hi = nseg;                       // off[s] <= a below lo, > a from hi (ascending input)
    {
        u32 w0 = guess > 31 ? guess - 31 : 0;
        if (w0 + 64 > nseg) w0 = nseg > 64 ? nseg - 64 : 0;
        const u32 nv = nseg - w0 < 64 ? nseg - w0 : 64;
        const u32 i = w0 + (lane < nv ? lane : nv - 1);
        const u32 k = (u32)__popcll(__ballot(lane < nv && seg_off[i] <= a));
        if (k > 0 && k < nv) return w0 + k;
        if (k == 0) {
            if (w0 == 0) return 0;
            hi = w0;
        } else {
            if (w0 + nv == nseg) return nseg;
            lo = w0 + nv;
        }
    }
    while (hi - lo > 64) {
        const u32 step = (hi - lo) / 65;         // probes lo + step .. lo + 64 step, all < hi
        const u32 k = (u32)__popcll(__ballot(seg_off[lo + (lane + 1) * step] <= a));
        const u32 nlo = k ? lo + k * step + 1 : lo;
        hi = k < 64 ? lo + (k + 1) * step : hi;
        lo = nlo;
    }
    const u32 i = lo + lane;
    return lo + (u32)__popcll(__ballot(i < hi && seg_off[i < nseg ? i : nseg - 1] <= a));
}

// a wave-uniform value the compiler cannot prove uniform (e.g. computed in VALU): back to SGPRs
__device__ __forceinline__ u64 uni64(u64 x) {
    return (u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)x) |
           ((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)(x >> 32)) << 32);
}
__device__ __forceinline__ u32 uni32(u32 x) { return (u32)__builtin_amdgcn_readfirstlane((int)x); }

// floor(x / g), wave-uniform, 2 <= g < 2^31, rg = 1.0f / g: an f32 estimate and at most two
// corrections when x < 2^32 and the quotient < 2^20 (every frame count in practice), the
// 64-bit division otherwise
__device__ __forceinline__ u64 spec_div(u64 x, u64 g, float rg) {
    if ((x >> 32) == 0 && x < (g << 20)) {
        const u32 xx = (u32)x, dd = (u32)g;
        u32 q = uni32((u32)((float)xx * rg));
        long long r = (long long)xx - (long long)q * dd;
        if (r < 0) { --q; r += dd; }
        if (r < 0) { --q; r += dd; }
        if (r >= (long long)dd) { ++q; r -= dd; }
        if (r >= (long long)dd) { ++q; r -= dd; }
        if (r >= 0 && r < (long long)dd) return q;
    }
    return uni64(x / g);
}

// wave-uniform loads through the scalar path (lgkmcnt: they do not wait behind the wave's
// payload loads, which vmcnt retires in order)
typedef __attribute__((address_space(4))) const u64 cu64;
__device__ __forceinline__ u64 sld64(const u64* p) { return *reinterpret_cast<cu64*>(reinterpret_cast<uintptr_t>(p)); }

// header bytes [p, p + 16) by vector loads (WEBSOCKET_BATCH_PAD makes the 32 B readable)
__device__ __forceinline__ void spec_words_v(const unsigned char* p, u64& w0, u64& w1) {
    const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
    const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
    ws_hdr_from32(q[0], q[1], (u32)(pa & 15), w0, w1);
}

// header bytes [p, p + 16) (wave-uniform p) by scalar loads: S1 never changes header bytes
__device__ __forceinline__ void spec_words_s(uintptr_t p, u64& w0, u64& w1) {
    const HdrWords hw = load_header(reinterpret_cast<const unsigned char*>(p));
    const u64 lo = (u64)hw.w0 | ((u64)hw.w1 << 32), mi = (u64)hw.w2 | ((u64)hw.w3 << 32), hi = (u64)hw.w4;
    const u32 sh = 8u * (u32)(p & 3);
    w0 = sh ? (lo >> sh) | (mi << (64 - sh)) : lo;
    w1 = sh ? (mi >> sh) | (hi << (64 - sh)) : mi;
}

__device__ __forceinline__ void spec_flag(u32* flags, u32* list, u32* head, u32 s) {
    const u32 old = __hip_atomic_fetch_or(gptr<u32>(flags + s), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!old) {
        const u32 i = __hip_atomic_fetch_add(gptr<u32>(head + SPEC_NMIS), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *gptr<u32>(list + i) = s;
    }
}

// descriptor of a matched frame (the out-params websocketframeDecode gives it)
__device__ __forceinline__ void spec_store_desc(WebsocketFrameDesc_t* d, u64 pos, u32 b0, u32 hdr, u32 masked, u32 g) {
    const u64 plen = g - hdr;
    const u64 dof = plen ? pos + hdr : WEBSOCKET_DATA_OFF_NULL;
    u32x4 q0, q1;
    q0.x = (u32)pos; q0.y = (u32)(pos >> 32); q0.z = (u32)dof; q0.w = (u32)(dof >> 32);
    q1.x = (u32)plen; q1.y = 0; q1.z = g;
    q1.w = (b0 >> 7) | ((b0 & 0x0Fu) << 8) | (masked << 16) | (hdr << 24);
    gu32x4* gd = gptr<u32x4>(d);
    gd[0] = q0;
    gd[1] = q1;
}

// XOR frame payload bytes [a, b) of this wave's range (range-relative, clamped to [-16, RW + 16],
// uniform) with `key` (rotated to the 16-B chunk phase): rows wholly inside take four XORs, only
// edge rows work out per-lane byte bounds. cov: the payload bytes of each lane's chunk.
__device__ __forceinline__ void spec_xor_rows(u32x4 (&v)[SPEC_U], u32 (&cov)[SPEC_U], int a, int b, u32 key, int xl) {
#pragma unroll
    for (int u = 0; u < SPEC_U; ++u) {
        if (b <= u * 1024 || a >= u * 1024 + 1024) continue;                // (uniform) not in row u
        if (a <= u * 1024 && b >= u * 1024 + 1024) {                        // (uniform) the whole row
            v[u].x ^= key; v[u].y ^= key; v[u].z ^= key; v[u].w ^= key;
            cov[u] = 0xFFFFu;
            continue;
        }
        const int xx = u * 1024 + xl;
        const int l2 = a > xx ? a - xx : 0, h2 = b < xx + 16 ? b - xx : 16;
        if (h2 > l2) ws_xor_range(key, l2, h2, v[u], cov[u]);
    }
}

template <int NT>
__global__ __launch_bounds__(SPEC_T) void ws_piece_spec_kernel(
    unsigned char* __restrict__ buf, const u64* __restrict__ seg_off, const u64* __restrict__ seg_len, u32 nseg,
    u32 max_frames, const u64* __restrict__ desc_base, WebsocketFrameDesc_t* __restrict__ desc,
    WebsocketSegResult_t* __restrict__ res, u32* head, u32* done, u32* flags, u32* list, u32* marks, u32 tag,
    u64 pbase, u64 c_lo, u64 c_hi, u64 lo, u64 hi, u64 ppw, u64 npieces, u32 wshift, u32 nchk, u32 chk_per,
    u32 spins, SpecSig S) {
    const u32 tid = threadIdx.x, lane = tid & 63;
    const u32 wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 bx = blockIdx.x;
    // block -> piece: two windows half a batch apart (as K2, ws_piece.hip)
    const u64 pw = (u64)(bx & ((1u << wshift) - 1u)) * ppw + (bx >> wshift);
    const bool pvalid = pw < npieces;
    const u64 pidx = pvalid ? pw : npieces - 1;
    const u64 wc0 = ((pbase + pidx) << (SPEC_SHIFT - 4)) + (u64)wv * (64 * SPEC_U);
    // ---- 1. payload loads: chunk rel = u * 64 + lane of the wave's 256, clamped into the batch's
    //         chunks [c_lo, c_hi) as med3(rel, A, B) (A <= B; only a batch's edge waves clamp)
    int A, B;
    {
        const long long dlo = (long long)(c_lo - wc0), dhi = (long long)(c_hi - 1 - wc0);
        const long long a0 = dhi < 0 ? dhi : 0, b0 = dlo > 255 ? dlo : 255;
        A = (int)(dlo > a0 ? dlo : a0);
        B = (int)(dhi < b0 ? dhi : b0);
    }
    const uintptr_t sbase = (reinterpret_cast<uintptr_t>(buf) & ~(uintptr_t)15) + (wc0 << 4) + (uintptr_t)(long long)A * 16;
    u32x4 v[SPEC_U];
#pragma unroll
    for (int u = 0; u < SPEC_U; ++u) {
        const int rel = u * 64 + (int)lane;
        const int rc = rel < A ? A : (rel > B ? B : rel);
        v[u] = ld16<NT>(reinterpret_cast<gu32x4*>(sbase + (u32)((rc - A) * 16)));
    }
    const u32 gw = bx * (SPEC_T / 64) + wv;
    u32* const myrepl = done + (gw % SPEC_REPL) * (SPEC_REPL_STRIDE / 4);
    // the checkers' verdict, polled now so the load is back by the stores (a wave that finds
    // it not published yet polls again there)
    u32 verdict = lane == 0 ? ld_agent(myrepl) : 0u;
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    constexpr long long RW = 64 * SPEC_U * 16;                              // this wave's bytes
    const u64 r0 = wc0 << 4, r1 = r0 + RW;                                  // origin-relative
    const u64 ra = r0 > lead0 ? r0 - lead0 : 0, rb = r1 - lead0;            // buffer-relative
    // ---- 2. the segment holding ra: a guess from the batch's extent (kernel arguments), checked
    //         by the four table entries of it and its successor, loaded at once
    u32 guess = 0;
    if (nseg > 2 && ra > lo) {
        const float f = (float)(u32)((ra - lo) >> 8) * S.gs;
        guess = uni32(f < (float)(nseg - 2) ? (u32)f : nseg - 2);
    }
    const u32 g1 = nseg > 1 ? guess + 1 : guess;
    const u64 o0 = pvalid ? sld64(seg_off + guess) : 0, o1 = pvalid ? sld64(seg_off + g1) : 0;
    const u64 l0 = pvalid ? sld64(seg_len + guess) : 0, l1 = pvalid ? sld64(seg_len + g1) : 0;
    // ---- 3. checker duty (the first nchk waves): the segment table is ascending and inside
    //         [lo, hi) (the piece decomposition assumes it); zero-length results written here
    if (gw < nchk) {
        const u64 s_beg = (u64)gw * chk_per;
        const u64 s_end = s_beg + chk_per < nseg ? s_beg + chk_per : nseg;
        bool bad = false;
        for (u64 sb = s_beg; sb < s_end; sb += 64) {
            const u64 s = sb + lane;
            if (s < s_end) {
                const u64 so = seg_off[s], sl = seg_len[s];
                const u64 pe = s ? seg_off[s - 1] + seg_len[s - 1] : 0;
                bad |= pe > so || so < lo || so > hi || sl > hi - so;
                if (sl == 0) ws_store_res(res + s, 0, 0, WEBSOCKET_SEG_OK);
            }
        }
        const bool any = __ballot(bad) != 0;
        u32 old = 0;
        if (lane == 0)
            old = __hip_atomic_fetch_add(gptr<u32>(head + SPEC_CTR), 1u + (any ? 0x10000u : 0u), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        old = (u32)__builtin_amdgcn_readlane((int)old, 0);
        if ((old & 0xFFFFu) + 1 == nchk) {       // the last checker publishes the verdict
            const u32 vd = ((old >> 16) || any) ? 2u : 1u;
            __hip_atomic_store(gptr<u32>(done + lane * (SPEC_REPL_STRIDE / 4)), vd, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    const int xl = (int)lane * 16;
    const u64 g = S.g;
    u32 cov[SPEC_U], segcov[SPEC_U];
#pragma unroll
    for (int u = 0; u < SPEC_U; ++u) { cov[u] = 0; segcov[u] = 0; }
    bool allseg = false;                                                    // one segment covers the range
    u32 s_first = 0, s_stop = 0;                                            // segments visited [s_first, s_stop)
    if (pvalid) {
        u32 s;
        bool hit = true;                         // s is guess or g1: its entries (and the next) are loaded
        if (o0 <= ra && (ra < o1 || nseg == 1)) s = guess;
        else if (guess == 0 && ra < o0) s = 0;
        else if (nseg > 1 && o1 <= ra && g1 + 1 == nseg) { s = g1; hit = false; }
        else {
            const u32 P = spec_count_le(seg_off, nseg, ra, guess, lane);
            s = P ? P - 1 : 0;
            hit = false;
        }
        s_first = s;
        bool fast = false;
        if (g >= SPEC_FAST_G) {
            // ---- 3a. fast path: one segment covers the range and every frame that touches it
            //          is a predicted frame (the frames fit in scalar registers, each lane
            //          picks its chunk's frame by two compares)
            const u64 so = hit ? o0 : sld64(seg_off + s), sl = hit ? l0 : sld64(seg_len + s);
            const long long sa = (long long)(so + lead0) - (long long)r0, send = sa + (long long)sl;
            if (sa < 0 && sa > -(1ll << 31) && send > 0 && so <= hi && sl <= hi - so) {
                const u32 x = (u32)(-sa), gg = (u32)g;
                u32 kA = uni32((u32)((float)x * S.rg)), t = kA * gg;     // f32 estimate, off by <= 1
                if (t > x) { --kA; t -= gg; }
                else if (x - t >= gg) { ++kA; t += gg; }
                const int F0 = (int)t - (int)x;                                    // (-g, 0]
                const int nfr = 1 + (F0 + (int)gg < (int)RW) + (F0 + 2 * (int)gg < (int)RW);
                const long long fend = (long long)F0 + (long long)nfr * gg;          // end of the last frame
                u32 jb = 3, nfull2 = 0;                 // frames j >= jb belong to segment s + 1
                u64 so2 = 0, sl2 = 0;
                if (send >= RW) {                       // one segment covers the range
                    fast = kA + (u32)nfr <= max_frames && fend <= send;
                } else if (s + 1 < nseg) {
                    // segment s ends inside the range on a frame boundary and s + 1 follows at once,
                    // covering the rest: one train of frames (the wave holds s + 1's first byte)
                    const u32 d = (u32)(send - F0);
                    jb = (d >= gg) + (d >= 2 * gg);
                    so2 = hit ? o1 : sld64(seg_off + s + 1);
                    sl2 = hit ? l1 : sld64(seg_len + s + 1);
                    if (d == jb * gg && kA + jb <= max_frames && (u32)nfr - jb <= max_frames && so2 == so + sl &&
                        sl2 < (1ull << 31) && so2 <= hi && sl2 <= hi - so2 && fend <= send + (long long)sl2) {
                        u32 q = uni32((u32)((float)(u32)sl2 * S.rg)), t2 = q * gg;
                        if (t2 > (u32)sl2) --q;
                        else if ((u32)sl2 - t2 >= gg) ++q;
                        nfull2 = q < max_frames ? q : max_frames;
                        fast = true;
                    }
                }
                if (fast) {
                    allseg = true;
                    s_stop = jb < 3 ? s + 2 : s + 1;
                    const u64 dbase = desc_base ? sld64(desc_base + s) : (u64)s * max_frames;
                    const u64 dbase2 = jb == 3 ? 0 : (desc_base ? sld64(desc_base + s + 1) : (u64)(s + 1) * max_frames);
                    if (jb < 3 && lane == 0)            // the predicted result of segment s + 1
                        ws_store_res(res + s + 1, (u64)nfull2 * gg, nfull2,
                                     nfull2 == max_frames && (u64)nfull2 * gg < sl2 ? WEBSOCKET_SEG_MAX_FRAMES
                                                                                    : WEBSOCKET_SEG_OK);
                    const u64 rpos = r0 - lead0;                                    // buffer offset of range byte 0
                    int Fj[3], Pj[3];
                    u32 RK[3];
                    bool bad = false, bad2 = false;
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const int F = F0 + j * (int)gg;
                        Fj[j] = F;
                        Pj[j] = 0x40000000;
                        RK[j] = 0;
                        if (j && F >= (int)RW) continue;
                        const u64 pos = rpos + (u64)(long long)F;
                        const uintptr_t pa = reinterpret_cast<uintptr_t>(buf) + pos;
                        const HdrWords hw = load_header(reinterpret_cast<const unsigned char*>(pa));
                        const u32 sh = 8u * (u32)(pa & 3);
                        const u32 d0 = (u32)((((u64)hw.w1 << 32) | hw.w0) >> sh);
                        const u32 d1 = (u32)((((u64)hw.w2 << 32) | hw.w1) >> sh);
                        const u32 d2 = (u32)((((u64)hw.w3 << 32) | hw.w2) >> sh);
                        const u32 d3 = (u32)((((u64)hw.w4 << 32) | hw.w3) >> sh);
                        u32 hdr, masked, key;
                        bool ok;
                        if ((d0 & S.fm[0]) == S.fe[0] && (d1 & S.fm[1]) == S.fe[1] && (d2 & S.fm[2]) == S.fe[2]) {
                            ok = true;
                            masked = 1;
                            hdr = S.fhdr;
                            key = S.f64 ? (d2 >> 16) | (d3 << 16) : d1;
                        } else {
                            ok = spec_match((u64)d0 | ((u64)d1 << 32), (u64)d2 | ((u64)d3 << 32), S, hdr, masked, key);
                        }
                        if (F >= 0) {                                               // this wave owns the header
                            const bool second = (u32)j >= jb;
                            if (!ok) {
                                if (second) bad2 = true;
                                else bad = true;
                            } else if (lane == 0) {
                                spec_store_desc(desc + (second ? dbase2 + (j - jb) : dbase + kA + j), pos, d0 & 0xFFu, hdr,
                                                masked, gg);
                            }
                        }
                        Pj[j] = F + (int)hdr;
                        RK[j] = ok && masked ? rotl32(key, 8u * ((u32)(F + (int)hdr) & 3u)) : 0u;
                    }
                    if (bad && lane == 0) spec_flag(flags, list, head, s);
                    if (bad2 && lane == 0) spec_flag(flags, list, head, s + 1);
                    // the XOR rule per lane: its chunk's frame j (x >= F_j), whole-payload chunks
                    // one XOR per dword, chunks holding header bytes byte-exact for frames j, j + 1
#pragma unroll
                    for (int u = 0; u < SPEC_U; ++u) {
                        const int xx = u * 1024 + xl;
                        const bool a1 = xx >= Fj[1], a2 = xx >= Fj[2];
                        const int P = a2 ? Pj[2] : (a1 ? Pj[1] : Pj[0]);
                        const int E = a2 ? Fj[2] + (int)gg : (a1 ? Fj[2] : Fj[1]);
                        const u32 rk = a2 ? RK[2] : (a1 ? RK[1] : RK[0]);
                        cov[u] = 0xFFFFu;
                        if (xx >= P && xx + 16 <= E) {
                            v[u].x ^= rk; v[u].y ^= rk; v[u].z ^= rk; v[u].w ^= rk;
                        } else {
                            u32 cdummy = 0;
                            const int l1 = P > xx ? P - xx : 0, h1 = E < xx + 16 ? E - xx : 16;
                            if (h1 > l1) ws_xor_range(rk, l1, h1, v[u], cdummy);
                            const int Pn = a2 ? 0x40000000 : (a1 ? Pj[2] : Pj[1]);
                            const u32 rkn = a2 ? 0u : (a1 ? RK[2] : RK[1]);
                            if (Pn < xx + 16) ws_xor_range(rkn, Pn > xx ? Pn - xx : 0, 16, v[u], cdummy);
                        }
                    }
                }
            }
        }
        for (u32 it = 1; !fast && s < nseg; ++s, ++it) {
            if ((it & 63) == 0) {                                           // an unordered batch stores nothing:
                const u32 cc = lane == 0 ? ld_agent(myrepl) : 0u;           // stop walking garbage early
                if (__builtin_amdgcn_readfirstlane(cc) == 2) break;
            }
            const u64 so = sld64(seg_off + s), sl = sld64(seg_len + s);
            if (so >= rb) break;
            if (sl == 0 || (so < ra && sl <= ra - so)) continue;           // empty, or ends before the range
            if (so > hi || sl > hi - so) {                                  // outside the batch: the checkers
                if (lane == 0) spec_flag(flags, list, head, s);             // mark it unordered, nothing is
                continue;                                                   // stored; never load past it
            }
            // segment start relative to the range (origin coordinates: so + lead0 - r0)
            const long long sa = (long long)(so + lead0) - (long long)r0, sbb = sa + (long long)sl;
            if (sa <= 0 && sbb >= RW) {
                allseg = true;                                              // chunks all inside: stored whole
            } else {
                const int SA = (int)(sa < -16 ? -16 : (sa > RW + 16 ? RW + 16 : sa));
                const int SB = (int)(sbb < -16 ? -16 : (sbb > RW + 16 ? RW + 16 : sbb));
#pragma unroll
                for (int u = 0; u < SPEC_U; ++u) {
                    const int x = u * 1024 + xl;
                    const int l2 = SA > x ? (SA - x < 16 ? SA - x : 16) : 0;
                    const int h2 = SB > x ? (SB - x < 16 ? SB - x : 16) : 0;
                    if (h2 > l2) segcov[u] |= (0xFFFFu >> (16 - h2)) & (0xFFFFu << l2);
                }
            }
            // frames predicted: nfull = min(sl / g, max_frames)
            const u64 q = spec_div(sl, g, S.rg);
            const u32 nfull = q < max_frames ? (u32)q : max_frames;
            if (sa >= 0 && sa < RW && lane == 0)                            // the wave holding byte 0: result
                ws_store_res(res + s, (u64)nfull * g, nfull,
                             nfull == max_frames && (u64)nfull * g < sl ? WEBSOCKET_SEG_MAX_FRAMES : WEBSOCKET_SEG_OK);
            // frames k = kA.. whose start lies in front of r1 (kA: the frame holding r0); their
            // range-relative starts fr in 32 bits (g < 2^30: fr in (-g, RW + g))
            u32 kA = 0;
            int fr = (int)sa;
            if (sa < 0) {
                const u64 qa = spec_div((u64)(-sa), g, S.rg);
                kA = (u32)qa;
                fr = (int)(sa + (long long)(qa * g));
            }
            const u64 dbase = desc_base ? sld64(desc_base + s) : (u64)s * max_frames;
            bool bad = false;
            for (u32 k = kA; fr < (int)RW; ++k, fr += (int)g) {
                const u64 rel = (u64)k * g, pos = so + rel;                 // segment- / buffer-relative
                u64 w0, w1;
                if (k >= nfull) {                                           // past the predicted frames: the
                    if (k == nfull && k < max_frames && fr >= 0 && sl - rel >= 2) {   // tail must stay incomplete
                        spec_words_s(reinterpret_cast<uintptr_t>(buf) + pos, w0, w1);
                        bad |= ws_parse(w0, w1, sl - rel).kind != WS_PARSE_INCOMPLETE;
                    }
                    break;
                }
                spec_words_s(reinterpret_cast<uintptr_t>(buf) + pos, w0, w1);
                u32 hdr, masked, key;
                const bool ok = spec_match(w0, w1, S, hdr, masked, key);
                if (fr >= 0) {                                              // this wave owns the header
                    if (!ok) bad = true;
                    else if (lane == 0) spec_store_desc(desc + dbase + k, pos, (u32)w0 & 0xFFu, hdr, masked, (u32)g);
                }
                if (!ok || !masked) continue;                               // the XOR rule
                const int qa = fr + (int)hdr, qb = fr + (int)g;
                if (qb <= 0 || qa >= (int)RW) continue;
                // (origin-relative payload start r0 + qa: the key rotated to the chunk phase)
                spec_xor_rows(v, cov, qa < -16 ? -16 : qa, qb > (int)RW + 16 ? (int)RW + 16 : qb,
                              rotl32(key, 8u * (((u32)r0 + (u32)qa) & 3u)), xl);
            }
            if (bad && lane == 0) spec_flag(flags, list, head, s);
        }
        if (!fast) s_stop = s < nseg ? s + 1 : nseg;
    }
    // ---- 4. wait for the checkers' verdict (bounded), then store
    if (lane == 0) {
        for (u32 n = 0; verdict == 0 && n < spins; ++n) {
            __builtin_amdgcn_s_sleep(2);
            verdict = ld_agent(myrepl);
        }
    }
    verdict = (u32)__builtin_amdgcn_readlane((int)verdict, 0);
    if (!pvalid || verdict == 2) return;                                    // S2 walks an unordered batch
    if (verdict == 0) {
        // gave up waiting: store nothing; S2 finishes this range's segments (their XOR is
        // undone on the ranges that did store, then they are walked exactly)
        if (lane == 0) {
            *gptr<u32>(marks + ((r0 >> SPEC_RANGE_SHIFT) - (pbase << (SPEC_SHIFT - SPEC_RANGE_SHIFT)))) = tag;
            __hip_atomic_fetch_add(gptr<u32>(head + SPEC_TMO), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (u32 s = s_first; s < s_stop; ++s) {
                const u64 so = sld64(seg_off + s), sl = sld64(seg_len + s);
                if (sl && !(so < ra && sl <= ra - so) && so < rb) spec_flag(flags, list, head, s);
            }
        }
        return;
    }
#pragma unroll
    for (int u = 0; u < SPEC_U; ++u) {
        const int rel = u * 64 + (int)lane;
        if (!cov[u] || rel < A || rel > B) continue;
        gu32x4* const pc = reinterpret_cast<gu32x4*>(sbase + (u32)((rel - A) * 16));
        if (cov[u] == 0xFFFFu || allseg || segcov[u] == 0xFFFFu) st16<NT>(v[u], pc);
        else ws_store_bytes(reinterpret_cast<gu8*>(pc), v[u], cov[u]);
    }
}

// ------------------------------------------------------------------------------------------
// S2: repair. One wave per segment, vector loads only (the wave rewrites payload bytes and
// then reads headers that may lie in them; the scalar cache would keep stale lines).

// unmask [P0, P1) by one wave, skipping the 4 KiB wave ranges whose S1 wave stored nothing
template <int NT>
__device__ __forceinline__ void spec_xor_stored(unsigned char* buf, unsigned char* P0, unsigned char* P1, u32 key,
                                                const u32* marks, u32 tag, u64 rbase, bool any_tmo, u32 lane) {
    if (!any_tmo) {
        unmask_payload<4, NT>(P0, P1, key, lane);
        return;
    }
    const uintptr_t org = reinterpret_cast<uintptr_t>(buf) & ~(uintptr_t)15;
    uintptr_t a = reinterpret_cast<uintptr_t>(P0);
    const uintptr_t e = reinterpret_cast<uintptr_t>(P1);
    while (a < e) {
        const u64 r = (u64)(a - org) >> SPEC_RANGE_SHIFT;
        uintptr_t b = org + ((uintptr_t)(r + 1) << SPEC_RANGE_SHIFT);
        if (b > e) b = e;
        if (marks[r - rbase] != tag) {
            // the key phase follows the byte's distance from P0
            const u32 sh = 8u * (u32)((a - reinterpret_cast<uintptr_t>(P0)) & 3);
            unmask_payload<4, NT>(reinterpret_cast<unsigned char*>(a), reinterpret_cast<unsigned char*>(b),
                                  sh ? (key >> sh) | (key << (32 - sh)) : key, lane);
        }
        a = b;
    }
}

// the reactor loop over segment s with vector header loads (ws_walk.h:walk_segment otherwise)
template <int NT>
__device__ __forceinline__ void spec_walk(unsigned char* __restrict__ buf, u32 s, const u64* __restrict__ seg_off,
                                          const u64* __restrict__ seg_len, u32 max_frames,
                                          const u64* __restrict__ desc_base, WebsocketFrameDesc_t* __restrict__ desc,
                                          WebsocketSegResult_t* __restrict__ res, u32 lane) {
    const u64 so = seg_off[s], sl = seg_len[s];
    const u64 dbase = desc_base ? desc_base[s] : (u64)s * max_frames;
    unsigned char* const seg = buf + so;
    u64 off = 0;
    u32 nf = 0;
    int status = WEBSOCKET_SEG_OK;
    while (off < sl) {
        if (nf >= max_frames) { status = WEBSOCKET_SEG_MAX_FRAMES; break; }
        if (sl - off < 2) break;                                        // websocketframe.c:121
        unsigned char* const p = seg + off;
        u64 w0, w1;
        spec_words_v(p, w0, w1);
        const WsHdr h = ws_parse(w0, w1, sl - off);
        if (h.kind == WS_PARSE_INCOMPLETE) break;
        if (h.kind == WS_PARSE_WRAP) { status = WEBSOCKET_SEG_ERR_LEN_WRAP; break; }
        if (h.masked) unmask_payload<4, NT>(p + h.hdr, p + h.hdr + h.plen, h.key, lane);
        if (h.ret == 0) break;                                          // (int) truncated to 0
        if (lane == 0) ws_store_desc(desc + dbase + nf, so + off, h);
        ++nf;
        if (h.ret < 0) { status = WEBSOCKET_SEG_ERR_DECODE; break; }    // net_reactor.c:518-520
        off += (u32)h.ret;                                              // net_reactor.c:525
    }
    if (lane == 0) ws_store_res(res + s, off, nf, status);
}

template <int NT>
__global__ __launch_bounds__(256) void ws_piece_spec_fix_kernel(
    unsigned char* __restrict__ buf, const u64* __restrict__ seg_off, const u64* __restrict__ seg_len, u32 nseg,
    u32 max_frames, const u64* __restrict__ desc_base, WebsocketFrameDesc_t* __restrict__ desc,
    WebsocketSegResult_t* __restrict__ res, const u32* head, u32* next_head, u32* next_done, u32* flags,
    const u32* list, const u32* marks, u32 tag, u64 pbase, SpecSig S, int* advice) {
    const u32 lane = threadIdx.x & 63;
    const u32 gw = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u32 nw = gridDim.x * 4;
    const u32 c = *gptr<u32>(head + SPEC_CTR), nmis = *gptr<u32>(head + SPEC_NMIS);
    const bool tmo = *gptr<u32>(head + SPEC_TMO) != 0;
    const u64 rbase = pbase << (SPEC_SHIFT - SPEC_RANGE_SHIFT);
    const u64 g = S.g;
    if (c >> 16) {
        // unordered (or outside [lo, hi)): S1 stored nothing; the reactor loop per segment
        for (u32 s = gw; s < nseg; s += nw) spec_walk<NT>(buf, s, seg_off, seg_len, max_frames, desc_base, desc, res, lane);
        for (u32 i = gw * 64 + lane; i < nmis; i += nw * 64) *gptr<u32>(flags + list[i]) = 0;
    } else {
        for (u32 i = gw; i < nmis; i += nw) {
            const u32 s = list[i];
            const u64 so = seg_off[s], sl = seg_len[s];
            // undo S1's XOR where it stored: the same rule over the same (unchanged) header bytes
            for (u64 k = 0; k < max_frames && (k + 1) * g <= sl; ++k) {
                unsigned char* const p = buf + so + k * g;
                u64 w0, w1;
                spec_words_v(p, w0, w1);
                u32 hdr, masked, key;
                if (spec_match(w0, w1, S, hdr, masked, key) && masked)
                    spec_xor_stored<NT>(buf, p + hdr, p + g, key, marks, tag, rbase, tmo, lane);
            }
            spec_walk<NT>(buf, s, seg_off, seg_len, max_frames, desc_base, desc, res, lane);
            if (lane == 0) *gptr<u32>(flags + s) = 0;
        }
    }
    if (gw == 0) {
        // the next call's head and verdict words rest at zero
        gptr<u32>(next_done)[lane * (SPEC_REPL_STRIDE / 4)] = 0;
        if (lane == 0) {
            gu32* nh = gptr<u32>(next_head);
            nh[SPEC_CTR] = 0;
            nh[SPEC_NMIS] = 0;
            nh[SPEC_TMO] = 0;
            // the host's next path choice: stay speculative while at most 1/32 of the segments
            // needed the exact walk; the frame length to predict with next time
            if (advice) {
                __hip_atomic_store(advice, (c >> 16) == 0 && (u64)nmis * 32 <= nseg ? 1 : 0, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(advice + 1, (int)ws_first_frame_len(buf, seg_off, seg_len, nseg), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
extern WsOpt ws_piece_win;
extern WsOpt ws_k2_timing;
int ws_k2_mark(hipStream_t st, bool end, size_t* slot);

// spec workspace: [head A, head B: 4 u32 each][verdict words A, B: SPEC_REPL x SPEC_REPL_STRIDE each]
//                 [flags: nseg u32][list: nseg u32][marks: one u32 per 4 KiB range]
#define SPEC_OFF_DONE 1024
#define SPEC_DONE_BYTES (SPEC_REPL * SPEC_REPL_STRIDE)
size_t ws_spec_flags_off() { return SPEC_OFF_DONE + 2 * SPEC_DONE_BYTES; }

size_t ws_spec_workspace_bytes(u64 span, u32 nseg) {
    const u64 ranges = ((span + 15) >> SPEC_RANGE_SHIFT) + 8;
    return ws_spec_flags_off() + (size_t)nseg * 8 + (size_t)ranges * 4 + 64;
}

// bytes that must be zero when the workspace is (re)allocated: heads, verdict words, flags
size_t ws_spec_zero_bytes(u32 nseg) { return ws_spec_flags_off() + (size_t)nseg * 4; }

// S1 can run only when its checkers are a small part of the grid: <= 1024 waves of <= 256 segments
bool ws_spec_fits(u64 span, u32 nseg) {
    const u64 npieces = (span + (1ull << SPEC_SHIFT) - 1) >> SPEC_SHIFT;
    const u64 waves = (npieces + 2) * (SPEC_T / 64);
    const u64 nchk = waves < 1024 ? waves : 1024;
    return npieces >= 1 && nseg >= 1 && (u64)nseg <= nchk * 256;
}

// g: the frame wire length to predict every segment with (2 <= g < 2^30)
int ws_launch_piece_spec(const WsLaunch& L, u64 lo, u64 hi, unsigned char* sws, u32 parity, u32 tag, u32 g,
                         int* advice_dev) {
    const u64 lead0 = reinterpret_cast<uintptr_t>(L.buf) & 15;
    const u64 lo_org = lo + lead0, hi_org = hi + lead0;
    const u64 npieces = hi_org > lo_org ? ((hi_org - 1) >> SPEC_SHIFT) - (lo_org >> SPEC_SHIFT) + 1 : 0;
    if (!npieces || g < 2 || g >= (1u << 30)) return ws_set_msg("spec decode: empty range or frame length out of range");
    const u64 pbase = lo_org >> SPEC_SHIFT, c_lo = lo_org >> 4, c_hi = (hi_org + 15) >> 4;
    const u32 p = parity & 1;
    u32* head = reinterpret_cast<u32*>(sws) + SPEC_HEAD_WORDS * p;
    u32* next_head = reinterpret_cast<u32*>(sws) + SPEC_HEAD_WORDS * (p ^ 1);
    u32* done = reinterpret_cast<u32*>(sws + SPEC_OFF_DONE + p * SPEC_DONE_BYTES);
    u32* next_done = reinterpret_cast<u32*>(sws + SPEC_OFF_DONE + (p ^ 1) * SPEC_DONE_BYTES);
    u32* flags = reinterpret_cast<u32*>(sws + ws_spec_flags_off());
    u32* list = flags + L.nseg;
    u32* marks = list + L.nseg;
    const int pwin = ws_piece_win;
    u32 wshift = (u32)(pwin < 0 ? 0 : (pwin > 6 ? 6 : pwin));
    while (wshift && (npieces >> wshift) < 256) --wshift;                // small batches: one window
    const u64 ppw = (npieces + (1ull << wshift) - 1) >> wshift;
    const u64 grid = ppw << wshift;
    const u64 waves = grid * (SPEC_T / 64);
    const u32 nchk = (u32)(waves < 1024 ? waves : 1024);
    const u32 chk_per = (u32)((L.nseg + nchk - 1) / nchk);
    if (chk_per > 256) return ws_set_msg("spec decode: too many segments for the checkers");
    SpecSig S = spec_sig(g);
    S.gs = (float)L.nseg * 256.0f / (float)(hi - lo);
    size_t tslot = 0;
    int rc;
    const int timing = ws_k2_timing;
    if (timing && (rc = ws_k2_mark(L.stream, false, &tslot))) return rc;
    hipLaunchKernelGGL(ws_piece_spec_kernel<1>, dim3((u32)grid), dim3(SPEC_T), ws_piece_dyn_lds(L), L.stream, L.buf,
                       L.seg_off, L.seg_len, L.nseg, L.max_frames, L.desc_base, L.desc, L.res, head, done, flags, list,
                       marks, tag, pbase, c_lo, c_hi, lo, hi, ppw, npieces, wshift, nchk, chk_per,
                       (u32)(int)ws_spec_spins, S);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ws_set_err("ws_piece_spec_kernel launch", e);
    if (timing && (rc = ws_k2_mark(L.stream, true, &tslot))) return rc;
    const u32 fix_blocks = (u32)((L.nseg + 3) / 4 < 256 ? (L.nseg + 3) / 4 : 256);
    hipLaunchKernelGGL(ws_piece_spec_fix_kernel<1>, dim3(fix_blocks), dim3(256), 0, L.stream, L.buf, L.seg_off,
                       L.seg_len, L.nseg, L.max_frames, L.desc_base, L.desc, L.res, head, next_head, next_done, flags,
                       list, marks, tag, pbase, S, advice_dev);
    e = hipGetLastError();
    if (e != hipSuccess) return ws_set_err("ws_piece_spec_fix_kernel launch", e);
    return 0;
}
