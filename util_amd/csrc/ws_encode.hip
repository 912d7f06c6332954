// ws_encode.hip — batch frame encode + client-side masking.
//
// For every frame descriptor: the header websocketframeEncode writes
// (websocketframe.c:167-202: first byte from (prev_is_fin, is_fin, type), 7/16/64-bit
// length), plus — when `masked` — the MASK bit and the 4-byte key (RFC 6455 §5.3,
// which the reference's encoder never sets), followed by the payload XORed with the
// key. Frames are laid out back to back in d_dst.
//
// Default front (enc_front 1), before E3:
// F1 one thread per frame: wire bytes of each 256-frame tile.
// F2 one block: exclusive scan of the tile sums; d_wire_off[n] = the total.
// F3 one thread per frame: its wire offset (tile prefix + block scan) -> d_wire_off[i];
//    every 16 KiB output piece whose first byte lies in the frame's wire range gets the
//    frame index (pieces past the end: none); and the frame's edge chunks (E4 below).
// E3 one-shot 256-thread block per output piece, 4 x 16 B chunks per lane: the wave
//    reads up to 64 frame records from its piece's first frame, then every chunk that
//    lies inside one payload is one unaligned 16-B source load + XOR + aligned store.
// E4 (edge chunks) every chunk whose first byte lies in the frame's wire extent and that
//    is not inside one payload (header bytes, frame edges): frames with >= 32 B payloads
//    OR byte-shifted header and masked 16-B source windows, the rest assemble byte by
//    byte; one 16-B store each. Every output chunk is written exactly once.
// enc_front 0: E1 hipcub exclusive scan -> E2 piece pointers -> E3 -> E4 as its own
// kernel (after E3, or with "encode_side" on a side stream concurrently with E2+E3 —
// measured slower on MI355X).
#include <hipcub/hipcub.hpp>

#include "ws_common.h"

#define ENC_T 256
#define ENC_U 4
#define ENC_SHIFT 14
#define ENC_NONE 0xFFFFFFFFu

__device__ __forceinline__ u32 enc_hl(u64 len) { return len < 126 ? 2u : (len <= 0xFFFFull ? 4u : 10u); }

struct EncFrame {
    u64 src, len, off;   // payload source offset, payload length, wire offset (dst-relative)
    u32 key, hl;         // key (LE), header bytes incl. mask key
    u32 b0, masked;
};

// record i with its wire offset `off` (dst-relative)
__device__ __forceinline__ EncFrame enc_load_at(const WebsocketEncodeDesc_t* f, u32 i, u64 off) {
    const gu32x4* q = gptr<u32x4>(f + i);
    const u32x4 a = q[0];
    const u32 w4 = gptr<u32>(f + i)[4], w5 = gptr<u32>(f + i)[5];
    EncFrame e;
    e.src = (u64)a.x | ((u64)a.y << 32);
    e.len = (u64)a.z | ((u64)a.w << 32);
    e.key = w4;
    const u32 type = w5 & 0xFFu, fin = (w5 >> 8) & 0xFFu, prev_fin = (w5 >> 16) & 0xFFu;
    e.masked = (w5 >> 24) != 0;
    const u32 op = prev_fin ? type : 0u;                                     // websocketframe.c:176-202
    e.b0 = (fin ? (op | 0x80u) : op) & 0xFFu;
    e.hl = enc_hl(e.len) + (e.masked ? 4u : 0u);
    e.off = off;
    return e;
}

__device__ __forceinline__ EncFrame enc_load(const WebsocketEncodeDesc_t* f, const u64* wire_off, u32 i) {
    return enc_load_at(f, i, wire_off[i]);
}

// byte j of the frame's header (j < hl)
__device__ __forceinline__ u32 enc_header_byte(const EncFrame& e, u32 j) {
    const u32 n = enc_hl(e.len);
    if (j == 0) return e.b0;
    if (j == 1) return (n == 2 ? (u32)e.len : (n == 4 ? 126u : 127u)) | (e.masked ? 0x80u : 0u);
    if (j < n) return (u32)(e.len >> (8 * (n - 1 - j))) & 0xFFu;            // big-endian extended length
    return (e.key >> (8 * (j - n))) & 0xFFu;                                 // mask key, wire order
}

struct WireLen {
    const WebsocketEncodeDesc_t* f;
    u32 n;
    __host__ __device__ u64 operator()(u32 i) const {
        if (i >= n) return 0;
        const u64 len = f[i].len;
        return (u64)(len < 126 ? 2u : (len <= 0xFFFFull ? 4u : 10u)) + (f[i].masked ? 4u : 0u) + len;
    }
};

__global__ __launch_bounds__(256) void ws_enc_ptr_kernel(const WebsocketEncodeDesc_t* __restrict__ f, u32 n,
                                                         const u64* __restrict__ wire_off, u32* __restrict__ ptr,
                                                         u64 lead0, u64 npieces) {
    const u32 i = blockIdx.x * 256 + threadIdx.x;
    if (i > n) return;
    const u64 a = i ? wire_off[i] + lead0 : 0;                               // frame 0 also owns the origin
    const u64 b = i < n ? wire_off[i + 1] + lead0 : ((npieces) << ENC_SHIFT);
    const u32 val = i < n ? i : ENC_NONE;                                    // i == n: pieces past the end
    for (u64 p = (a + (1ull << ENC_SHIFT) - 1) >> ENC_SHIFT; (p << ENC_SHIFT) < b && p < npieces; ++p) ptr[p] = val;
}

__device__ __forceinline__ void put_byte(u32x4& w, u32 b, u32 v) {
    const u32 sh = 8u * (b & 3);
    w.x |= b < 4 ? v << sh : 0u;
    w.y |= (b >> 2) == 1 ? v << sh : 0u;
    w.z |= (b >> 2) == 2 ? v << sh : 0u;
    w.w |= b >= 12 ? v << sh : 0u;
}

typedef u32x4 __attribute__((aligned(1))) u32x4u;

// Fast edge path of frame i (payload >= 32 B, its extent not clipped, and a next payload
// entering its tail chunk >= 16 B long): the head chunk [X0, +16) = header + payload
// bytes [0, 16) (only if the header reaches past X0), the tail chunk [XT, +16) = payload
// bytes [len-16, len) + the next frame's header (+ its payload bytes [0, 16)). Frame-
// local, so E3 (which stores these chunks for eligible frames) and E4 (which skips them)
// agree on it. nx: frame i+1's record (unused when i+1 == n).
__device__ __forceinline__ bool enc_edge_eligible(const EncFrame& e, const EncFrame& nx, u32 i, u32 n, u64 lead0,
                                                  u64 out_lo, u64 out_hi) {
    const u64 o = e.off + lead0, d1 = o + e.hl + e.len, XT = d1 & ~15ull;
    if (!(e.len >= 32 && (i > 0 || (o & 15) == 0) && o >= out_lo && XT + 16 <= out_hi)) return false;
    const bool npay = (d1 & 15) && i + 1 < n && d1 + nx.hl < XT + 16;
    return !npay || nx.len >= 16;
}

// 16 bytes as two little-endian words; byte shifts move bytes to higher (shl) or lower
// (shr) addresses, bytes shifted past either end are dropped
struct U128 {
    u64 lo, hi;
};
__device__ __forceinline__ U128 u128_of(const u32x4 w) {
    return {(u64)w.x | ((u64)w.y << 32), (u64)w.z | ((u64)w.w << 32)};
}
__device__ __forceinline__ u32x4 u32x4_of(const U128 a) {
    return (u32x4){(u32)a.lo, (u32)(a.lo >> 32), (u32)a.hi, (u32)(a.hi >> 32)};
}
__device__ __forceinline__ U128 u128_shl(const U128 a, u32 nb) {
    const u32 s = 8u * nb;
    if (s == 0) return a;
    if (s >= 128) return {0, 0};
    if (s < 64) return {a.lo << s, (a.hi << s) | (a.lo >> (64 - s))};
    return {0, a.lo << (s - 64)};
}
__device__ __forceinline__ U128 u128_shr(const U128 a, u32 nb) {
    const u32 s = 8u * nb;
    if (s == 0) return a;
    if (s >= 128) return {0, 0};
    if (s < 64) return {(a.lo >> s) | (a.hi << (64 - s)), a.hi >> s};
    return {a.hi >> (s - 64), 0};
}
// 16 payload bytes from a source window XORed with the key at phase r (byte t gets key byte (r + t) & 3)
__device__ __forceinline__ U128 u128_masked(const u32x4 w, u32 key, u32 r) {
    const u32 k = rotl32(key, (32u - 8u * (r & 3u)) & 31u);
    const u64 kk = (u64)k | ((u64)k << 32);
    const U128 a = u128_of(w);
    return {a.lo ^ kk, a.hi ^ kk};
}
// the frame's header (websocketframe.c:176-202 + MASK bit and key) as bytes [0, hl), zero above
__device__ __forceinline__ U128 enc_header128(const EncFrame& e) {
    const u32 n = enc_hl(e.len);
    const u32 b1 = (n == 2 ? (u32)e.len : (n == 4 ? 126u : 127u)) | (e.masked ? 0x80u : 0u);
    U128 h = {(u64)e.b0 | ((u64)b1 << 8), 0};
    if (n == 4) h.lo |= (u64)(((u32)e.len >> 8) & 0xFFu) << 16 | (u64)((u32)e.len & 0xFFu) << 24;
    if (n == 10) {
        const u64 be = __builtin_bswap64(e.len);                         // big-endian 64-bit length
        h.lo |= be << 16;
        h.hi = be >> 48;
    }
    if (e.masked) {
        if (n == 10) h.hi |= (u64)e.key << 16;                           // bytes 10..13
        else h.lo |= (u64)e.key << (8u * n);                             // bytes 2..5 / 4..7
    }
    return h;
}

// Assemble and store the eligible frame's head / tail chunks that start in [rlo, rhi)
// (origin-relative): the 16-B source windows they need are loaded together, and each
// chunk is the OR of byte-shifted header and masked-window words (no byte loop).
// the three 16-B source windows of an edge: the payload's first and last 16 bytes and the next
// payload's first 16 bytes
struct EncWin {
    u32x4 h, t, n;
};
__device__ __forceinline__ u32x4 enc_win16(const unsigned char* src, u64 at) {
    return *reinterpret_cast<const WS_GLOBAL u32x4u*>(reinterpret_cast<uintptr_t>(src + at));
}

__device__ __forceinline__ void enc_edge_store_win(gu32x4* base, const EncFrame& e, const EncFrame& nx, bool nxt,
                                                   u64 lead0, u64 rlo, u64 rhi, const EncWin& W);

__device__ __forceinline__ void enc_edge_store(const unsigned char* __restrict__ src, gu32x4* base,
                                               const EncFrame& e, const EncFrame& nx, bool nxt, u64 lead0,
                                               u64 rlo, u64 rhi) {
    const u64 o = e.off + lead0, d0 = o + e.hl, d1 = d0 + e.len;
    const u64 X0 = (o + 15) & ~15ull, XT = d1 & ~15ull;
    const bool head = X0 < d0 && X0 >= rlo && X0 < rhi, tail = (d1 & 15) != 0 && XT >= rlo && XT < rhi;
    const bool npay = tail && nxt && d1 + nx.hl < XT + 16;
    EncWin W = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    if (head) W.h = enc_win16(src, e.src);
    if (tail) W.t = enc_win16(src, e.src + e.len - 16);
    if (npay) W.n = enc_win16(src, nx.src);
    enc_edge_store_win(base, e, nx, nxt, lead0, rlo, rhi, W);
}

__device__ __forceinline__ void enc_edge_store_win(gu32x4* base, const EncFrame& e, const EncFrame& nx, bool nxt,
                                                   u64 lead0, u64 rlo, u64 rhi, const EncWin& W) {
    const u64 o = e.off + lead0, d0 = o + e.hl, d1 = d0 + e.len;
    const u64 X0 = (o + 15) & ~15ull, XT = d1 & ~15ull;
    const bool head = X0 < d0 && X0 >= rlo && X0 < rhi, tail = (d1 & 15) != 0 && XT >= rlo && XT < rhi;
    const u64 dn0 = d1 + nx.hl;                                          // next payload start
    const bool npay = tail && nxt && dn0 < XT + 16;                      // next payload enters the tail chunk
    const u32x4 wh = W.h, wt = W.t, wn = W.n;
    const u32 kh = e.masked ? e.key : 0u, kn = nx.masked ? nx.key : 0u;
    if (head) {                                                          // header bytes from X0, then payload [0, ..)
        U128 w = u128_shr(enc_header128(e), (u32)(X0 - o));
        const U128 p = u128_shl(u128_masked(wh, kh, 0), (u32)(d0 - X0));
        w.lo |= p.lo;
        w.hi |= p.hi;
        base[X0 >> 4] = u32x4_of(w);
    }
    if (tail) {                                                          // payload [len-16, len) then the next frame
        const u32 r = (u32)(d1 - XT);                                    // payload bytes in the chunk, 1..15
        U128 w = u128_shr(u128_masked(wt, kh, (u32)e.len), 16u - r);
        if (nxt) {
            const U128 h = u128_shl(enc_header128(nx), r);
            w.lo |= h.lo;
            w.hi |= h.hi;
            if (npay) {
                const U128 p = u128_shl(u128_masked(wn, kn, 0), (u32)(dn0 - XT));
                w.lo |= p.lo;
                w.hi |= p.hi;
            }
            base[XT >> 4] = u32x4_of(w);
        } else {
            ws_store_bytes(reinterpret_cast<gu8*>(base + (XT >> 4)), u32x4_of(w), (1u << r) - 1u);   // past the batch
        }
    }
}

template <int NT, int FUSED>
__global__ __launch_bounds__(ENC_T) void ws_enc_copy_kernel(const unsigned char* __restrict__ src,
                                                            const WebsocketEncodeDesc_t* __restrict__ f, u32 n,
                                                            const u64* __restrict__ wire_off,
                                                            const u32* __restrict__ ptr, unsigned char* __restrict__ dst,
                                                            u64 capacity, u32 npieces) {
    const u32 tid = threadIdx.x, lane = tid & 63;
    // output piece: block b -> piece b. Measured and not kept (round 5): 2-8 windows
    // (+0.6-2 %), the four blocks of every 32 on one XCD taking consecutive pieces (+0.8 %, though
    // E3's read over-fetch drops 1.036 -> 1.017 x)
    const u32 pb = blockIdx.x;
    if (pb >= npieces) return;                                               // the spare blocks
    const u32 wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u64 lead0 = reinterpret_cast<uintptr_t>(dst) & 15;
    gu32x4* const base = reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(dst) & ~(uintptr_t)15);
    const u64 total = min(wire_off[n], capacity);                            // never write past the capacity
    const u64 out_lo = lead0, out_hi = lead0 + total;                        // origin-relative output
    const u64 r0 = (((u64)pb << ENC_SHIFT) + (u64)wv * (64 * ENC_U * 16));  // origin-relative
    const u64 r1 = r0 + 64 * ENC_U * 16;
    const u32 first = *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(ptr + pb));
    // the next piece's first frame: the frames that touch this piece are exactly [first, that
    // one] (it holds the next piece's first byte), so the first record load takes only those —
    // with pieces dealt round-robin over the XCDs, 16 records per wave would pull each record
    // line into most of the 8 L2s
    const u32 nxt = pb + 1 < npieces ? *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(ptr + pb + 1)) : ENC_NONE;
    if (first == ENC_NONE) return;
    const bool exact = nxt != ENC_NONE && nxt >= first && nxt - first < 16u;
    // chunk state: fast = one payload source for the whole chunk
    u64 fsrc[ENC_U];
    u32 fkey[ENC_U];
    u32 kind[ENC_U];                                                          // 1: inside one payload
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) { kind[u] = 0; fsrc[u] = 0; fkey[u] = 0; }
    // records load `step` at a time: 16 first (a 4 KiB wave range rarely needs more), 64 after
    // that — 64 lanes loading would fetch 2 KiB of records per wave, into every XCD's L2
    for (u32 k = first, step = exact ? nxt - first + 1 : 16; k < n;) {
        const u32 j = k + lane;
        const bool valid = j < n && lane < step;
        EncFrame e = {};
        if (valid) e = enc_load(f, wire_off, j);
        const u64 eo = e.off + lead0, ee = eo + e.hl + e.len;                // origin-relative extent
        const u64 past = __ballot(valid && eo >= r1);
        const u32 nlim = past ? (u32)__builtin_ctzll(past) : 64u;
        u64 hm = __ballot(valid && lane < nlim && ee > r0);
        while (hm) {
            const int i = __builtin_ctzll(hm);
            hm &= hm - 1;
            EncFrame g;
            g.src = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)e.src, i)) |
                    ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(e.src >> 32), i) << 32);
            g.len = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)e.len, i)) |
                    ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(e.len >> 32), i) << 32);
            g.off = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)eo, i)) |
                    ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(eo >> 32), i) << 32);   // origin-relative
            g.key = (u32)__builtin_amdgcn_readlane((int)e.key, i);
            g.hl = (u32)__builtin_amdgcn_readlane((int)e.hl, i);
            g.b0 = (u32)__builtin_amdgcn_readlane((int)e.b0, i);
            g.masked = (u32)__builtin_amdgcn_readlane((int)e.masked, i);
            const u64 d0 = g.off + g.hl, d1 = d0 + g.len;                    // payload (origin-relative)
            const u32 rk = g.masked ? rotl32(g.key, 8u * (u32)(d0 & 3)) : 0u;  // key phase of aligned chunks
#pragma unroll
            for (int u = 0; u < ENC_U; ++u) {
                const u64 x = r0 + (u64)(u * 1024 + lane * 16);
                if (x + 16 <= g.off || x >= d1) continue;                    // no byte of this frame
                if (x >= d0 && x + 16 <= d1) {                               // inside the payload
                    kind[u] = 1;
                    fsrc[u] = g.src + (x - d0);
                    fkey[u] = rk;
                    continue;
                }
                // chunks with header bytes or a frame edge: below (FUSED) or ws_enc_edge_kernel
            }
        }
        if (FUSED) {
            // edge chunks of this batch's eligible frames that start in this wave's range: the
            // next frame's record from lane + 1 (the batch's last lane loads it); the source
            // windows are mostly lines this block is streaming anyway
            EncFrame nx;
            nx.src = __shfl_down(e.src, 1, 64); nx.len = __shfl_down(e.len, 1, 64);
            nx.off = __shfl_down(e.off, 1, 64); nx.key = __shfl_down(e.key, 1, 64);
            nx.hl = __shfl_down(e.hl, 1, 64); nx.b0 = __shfl_down(e.b0, 1, 64);
            nx.masked = __shfl_down(e.masked, 1, 64);
            const bool nxt = j + 1 < n;
            const bool mine = valid && lane < nlim && ee > r0;
            if (mine && lane == step - 1 && nxt) nx = enc_load(f, wire_off, j + 1);
            if (mine && enc_edge_eligible(e, nx, j, n, lead0, out_lo, out_hi))
                enc_edge_store(src, base, e, nx, nxt, lead0, r0, r1);
        }
        if (nlim < step || exact) break;
        k += step;
        step = 64;
    }
    // payload-interior chunks: one unaligned 16-B source load each (issued together)
    u32x4 v[ENC_U];
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
        v[u] = (u32x4){0, 0, 0, 0};
        if (kind[u] == 1) v[u] = *reinterpret_cast<const WS_GLOBAL u32x4u*>(reinterpret_cast<uintptr_t>(src + fsrc[u]));
    }
    // (nt stores: sc1|nt measured +5 %, profiles/r04_store_sc1nt_ab.log — unlike the in-place
    // decode kernels, where it gains)
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
        const u64 x = r0 + (u64)(u * 1024 + lane * 16);
        if (kind[u] == 1 && x + 16 <= out_hi) st16<NT>(v[u] ^ fkey[u], base + (x >> 4));
    }
}

// Every 16-B output chunk that is not inside one payload (header bytes, frame edges,
// the batch's first and last chunk): assembled by the frame whose wire extent holds the
// chunk's first byte (frame 0 also takes a chunk starting before the output) and stored
// once. Eligible frames (enc_edge_eligible) take the shift path; the rest byte by byte —
// header bytes computed, payload bytes loaded — walking the following frames with their
// offsets accumulated from e.off (no wire_off reads past frame i: the front kernel calls
// this while other blocks are still writing wire_off). skip_eligible: E3 (encode_fused)
// stores the eligible frames' chunks.
__device__ __forceinline__ void enc_edges(const unsigned char* __restrict__ src, const WebsocketEncodeDesc_t* __restrict__ f,
                                          u32 n, u32 i, const EncFrame& e, const EncFrame& nx, unsigned char* dst,
                                          u64 total, bool skip_eligible) {
    const u64 lead0 = reinterpret_cast<uintptr_t>(dst) & 15;
    gu32x4* const base = reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(dst) & ~(uintptr_t)15);
    const u64 out_lo = lead0, out_hi = lead0 + total;
    const u64 o = e.off + lead0, d0 = o + e.hl, d1 = d0 + e.len;
    if (enc_edge_eligible(e, nx, i, n, lead0, out_lo, out_hi)) {
        if (!skip_eligible) enc_edge_store(src, base, e, nx, i + 1 < n, lead0, 0, ~0ull);
        return;
    }
    u64 X = i ? ((o + 15) & ~15ull) : (o & ~15ull);                           // first chunk start owned
    const u64 lim = d1 < out_hi ? d1 : out_hi;                               // interior chunks end here
    for (; X < d1 && X < out_hi; X += 16) {
        if (X >= d0 && X + 16 <= lim) {                                      // payload interior: copy kernel
            X = (lim - 16) & ~15ull;                                         // last interior chunk
            continue;
        }
        u32x4 w = {0, 0, 0, 0};
        u32 g = i;
        EncFrame h = e;
        for (;;) {
            const u64 ho = h.off + lead0, hd0 = ho + h.hl, hd1 = hd0 + h.len;
            const u64 lo = ho > X ? ho : X, hi = hd1 < X + 16 ? hd1 : X + 16;
            // this frame's payload bytes in the chunk come from ONE 16-B window of the source
            // (kept inside the payload: start = min(first index, len - 16)); byte loads only
            // for payloads shorter than 16 B
            const u64 pa = lo > hd0 ? lo - hd0 : 0;                          // first payload index needed
            const u64 wst = h.len >= 16 ? (pa < h.len - 16 ? pa : h.len - 16) : 0;
            u32x4 win = {0, 0, 0, 0};
            if (h.len >= 16 && hi > hd0)
                win = *reinterpret_cast<const WS_GLOBAL u32x4u*>(reinterpret_cast<uintptr_t>(src + h.src + wst));
            for (u64 y = lo; y < hi; ++y) {
                u32 v;
                if (y < hd0) {
                    v = enc_header_byte(h, (u32)(y - ho));
                } else {
                    const u64 pi = y - hd0;
                    if (h.len >= 16) {
                        const u32 q = (u32)(pi - wst);
                        const u32 wq = q < 4 ? win.x : (q < 8 ? win.y : (q < 12 ? win.z : win.w));
                        v = (wq >> (8u * (q & 3))) & 0xFFu;
                    } else {
                        v = *reinterpret_cast<const gu8*>(reinterpret_cast<uintptr_t>(src + h.src + pi));
                    }
                    if (h.masked) v ^= (h.key >> (8 * (u32)(pi & 3))) & 0xFFu;
                }
                put_byte(w, (u32)(y - X), v);
            }
            if (hd1 >= X + 16 || ++g >= n) break;
            h = enc_load_at(f, g, h.off + h.hl + h.len);
        }
        gu32x4* const pc = base + (X >> 4);
        if (X >= out_lo && X + 16 <= out_hi) {
            *pc = w;
        } else {
            gu8* const pb = reinterpret_cast<gu8*>(pc);
            for (u32 q = 0; q < 16; ++q) {
                if (X + q < out_lo || X + q >= out_hi) continue;
                const u32 wq = q < 4 ? w.x : (q < 8 ? w.y : (q < 12 ? w.z : w.w));
                pb[q] = (unsigned char)(wq >> (8u * (q & 3)));
            }
        }
    }
}

// E4 of the hipcub front (enc_front 0): one thread per frame, offsets from E1's wire_off
__global__ __launch_bounds__(256) void ws_enc_edge_kernel(const unsigned char* __restrict__ src,
                                                          const WebsocketEncodeDesc_t* __restrict__ f, u32 n,
                                                          const u64* __restrict__ wire_off,
                                                          unsigned char* __restrict__ dst, u64 capacity,
                                                          u32 enc_fused) {
    const u32 i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const u64 total = min(wire_off[n], capacity);
    EncFrame e = enc_load(f, wire_off, i), nx = {};
    if (i + 1 < n) nx = enc_load(f, wire_off, i + 1);
    enc_edges(src, f, n, i, e, nx, dst, total, enc_fused != 0);
}

// ---- front (enc_front 1): F1 tile sums -> F2 tile scan -> F3 offsets + piece pointers + edges
// (256-frame tiles; 64-frame tiles, barrier-free, made F2's one-block scan 5 -> 32 us)
#define ENC_TILE 256

__device__ __forceinline__ u64 enc_wave_incl(u64 v, u32 lane) {
#pragma unroll
    for (u32 d = 1; d < 64; d <<= 1) {
        const u64 t = __shfl_up((unsigned long long)v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// F1: wire bytes of each 256-frame tile
__global__ __launch_bounds__(ENC_TILE) void ws_enc_tsum_kernel(const WebsocketEncodeDesc_t* __restrict__ f, u32 n,
                                                               u64* __restrict__ tsum) {
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const u32 i = blockIdx.x * ENC_TILE + tid;
    u64 wl = 0;
    if (i < n) {
        const u64 len = f[i].len;
        wl = (u64)enc_hl(len) + (f[i].masked ? 4u : 0u) + len;
    }
    const u64 incl = enc_wave_incl(wl, lane);
    __shared__ u64 ws[ENC_TILE / 64];
    if (lane == 63) ws[wv] = incl;
    __syncthreads();
    if (tid == 0) tsum[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// F2 (one block): exclusive scan of the B tile sums in place, t[B] = wire_off[n] = total
__global__ __launch_bounds__(1024) void ws_enc_tscan_kernel(u64* __restrict__ t, u32 B, u64* __restrict__ wire_off,
                                                            u32 n) {
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const u32 C = (B + 1023) / 1024, lo = tid * C < B ? tid * C : B, hi = lo + C < B ? lo + C : B;
    u64 sum = 0;
    for (u32 j = lo; j < hi; ++j) sum += t[j];
    const u64 incl = enc_wave_incl(sum, lane);
    __shared__ u64 ws[16];
    if (lane == 63) ws[wv] = incl;
    __syncthreads();
    u64 run = incl - sum;
    for (u32 w = 0; w < wv; ++w) run += ws[w];
    const u64 total = run + sum;                                             // thread 1023: the batch total
    __syncthreads();                                                         // every thread has read its sums
    for (u32 j = lo; j < hi; ++j) {
        const u64 v = t[j];
        t[j] = run;
        run += v;
    }
    if (tid == 1023) {
        t[B] = total;
        wire_off[n] = total;
    }
}

// F3: one thread per frame — wire offset (tile prefix + block scan), E2's piece pointers,
// E4's edge chunks
__global__ __launch_bounds__(ENC_TILE) void ws_enc_front_kernel(const unsigned char* __restrict__ src,
                                                                const WebsocketEncodeDesc_t* __restrict__ f, u32 n,
                                                                const u64* __restrict__ tpre, u32 B,
                                                                u64* __restrict__ wire_off, u32* __restrict__ ptr,
                                                                u64 npieces, unsigned char* __restrict__ dst,
                                                                u64 capacity, u32 enc_fused) {
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const u32 i = blockIdx.x * ENC_TILE + tid;
    EncFrame e = {}, nx = {};
    if (i < n) e = enc_load_at(f, i, 0);
    if (i + 1 < n) nx = enc_load_at(f, i + 1, 0);
    const u64 wl = i < n ? e.hl + e.len : 0;
    const u64 incl = enc_wave_incl(wl, lane);
    __shared__ u64 ws[ENC_TILE / 64];
    if (lane == 63) ws[wv] = incl;
    __syncthreads();
    u64 off = tpre[blockIdx.x] + incl - wl;                                  // tile prefix + block scan
    for (u32 w = 0; w < wv; ++w) off += ws[w];
    if (i >= n) return;
    const u64 all = tpre[B];
    wire_off[i] = off;
    e.off = off;
    nx.off = off + wl;
    const u64 lead0 = reinterpret_cast<uintptr_t>(dst) & 15;
    // piece pointers (ws_enc_ptr_kernel): pieces whose first byte lies in this frame's wire
    // range get i (frame 0 also owns the origin); the last frame also marks the pieces past the end
    const u64 a = i ? off + lead0 : 0, b = off + wl + lead0;
    for (u64 p = (a + (1ull << ENC_SHIFT) - 1) >> ENC_SHIFT; (p << ENC_SHIFT) < b && p < npieces; ++p) ptr[p] = i;
    if (i == n - 1)
        for (u64 p = (b + (1ull << ENC_SHIFT) - 1) >> ENC_SHIFT; p < npieces; ++p) ptr[p] = ENC_NONE;
    // the edge windows are loaded once the offsets say which are needed: loading all three
    // up front (in flight during the scan) measured 61 -> 92 us on cfg2, the random
    // source lines being this kernel's bound (profiles/r02_encode_front_ab.log)
    enc_edges(src, f, n, i, e, nx, dst, min(all, capacity), enc_fused != 0);
}

// Measured and dropped (round 2): E4 on a side stream, edges fused into E3,
// E3 over two windows or XCD-contiguous pieces, fewer E3 blocks per CU.
WsOpt ws_enc_front{1};    // "enc_front": 1 F1-F3 front (tile sums, tile scan, one thread per frame: offsets,
                          // piece pointers, edge chunks) before E3; 0 hipcub scan + E2, E3, then E4
                          // (round 5: F1-F3 as ONE launch with a decoupled look-back over 256- or 1024-frame
                          // tiles measured no faster, 76 us against 73; not kept)

extern "C" WSFRAME_AMD_EXPORT int websocketframeBatchEncodeDevice(const unsigned char* d_src,
                                                                  const WebsocketEncodeDesc_t* d_frames,
                                                                  unsigned int nframes, unsigned char* d_dst,
                                                                  unsigned long long dst_capacity,
                                                                  unsigned long long* d_wire_off, void* hip_stream) {
    if (nframes == 0) return 0;
    if (!d_src || !d_frames || !d_dst || !d_wire_off) return ws_set_msg("websocketframeBatchEncodeDevice: invalid argument");
    if (reinterpret_cast<uintptr_t>(d_frames) & 7) return ws_set_msg("websocketframeBatchEncodeDevice: d_frames not 8-B aligned");
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    const u64 lead0 = reinterpret_cast<uintptr_t>(d_dst) & 15;
    const u64 npieces = (dst_capacity + lead0 + (1ull << ENC_SHIFT) - 1) >> ENC_SHIFT;
    const bool front = ws_enc_front != 0;
    const u32 fused = 0u;
    hipError_t e;
    int rc;
    void* ws = nullptr;
    u32* ptr = nullptr;
    WsSlot slot;
    if ((rc = slot.acquire(st))) return rc;
    if (front) {
        // F1 tile sums -> F2 tile scan (also wire_off[n]) -> F3 offsets, piece pointers, edges
        const u32 B = (nframes + ENC_TILE - 1) / ENC_TILE, blocks = B;
        const size_t ptr_off = ((size_t)(B + 1) * 8 + 255) & ~(size_t)255;
        if ((rc = slot.encode_workspace(ptr_off + npieces * 4 + 16, &ws))) return rc;
        u64* tpre = reinterpret_cast<u64*>(ws);
        ptr = reinterpret_cast<u32*>(reinterpret_cast<unsigned char*>(ws) + ptr_off);
        hipLaunchKernelGGL(ws_enc_tsum_kernel, dim3(blocks), dim3(ENC_TILE), 0, st, d_frames, nframes, tpre);
        hipLaunchKernelGGL(ws_enc_tscan_kernel, dim3(1), dim3(1024), 0, st, tpre, B, (u64*)d_wire_off, nframes);
        hipLaunchKernelGGL(ws_enc_front_kernel, dim3(blocks), dim3(ENC_TILE), 0, st, d_src, d_frames, nframes, tpre, B,
                           (u64*)d_wire_off, ptr, npieces, d_dst, (u64)dst_capacity, fused);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("encode front launch", e);
    } else {
        // E1 hipcub scan -> E2 piece pointers (E4 after E3, or on a side stream)
        WireLen op{d_frames, nframes};
        hipcub::CountingInputIterator<u32> cnt(0);
        hipcub::TransformInputIterator<u64, WireLen, hipcub::CountingInputIterator<u32>> in(cnt, op);
        size_t scan_bytes = 0;
        if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, in, d_wire_off, nframes + 1, st)) != hipSuccess)
            return ws_set_err("hipcub scan (size)", e);
        const size_t ptr_off = (scan_bytes + 255) & ~(size_t)255;
        if ((rc = slot.encode_workspace(ptr_off + npieces * 4 + 16, &ws))) return rc;
        if ((e = hipcub::DeviceScan::ExclusiveSum(ws, scan_bytes, in, d_wire_off, nframes + 1, st)) != hipSuccess)
            return ws_set_err("hipcub scan", e);
        ptr = reinterpret_cast<u32*>(reinterpret_cast<unsigned char*>(ws) + ptr_off);
        hipLaunchKernelGGL(ws_enc_ptr_kernel, dim3((nframes + 1 + 255) / 256), dim3(256), 0, st, d_frames, nframes,
                           d_wire_off, ptr, lead0, npieces);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_enc_ptr_kernel launch", e);
    }
    if (npieces) {
        hipLaunchKernelGGL((ws_enc_copy_kernel<1, 0>), dim3((u32)npieces), dim3(ENC_T), 0, st, d_src, d_frames,
                           nframes, d_wire_off, ptr, d_dst, (u64)dst_capacity, (u32)npieces);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_enc_copy_kernel launch", e);
    }
    if (front) return 0;
    hipLaunchKernelGGL(ws_enc_edge_kernel, dim3((nframes + 255) / 256), dim3(256), 0, st, d_src, d_frames, nframes,
                       d_wire_off, d_dst, (u64)dst_capacity, fused);
    if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_enc_edge_kernel launch", e);
    return 0;
}
