// ws_common.h — shared device types and the RFC 6455 header parse used by every
// decode kernel (one definition, so the walker, the split walk kernel and the
// fallback paths cannot drift apart).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/wsframe_amd.h"

typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Global-address-space views: hot loops must emit global_load/store, not flat_*
// (flat ops complete out of order, so hipcc drains vmcnt+lgkmcnt before each one
// and every load becomes its own round trip).
// the unmask kernel's unit (ws_piece.hip K2, also behind the raw-stream path): one-shot
// 256-thread blocks over WS_PIECE_U KiB per wave, 2^WS_PIECE_SHIFT bytes per block
#ifndef WS_PIECE_U
#define WS_PIECE_U 4
#define WS_PIECE_SHIFT 14                   // 16 KiB = 256 threads * WS_PIECE_U * 16 B
#endif
#define WS_GLOBAL __attribute__((address_space(1)))
typedef WS_GLOBAL u32x4 gu32x4;
typedef WS_GLOBAL u32 gu32;
typedef WS_GLOBAL u64 gu64;
typedef WS_GLOBAL unsigned char gu8;
// Constant-address-space view: wave-uniform loads through it become s_load_*.
typedef __attribute__((address_space(4))) const u32 cu32;

template <typename T>
__device__ __forceinline__ WS_GLOBAL T* gptr(const void* p) {
    return reinterpret_cast<WS_GLOBAL T*>(reinterpret_cast<uintptr_t>(p));
}

// Cache policy of the payload stream (A/B-able): 0 plain, 1 nontemporal loads+stores, 2 nt stores,
// 4 nontemporal loads + the caller's own sc1|nt buffer stores (st16<4> is an nt store).
template <int NT>
__device__ __forceinline__ u32x4 ld16(const gu32x4* p) {
    if constexpr (NT == 1 || NT == 4) return __builtin_nontemporal_load(p);
    else return *p;
}
#ifndef WS_ST16_PLAIN
#define WS_ST16_PLAIN 0   // (A/B builds: 1 = every st16 a plain store)
#endif
template <int NT>
__device__ __forceinline__ void st16(u32x4 v, gu32x4* p) {
    if constexpr (NT >= 1 && !WS_ST16_PLAIN) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// A wave-uniform buffer descriptor over `bytes` from p, for `buffer_store_dwordx4 … nt sc1`
// stores at per-lane offsets (stores outside [0, bytes) are dropped by the hardware)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(uintptr_t p, u32 bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void st16_sc1nt(u32x4 v, __amdgpu_buffer_rsrc_t r, u32 off) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), r,
                                           (int)off, 0, 18);
}

__device__ __forceinline__ u32 rotl32(u32 x, u32 r) { return r ? (x << r) | (x >> (32 - r)) : x; }

// Result of parsing one frame header (websocketframe.c:112-165).
enum { WS_PARSE_INCOMPLETE = 0, WS_PARSE_FRAME = 1, WS_PARSE_WRAP = 2 };
struct WsHdr {
    int kind;      // WS_PARSE_*
    u32 b0, b1;    // header bytes 0 and 1
    u32 hdr;       // 2 + ext + mask
    u32 masked;    // MASK bit
    u32 key;       // little-endian masking key (valid if masked)
    u64 plen;      // payload length
    int ret;       // (int) return value (:164)
};

// h0 = header bytes 0..7, h1 = bytes 8..15 (little-endian), avail = bytes left (>= 2).
// Mirrors websocketframe.c:121-164 exactly, plus the batch fence: a MASKED frame
// whose u64 length sum wraps and would pass the :149 check is WS_PARSE_WRAP (the
// reference would unmask past the buffer: undefined behaviour).
__device__ __forceinline__ WsHdr ws_parse(u64 h0, u64 h1, u64 avail) {
    WsHdr r;
    r.b0 = (u32)h0 & 0xFFu;
    r.b1 = (u32)(h0 >> 8) & 0xFFu;
    const u32 p7 = r.b1 & 0x7Fu;                                   // :129
    r.masked = r.b1 >> 7;                                          // :126-127
    const u32 ext = p7 < 126 ? 0u : (p7 == 126 ? 2u : 8u);         // :134-145
    r.hdr = 2u + ext + (r.masked ? 4u : 0u);
    r.kind = WS_PARSE_INCOMPLETE;
    r.key = 0;
    r.plen = 0;
    r.ret = 0;
    if (avail < r.hdr) return r;                                   // :131,136,142
    if (ext == 0) r.plen = p7;
    else if (ext == 2) r.plen = ((h0 >> 16) & 0xFFu) << 8 | ((h0 >> 24) & 0xFFu);   // memReadBE16
    else r.plen = __builtin_bswap64((h0 >> 16) | (h1 << 48));                          // memReadBE64
    const u64 total = (u64)r.hdr + r.plen;                         // u64, may wrap (:149)
    if (avail < total) return r;                                   // :149-150
    if (r.masked && total < r.plen) { r.kind = WS_PARSE_WRAP; return r; }
    r.key = ext == 0 ? (u32)(h0 >> 16) : (ext == 2 ? (u32)(h0 >> 32) : (u32)(h1 >> 16));
    r.ret = (int)(u32)total;                                       // :164, truncating
    r.kind = WS_PARSE_FRAME;
    return r;
}

// Header bytes [p, p+16) from the 32 bytes x0|x1 loaded at floor16(p), o = p & 15,
// as two little-endian u64 (bytes 0..7, 8..15). Branch-free on purpose: a divergent
// per-lane dword select around these loads produced nondeterministic header reads
// under load on ROCm 7.2.
__device__ __forceinline__ void ws_hdr_from32(const u32x4 x0, const u32x4 x1, u32 o, u64& h0, u64& h1) {
    const u64 w0 = (u64)x0.x | ((u64)x0.y << 32), w1 = (u64)x0.z | ((u64)x0.w << 32);
    const u64 w2 = (u64)x1.x | ((u64)x1.y << 32), w3 = (u64)x1.z | ((u64)x1.w << 32);
    const u32 sh = 8u * (o & 7);
    const bool up = o >= 8;
    const u64 a0 = up ? w1 : w0, a1 = up ? w2 : w1, a2 = up ? w3 : w2;
    h0 = sh ? (a0 >> sh) | (a1 << (64 - sh)) : a0;
    h1 = sh ? (a1 >> sh) | (a2 << (64 - sh)) : a1;
}

// The wire length of the batch's first frame (of the first segment with >= 2 bytes among the
// first 8), 0 unless it is a plain complete frame: K1's first-step stride guess for the next
// call on the stream (ws_piece.hip; a wrong guess costs loads only). One thread.
__device__ __forceinline__ u32 ws_first_frame_len(const unsigned char* buf, const u64* seg_off, const u64* seg_len,
                                                  u32 nseg) {
    for (u32 s = 0; s < nseg && s < 8; ++s) {
        const u64 so = seg_off[s], sl = seg_len[s];
        if (sl < 2) continue;
        const uintptr_t pa = reinterpret_cast<uintptr_t>(buf + so);
        const WS_GLOBAL u32x4* q = reinterpret_cast<const WS_GLOBAL u32x4*>(pa & ~(uintptr_t)15);
        u64 h0, h1;
        ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
        const WsHdr h = ws_parse(h0, h1, sl);
        return h.kind == WS_PARSE_FRAME && h.ret > 1 && (u64)h.hdr + h.plen == (u64)(u32)h.ret ? (u32)h.ret : 0u;
    }
    return 0;
}

// Descriptor as two 16-B stores (WebsocketFrameDesc_t layout).
__device__ __forceinline__ void ws_store_desc(WebsocketFrameDesc_t* d, u64 frame_off, const WsHdr& h) {
    const u64 dof = h.plen ? frame_off + h.hdr : WEBSOCKET_DATA_OFF_NULL;
    u32x4 q0, q1;
    q0.x = (u32)frame_off; q0.y = (u32)(frame_off >> 32); q0.z = (u32)dof; q0.w = (u32)(dof >> 32);
    q1.x = (u32)h.plen; q1.y = (u32)(h.plen >> 32); q1.z = (u32)h.ret;
    q1.w = (h.b0 >> 7) | ((h.b0 & 0x0Fu) << 8) | (h.masked << 16) | (h.hdr << 24);
    gu32x4* g = gptr<u32x4>(d);
    g[0] = q0;
    g[1] = q1;
}

__device__ __forceinline__ void ws_store_res(WebsocketSegResult_t* res, u64 consumed, u32 nf, int status) {
    u32x4 r;
    r.x = (u32)consumed; r.y = (u32)(consumed >> 32); r.z = nf; r.w = (u32)status;
    *gptr<u32x4>(res) = r;
}

// Frame table entry in LDS for one round: the item's payload range relative to the
// round start, clamped to [-16, round bytes + 16] (so 32 bits suffice for any
// segment size), and its key pre-rotated for 16-B-aligned chunks: byte j of a
// chunk at offset x takes key[(x + j - p0) & 3] = byte (j & 3) of rotl(key, 8*(p0 & 3)).
// Unmasked / empty items keep their position with an empty range, so the table
// stays sorted and non-overlapping.
struct Item {
    int p0, p1;
    u32 rkey, pad;
};

// Store the bytes of w selected by cov (bit q = byte q) into the 16-B chunk at p: a
// dword store for every fully selected dword, byte stores only inside partial dwords
// (one lane issuing 16 byte stores per chunk was measured far slower than 16-B stores).
__device__ __forceinline__ void ws_store_bytes(WS_GLOBAL unsigned char* p, const u32x4 w, const u32 cov) {
    WS_GLOBAL u32* const pd = reinterpret_cast<WS_GLOBAL u32*>(p);
#pragma unroll
    for (u32 d = 0; d < 4; ++d) {
        const u32 nib = (cov >> (4 * d)) & 15u;
        const u32 v = d == 0 ? w.x : (d == 1 ? w.y : (d == 2 ? w.z : w.w));
        if (nib == 15u) {
            pd[d] = v;
        } else if (nib) {
#pragma unroll
            for (u32 b = 0; b < 4; ++b)
                if ((nib >> b) & 1u) p[4 * d + b] = (unsigned char)(v >> (8u * b));
        }
    }
}

// nibble n (n < 16) -> byte mask (bit i -> 0xFF in byte i): the multiply spreads bit i to
// bit 8i (the four shifted copies of n do not overlap), giving v_perm_b32 selector bytes
// 0x0C (-> 0x00) or 0x0D (-> 0xFF)
__device__ __forceinline__ u32 nib_to_bytemask(u32 n) {
    const u32 sel = ((n * 0x00204081u) & 0x01010101u) | 0x0C0C0C0Cu;
    return __builtin_amdgcn_perm(0u, 0u, sel);
}

// OR the XOR masks of the bytes [lo, hi) of a 16-B chunk (0 <= lo < hi <= 16) under `key`
// (rotated to the chunk's phase: chunk byte i takes key byte i & 3) into m0..m3, and their
// byte bits into cov. A chunk wholly inside the range — all but the frame-edge chunks —
// takes four ORs; the byte-mask build runs only when some lane of the wave has an edge.
__device__ __forceinline__ void ws_or_masks(u32 key, int lo, int hi, u32& m0, u32& m1, u32& m2, u32& m3, u32& cov) {
    if ((lo | (16 - hi)) == 0) {
        m0 |= key; m1 |= key; m2 |= key; m3 |= key;
        cov = 0xFFFFu;
        return;
    }
    const u32 bits = (0xFFFFu >> (16 - hi)) & (0xFFFFu << lo);
    cov |= bits;
    m0 |= key & nib_to_bytemask(bits & 15u);
    m1 |= key & nib_to_bytemask((bits >> 4) & 15u);
    m2 |= key & nib_to_bytemask((bits >> 8) & 15u);
    m3 |= key & nib_to_bytemask(bits >> 12);
}


// As ws_or_masks, XOR-ing straight into the chunk's data (the ranges of different frames
// never share a byte, so applying each frame's masks at once equals OR-ing them first):
// no mask registers. The data must be loaded — a wave that waits for its frame records
// (loaded after its payload) has its payload back anyway (vmcnt retires in order).
__device__ __forceinline__ void ws_xor_range(u32 key, int lo, int hi, u32x4& v, u32& cov) {
    if ((lo | (16 - hi)) == 0) {
        v.x ^= key; v.y ^= key; v.z ^= key; v.w ^= key;
        cov = 0xFFFFu;
        return;
    }
    const u32 bits = (0xFFFFu >> (16 - hi)) & (0xFFFFu << lo);
    cov |= bits;
    v.x ^= key & nib_to_bytemask(bits & 15u);
    v.y ^= key & nib_to_bytemask((bits >> 4) & 15u);
    v.z ^= key & nib_to_bytemask((bits >> 8) & 15u);
    v.w ^= key & nib_to_bytemask(bits >> 12);
}

// Chunk at round offset x straddles payload edges: OR the byte ranges of every
// table item from j on that touches it, XOR, and store exactly those bytes (one
// 16-B store if the chunk turns out fully covered).
template <int NT>
__device__ __forceinline__ void ws_store_partial(const u32x4 v, gu32x4* const pc, const Item* tab, u32 j,
                                                 const u32 cnt, const int x) {
    u32 m0 = 0, m1 = 0, m2 = 0, m3 = 0, cov = 0;
    for (u32 i = j; i < cnt; ++i) {
        const Item t = tab[i];
        if (t.p0 >= x + 16) break;
        const int lo = t.p0 > x ? t.p0 - x : 0, hi = t.p1 < x + 16 ? t.p1 - x : 16;
        if (hi <= lo) continue;
        ws_or_masks(t.rkey, lo, hi, m0, m1, m2, m3, cov);
    }
    u32x4 mm;
    mm.x = m0; mm.y = m1; mm.z = m2; mm.w = m3;
    const u32x4 w = v ^ mm;
    if (cov == 0xFFFFu) {
        st16<NT>(w, pc);
    } else if (cov) {
        ws_store_bytes(reinterpret_cast<gu8*>(pc), w, cov);
    }
}

// One round of the unmask over chunks [0, lim] of `rb` (data already loaded into v:
// lane `tid` holds chunk min(tid + u*T, lim) in v[u]). Wave w's slot u covers chunks
// [u*T + 64w, +64): a wave-uniform item cursor advances monotonically over the table
// (broadcast LDS reads) and each lane steps 0-1 items for its own chunk. Full chunks
// take one 16-B store; chunks straddling payload edges store exactly the payload
// bytes. Every chunk is stored by its owning lane only: clamped duplicates never store
// (another wave may already have stored that chunk: no double XOR).
template <int T, int U, int NT>
__device__ __forceinline__ void ws_xor_round(const u32x4 (&v)[U], gu32x4* const rb, const u32 lim, const Item* tab,
                                             const u32 cnt, const u32 tid) {
    const u32 wv = tid >> 6, ln = tid & 63;
    u32 icur = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32 lw = (u32)(u * T) + 64u * wv;               // wave-uniform first chunk
        if (lw > lim) break;
        while (icur < cnt && tab[icur].p1 <= (int)(lw * 16)) ++icur;
        const u32 lc = lw + ln;
        if (lc > lim) continue;   // clamped duplicate: never store (another wave may have stored it)
        const int x = (int)(lc * 16);
        u32 j = icur;
        Item it = tab[j < cnt ? j : 0];
        while (j < cnt && it.p1 <= x) { ++j; it = tab[j < cnt ? j : 0]; }
        if (j >= cnt || it.p0 >= x + 16) continue;              // no payload byte in this chunk
        gu32x4* const pc = rb + lc;
        if (it.p0 <= x && it.p1 >= x + 16) {
            st16<NT>(v[u] ^ it.rkey, pc);
            continue;
        }
        ws_store_partial<NT>(v[u], pc, tab, j, cnt, x);
    }
}

// ---------------------------------------------------------------------------------------------
// One round of the reactor loop (net_reactor.c:515-526) over a segment window staged in
// LDS, by stride speculation, for a whole wavefront: lane k parses the header at
// off + k*g (g = the last frame length; seeded with the length of the frame at `off`),
// the chain is right up to the first lane whose length differs (ballot), so a run of up
// to 64 equal frames costs one round. Window coordinates: X = segment offset + lead
// (lead = the segment's 16-B phase); the window holds X in [W0, W0 + 16*nchunks) and
// owns headers starting in [W0, W1) (W1 + 16 <= its end, so a header never passes it).
// Used by the one-workgroup-per-segment kernels (ws_segfuse.hip, ws_reasm.hip).
struct WsRound {
    WsHdr h;        // this lane's parse
    u64 pos;        // this lane's candidate frame offset (segment-relative)
    u32 mm;         // first lane that does not continue the chain (64: all continue)
    u32 code_m;     // its code: 0 continue, 1 consumed + new stride, 2 consumed + end (ret <= 0),
                    // 3 not consumed + end, 4 header past the window (continue in the next one)
    u32 ntake;      // lanes [0, ntake) consumed a frame (descriptor if ret != 0)
    int ret_m, st_m;
};

__device__ __forceinline__ WsRound ws_lds_round(const u32x4* win, u64 W0, u64 W1, u64 lead, u64 sl, u64 off,
                                                u64& g, u32 nf, u32 max_frames, u32 lane) {
    if (g == 0 && off + lead < W1 && off < sl) {                       // stride seed
        const u32 o = (u32)(off + lead - W0);
        u64 h0, h1;
        ws_hdr_from32(win[o >> 4], win[(o >> 4) + 1], o & 15u, h0, h1);
        const WsHdr h = ws_parse(h0, h1, sl - off);
        if (h.kind == WS_PARSE_FRAME && h.ret > 0) g = (u32)h.ret;
    }
    WsRound r;
    r.pos = off + (u64)lane * g;
    const bool cand = lane == 0 || g > 0;
    const u64 X = r.pos + lead;
    const bool inwin = X < W1;
    const bool eval = cand && r.pos < sl && inwin;
    const u32 o = eval ? (u32)(X - W0) : 0u;
    u64 h0, h1;
    ws_hdr_from32(win[o >> 4], win[(o >> 4) + 1], o & 15u, h0, h1);
    r.h = ws_parse(h0, h1, eval ? sl - r.pos : 0);
    u32 code = 3;
    int st = WEBSOCKET_SEG_OK;
    if (cand) {
        if (r.pos >= sl) code = 3;
        else if (nf + lane >= max_frames) { code = 3; st = WEBSOCKET_SEG_MAX_FRAMES; }
        else if (!inwin) code = 4;
        else if (sl - r.pos < 2) code = 3;                                 // websocketframe.c:121
        else if (r.h.kind == WS_PARSE_INCOMPLETE) code = 3;
        else if (r.h.kind == WS_PARSE_WRAP) { code = 3; st = WEBSOCKET_SEG_ERR_LEN_WRAP; }
        else if (r.h.ret <= 0) { code = 2; st = r.h.ret < 0 ? WEBSOCKET_SEG_ERR_DECODE : WEBSOCKET_SEG_OK; }
        else code = (u64)(u32)r.h.ret == g ? 0u : 1u;
    }
    const u64 stop = __ballot(code != 0);
    r.mm = stop ? (u32)__builtin_ctzll(stop) : 64u;
    const u32 src = r.mm < 64 ? r.mm : 63;
    r.code_m = r.mm < 64 ? (u32)__shfl((int)code, (int)src) : 0u;
    r.ret_m = __shfl(r.h.ret, (int)src);
    r.st_m = __shfl(st, (int)src);
    r.ntake = r.mm + ((r.code_m == 1 || r.code_m == 2) ? 1u : 0u);
    return r;
}

// Advance the loop state past a round; false = no more rounds in this window (the walk
// ended: walking = false, or the next header lies in the next window).
__device__ __forceinline__ bool ws_round_advance(const WsRound& r, u64& off, u64& g, u32& nf, int& status,
                                                 bool& walking) {
    if (r.mm == 64) { nf += 64; off += 64 * g; return true; }
    const u64 pos_m = off + (u64)r.mm * g;
    nf += r.mm;
    if (r.code_m == 1) { nf += 1; off = pos_m + (u32)r.ret_m; g = (u32)r.ret_m; return true; }
    off = pos_m;
    if (r.code_m == 4) return false;
    if (r.code_m == 2 && r.ret_m != 0) nf += 1;                        // ret < 0 keeps its descriptor
    status = r.st_m;
    walking = false;
    return false;
}

// host side
// a launch-tuning option (websocketframeGpuSetOption): atomic, so concurrent calls and
// SetOption never race; each launcher reads the knobs it needs once per call
typedef std::atomic<int> WsOpt;
int ws_set_err(const char* what, hipError_t e);
int ws_set_msg(const char* msg);

// kernel launchers (one per translation unit)
struct WsLaunch {
    unsigned char* buf;
    const u64* seg_off;
    const u64* seg_len;
    u32 nseg;
    u32 max_frames;
    const u64* desc_base;
    WebsocketFrameDesc_t* desc;
    WebsocketSegResult_t* res;
    hipStream_t stream;
    int cus;
    int lds_per_cu;       // bytes of LDS per CU (hipDeviceProp_t::maxSharedMemoryPerMultiProcessor)
    int pwin = -1;        // K2's log2 piece windows for this call (-1: the batch rule, piece_wshift)
};
int ws_launch_walker(const WsLaunch& L, const u32* gate = nullptr, u32 gate_gen = 0);
size_t ws_piece_workspace_bytes(u64 span, u32 nseg, u32 max_frames);
struct WsSegRec {         // K1 -> K2: one rx segment, origin-relative [lo, hi) (< 2^48, as the items)
    u64 w0, w1;           // and its item count: w0 = lo | cnt[15:0] << 48, w1 = hi | cnt[31:16] << 48
};                        // (one 16-B scalar load in K2 instead of three dependent ones)
struct PieceWs {          // ws_piece.hip workspace views after K1
    u32* disorder;
    u32* nonuni;          // K1's count of segments with frames of several lengths (K2 reads + clears)
    u64* ptr;
    u32* nwork;           // items per segment (frames walked, incl. an unconsumed ret==0 frame)
    u32x4* items;         // per descriptor slot s*max_frames+k: P0|rk_lo<<48, P1|rk_hi<<48 (origin-relative)
    WsSegRec* segr = nullptr;   // per segment (K1 writes it; the raw-stream path leaves it null)
    u64 npieces, pbase, c_lo, c_hi;
};
int ws_launch_piece_scan(const WsLaunch& L, u64 lo, u64 hi, unsigned char* ws, u32 gen, PieceWs* out,
                         bool count_nonuniform = false, u32 g0 = 0);
int ws_launch_piece_unmask(const WsLaunch& L, const PieceWs& P, u32 gen, int* advice = nullptr, u32 g0 = 0);
int ws_piece_dyn_lds(const WsLaunch& L, u64 npieces, u32 g0 = 0);
u32 ws_next_gen();
int ws_device_info(int* cus, int* lds_per_cu);
// auxiliary workspace: device scratch whose first WS_AUX_HEAD bytes are zero at allocation +
// pinned, device-visible host scratch (eager calls)
#define WS_AUX_HEAD 256
// zeroed at allocation (and when a capture adopts a slot): the head and the 256 B after it, where
// the raw stream's device walk keeps its plan (RwPlan::seen_max is read before its first write)
#define WS_AUX_ZERO (WS_AUX_HEAD + 512)
#define WS_SIDE_EVENTS 4          // the raw stream's split walk: side start + one per part (RW_NP 3)
struct WsAux {
    void* d;              // device scratch
    void* h;              // pinned host scratch (nullptr until requested)
    void* h_dev;          // its device address
    bool* state_ok;       // the owner's flag: the head holds a resting state
};
// The workspace slot of (HIP stream, graph capture), pinned for one call (ws_api.hip): every
// buffer a call needs comes from the one slot it acquired, and LRU eviction never takes a
// pinned slot. Buffers grow on demand (eagerly: after draining the stream).
struct WsStreamWs;
struct WsSlot {
    WsStreamWs* w = nullptr;
    hipStream_t st = nullptr;
    int cus = 0, lds = 0;
    ~WsSlot();
    int acquire(hipStream_t stream);
    void release();
    int workspace(size_t bytes, size_t zero_bytes, void** out);   // decode / reassembly / stream
    int encode_workspace(size_t bytes, void** out);
    int aux(size_t dbytes, size_t hbytes, WsAux* out);
    int advice(int** host, int** dev);                             // the stride hint words (eager)
    int side(hipStream_t* side, hipEvent_t* ev, int prio);         // the raw stream's split walk: side stream + events
};
bool ws_capturing(hipStream_t stream);
int ws_launch_piece(const WsLaunch& L, u64 lo, u64 hi, unsigned char* ws, u32 gen, int* advice,
                    const u32** disorder_out, bool* fallback_needed, u32 g0 = 0);
// the batch decode with every segment inside [lo, hi) of buf (ws_api.hip); `ws`
// (optional) is a caller-owned workspace of ws_decode_workspace_bytes() bytes whose
// first 16 bytes were zeroed once after allocation, else the per-device one is used
// (concurrent calls on one device must then not overlap)
int ws_decode_range(unsigned char* buf, u64 lo, u64 hi, const u64* seg_off, const u64* seg_len, u32 nseg,
                    u32 max_frames, const u64* desc_base, WebsocketFrameDesc_t* desc, WebsocketSegResult_t* res,
                    hipStream_t stream, void* ws = nullptr, size_t ws_bytes = 0);
size_t ws_decode_workspace_bytes(u64 span, u32 nseg, u32 max_frames);
int ws_launch_segfuse(const WsLaunch& L);
bool ws_segfuse_fits(u64 span, u32 nseg, u32 max_frames);

// Block -> work item with the items split into 2^wsh windows of ppw items streamed side by side
// (block b takes item (b mod 2^wsh) * ppw + b / 2^wsh; wsh = 0 keeps b): two distant address
// windows in flight beat one compact window on this HBM (tools/exp_win.sh).
__device__ __forceinline__ u32 ws_winn(u32 b, u32 wsh, u32 ppw) {
    return wsh ? (b & ((1u << wsh) - 1u)) * ppw + (b >> wsh) : b;
}
// the grid of ws_winn for n items in 2^wsh windows (fewer windows for small n): {wsh, ppw, blocks}
struct WsWinGrid { u32 wsh, ppw, blocks; };
static inline WsWinGrid ws_win_grid(u32 n, int opt) {
    u32 wsh = opt > 0 && opt <= 3 ? (u32)opt : 0u;
    while (wsh && (n >> wsh) < 256) --wsh;                 // (two windows from 512 items, as before)
    const u32 ppw = wsh ? (u32)(((u64)n + (1u << wsh) - 1) >> wsh) : n;
    return WsWinGrid{wsh, ppw, wsh ? ppw << wsh : n};
}
extern WsOpt ws_seg_win;
