// ws_piece.hip — decode as "walk, then one-shot unmask over fixed 16 KiB pieces".
//
// The streaming ceiling of this part for an in-place read+write is reached only by
// ONE-SHOT waves (load once, store once, exit): every persistent pattern measured
// stays near 5.0–5.5 TB/s, while one-shot 256x4 blocks reach 5.9–6.1 TB/s, even
// with a chain of 4 dependent table lookups resolved while their payload loads are
// in flight (tools/calib.py modes 4, 5, 40-49, 60-65).
//
// K1 ws_piece_scan_kernel — 16 lanes per rx segment run the reactor loop
//   (net_reactor.c:515-526) over websocketframeDecode's header logic
//   (websocketframe.c:112-165, ws_parse) by stride speculation. Writes the descriptors
//   and segment result, one payload item per frame (origin-relative [P0, P1) +
//   pre-rotated key, indexed like the descriptor slot s*max_frames + k), the item count
//   per segment, and for every 16 KiB piece whose first byte lies in this segment's
//   ownership range [end of segment s-1, end of segment s) the first item that can touch
//   it. A segment that starts before the previous one ends (or lies outside [lo, hi))
//   marks the batch unordered. It also counts the segments whose frames are not all of
//   the first frame's length (or that stop on an error): K2 turns that count into the
//   host's hint for the next call's first step (g0 below: the first frame's length, used
//   only while nearly every segment is uniform).
// K2 ws_piece_unmask_kernel — one 256-thread block per piece, 4 chunks per lane:
//   payload loads first, then (while they are in flight) the piece pointer and the
//   items it leads to (16, then 64 per load, hopping to the next segment when the piece
//   extends past the current one), XOR masks accumulated per chunk, one 16-B store
//   per fully covered chunk, exact byte stores at payload edges. Every piece is
//   touched by exactly one block, so no byte is stored twice.
// Fallback: if the segments are not in ascending buffer order, K2 stores nothing and a
//   gated walker (ws_walker.hip) decodes the batch.
#include <mutex>
#include <vector>

#include "ws_walk.h"

#define PIECE_T 256
#define PIECE_U WS_PIECE_U
#define PIECE_SHIFT WS_PIECE_SHIFT
static_assert((1 << PIECE_SHIFT) == PIECE_T * PIECE_U * 16, "piece = one block's chunks");
#define PIECE_NONE 0xFFFFFFFFFFFFFFFFull

// item: w0 = P0 | rkey[15:0] << 48, w1 = P1 | rkey[31:16] << 48 (origin-relative bytes < 2^48)
__device__ __forceinline__ void put_item(gu32x4* it, u64 p0, u64 p1, u32 rk) {
    const u64 w0 = p0 | ((u64)(rk & 0xFFFFu) << 48), w1 = p1 | ((u64)(rk >> 16) << 48);
    u32x4 q;
    q.x = (u32)w0; q.y = (u32)(w0 >> 32); q.z = (u32)w1; q.w = (u32)(w1 >> 32);
    *it = q;
}

// pieces whose first byte is in [lo, hi) (origin-relative) get s << 32 | k; only pieces of the
// batch's table [pbase, pend) exist (a segment outside [lo, hi) of the call marks the batch
// unordered, and its pointers are clipped here). start, stride: the lanes of a group write one
// range together, lane j the pieces j, j + stride, ...
__device__ __forceinline__ u64 first_piece(u64 lo, u64 pbase) {
    const u64 p = (lo + (1ull << PIECE_SHIFT) - 1) >> PIECE_SHIFT;
    return p > pbase ? p : pbase;
}
__device__ __forceinline__ void put_ptrs(u64* ptr, u64 pbase, u64 pend, u64 lo, u64 hi, u32 s, u32 k, u64 start = 0,
                                         u64 stride = 1) {
    for (u64 p = first_piece(lo, pbase) + start; (p << PIECE_SHIFT) < hi && p < pend; p += stride)
        *gptr<u64>(ptr + (p - pbase)) = ((u64)s << 32) | k;
}

// What one segment walk needs (K1).
struct WalkArgs {
    const unsigned char* buf;
    const u64* seg_off;
    const u64* seg_len;
    u32 nseg, max_frames;
    const u64* desc_base;
    WebsocketFrameDesc_t* desc;
    WebsocketSegResult_t* res;
    u32x4* items;
    u64* ptr;
    u32* nwork;
    WsSegRec* segr;
    u32* disorder;
    u32 gen;
    u64 pbase, lo, hi;
    u32 g0;
    u32 alpha_ok;         // option "scan_alpha": alphabet speculation allowed
};

// G = 16 lanes per segment, header walk by STRIDE SPECULATION: lane k of the group parses the
// header at off + k*g (g = the last frame's length); the chain is right up to the first lane
// whose frame length differs (ballot), so a run of up to G equal frames is walked in one round
// trip and its items, descriptors and piece pointers are written by the lanes in parallel. 16
// keeps four segments in flight per wave (the walk is latency-bound; 8, 32, 64 lanes and one
// lane per segment measured slower in round 1). The group's segment is s (active groups); on
// return lane gl == 0 of the group holds its item count and whether its frames were not all of
// one length (or it stopped on an error).
#define WALK_G 16
#define WALK_PTR_OWN 64   // piece pointers of its frame a lane writes alone (the rest: the group; with 4, cfg4 ran 7 % slower: profiles/r04_ptr_own_ab.log)

// ST (measurement builds only, WS_K1_VARIANTS; the product is ST 15): which of K1's stores are made —
// 1 descriptors, 2 items, 4 piece pointers, 8 the per-segment records (result, count, WsSegRec)
template <int ST = 15>
__device__ __forceinline__ void walk_group(const WalkArgs& A, u32 s, bool active, u32 lane, u32& cnt_out,
                                           bool& nonu_out) {
    constexpr u32 G = WALK_G;
    const u32 gl = lane % G, gb = lane - gl;                                 // lane in group, group's first lane
    const u32 sc = active ? s : A.nseg - 1;                                  // inactive groups: harmless loads
    const u64 lead0 = reinterpret_cast<uintptr_t>(A.buf) & 15;
    const u64 pend = A.hi + lead0 ? ((A.hi + lead0 - 1) >> PIECE_SHIFT) + 1 : 0;   // end of the piece table
    const u64 so = A.seg_off[sc], sl = A.seg_len[sc];
    const u64 prev_end = sc ? A.seg_off[sc - 1] + A.seg_len[sc - 1] : 0;
    if (active && gl == 0 && (prev_end > so || so < A.lo || so > A.hi || sl > A.hi - so))
        *gptr<u32>(A.disorder) = A.gen;
    const u64 dbase = A.desc_base ? A.desc_base[sc] : (u64)sc * A.max_frames;
    const u64 ibase = (u64)sc * A.max_frames;
    const u64 sorg = so + lead0;
    const uintptr_t seg = reinterpret_cast<uintptr_t>(A.buf + so);
    if ((ST & 4) && active) put_ptrs(A.ptr, A.pbase, pend, sc ? prev_end + lead0 : 0, sorg, sc, 0, gl, G);
    // g0: the stride guess of the first step (the host's hint, 0 = none): lane k parses off + k*g0
    // at once; lane 0's frame is always the true first one, so a wrong guess costs nothing but
    // its loads (code 1 at lane 0 takes the true length)
    u64 off = 0, g = A.g0, walked_end = sorg;
    u32 nf = 0, extra = 0;
    int status = WEBSOCKET_SEG_OK;
    bool nonu = false;                       // frames of another length than the first, or an error stop
    const u64 gmask = (1ull << G) - 1;
    // ALPHABET SPECULATION (lengths that keep changing, e.g. cfg3): once a step ends after one
    // frame of a new length, the lanes speculate over the lengths seen so far (L0..L2, na of them)
    // instead of one stride: lane 0 parses the frame at off, lanes 1..na the frame after it for
    // each length, the next lanes the frame after that for each pair (and, with two lengths, each
    // triple) — 13 lanes cover three frames (15 cover four) while the lengths stay in the
    // alphabet, where stride lanes confirm one or two. A chain of three equal lengths goes back
    // to stride speculation.
    bool alpha = false;
    u32 L0 = 0, L1 = 0, L2 = 0, na = 0, rep = 0;
    // (selects only: an indexed form becomes a scratch array)
    auto add_len = [&](u32 x) {
        const bool add = x != 0 && x != L0 && !(na > 1 && x == L1) && !(na > 2 && x == L2);
        const u32 at = na < 3 ? na : rep;                                   // fill, then replace round-robin
        L0 = add && at == 0 ? x : L0;
        L1 = add && at == 1 ? x : L1;
        L2 = add && at == 2 ? x : L2;
        rep = add && na == 3 ? (rep == 2 ? 0u : rep + 1) : rep;
        na = add && na < 3 ? na + 1 : na;
    };
    auto len_at = [&](u32 i) -> u64 { return (u64)(i == 0 ? L0 : (i == 1 ? L1 : L2)); };
    while (__ballot(active)) {
        // this lane's candidate: its frame offset and its depth in the chain
        u64 pos = off;
        u32 depth = 0;
        bool cand = active;
        if (!alpha) {
            pos = off + (u64)gl * g;
            depth = gl;
            cand = active && (gl == 0 || g > 0);
        } else if (gl >= 1) {
            const u32 q = gl - 1;
            if (q < na) {
                depth = 1;
                pos = off + len_at(q);
            } else if (q - na < na * na) {
                const u32 r = q - na;
                depth = 2;
                pos = off + len_at(r / na) + len_at(r % na);
            } else if (na == 2 && q - 6 < 8) {
                const u32 r = q - 6;
                depth = 3;
                pos = off + len_at(r >> 2) + len_at((r >> 1) & 1) + len_at(r & 1);
            } else {
                cand = false;
            }
        }
        const bool eval = cand && pos < sl;
        const uintptr_t pa = seg + (eval ? pos : 0);
        const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
        const u32x4 x0 = q[0], x1 = q[1];                                  // WEBSOCKET_BATCH_PAD: readable
        u64 h0, h1;
        ws_hdr_from32(x0, x1, (u32)(pa & 15), h0, h1);
        const WsHdr h = ws_parse(h0, h1, eval ? sl - pos : 0);
        // per-lane outcome in the reactor loop's order (net_reactor.c:515-526):
        //   0 consumed, chain continues   1 consumed, length != g: step ends (stride lanes)
        //   2 consumed, walk ends (ret <= 0)   3 not consumed, walk ends
        u32 code = 3;
        int st = WEBSOCKET_SEG_OK;
        if (cand) {
            if (pos >= sl) code = 3;
            else if (nf + depth >= A.max_frames) { code = 3; st = WEBSOCKET_SEG_MAX_FRAMES; }
            else if (sl - pos < 2) code = 3;                                 // websocketframe.c:121
            else if (h.kind == WS_PARSE_INCOMPLETE) code = 3;
            else if (h.kind == WS_PARSE_WRAP) { code = 3; st = WEBSOCKET_SEG_ERR_LEN_WRAP; }
            else if (h.ret <= 0) { code = 2; st = h.ret < 0 ? WEBSOCKET_SEG_ERR_DECODE : WEBSOCKET_SEG_OK; }
            else code = alpha || (u64)(u32)h.ret == g ? 0u : 1u;
        }
        // the chain: mm = frames before the stopping one (G: none stops), the stopping lane's code,
        // and (alpha) the chain's lanes by depth
        u32 mm, code_m, lm = 0;
        u32 cl1 = 0, cl2 = 0, cl3 = 0;
        if (!alpha) {
            const u64 stop = (__ballot(code != 0) >> gb) & gmask;
            mm = stop ? (u32)__builtin_ctzll(stop) : G;                      // first non-continuing lane
            lm = mm < G ? mm : G - 1;
            code_m = mm < G ? (u32)__shfl((int)code, (int)(gb + lm)) : 0u;
        } else {
            // walk the tree: depth t's lane continues to the child for its length, if any
            const u32 maxd = na == 2 ? 3u : 2u;
            u32 lc = 0, qi = 0, t = 0;
            code_m = 1;                                                     // "stops after a consumed frame"
            for (;; ++t) {
                const u32 c = (u32)__shfl((int)code, (int)(gb + lc));
                if (c != 0) { code_m = c; break; }                          // 2 or 3: the walk ends here
                const u32 r = (u32)__shfl(h.ret, (int)(gb + lc));
                const u32 idx = r == L0 ? 0u : (na > 1 && r == L1 ? 1u : (na > 2 && r == L2 ? 2u : 3u));
                if (idx == 3u || t == maxd) break;                          // next length unknown: round ends
                qi = t == 0 ? idx : qi * na + idx;
                lc = t == 0 ? 1 + qi : (t == 1 ? 1 + na + qi : 1 + na + na * na + qi);
                if (t == 0) cl1 = lc; else if (t == 1) cl2 = lc; else cl3 = lc;
            }
            mm = t;
            lm = lc;
        }
        const int ret_m = __shfl(h.ret, (int)(gb + lm));
        const int st_m = __shfl(st, (int)(gb + lm));
        const u32 ntake = active ? mm + ((code_m == 1 || code_m == 2) ? 1u : 0u) : 0u;
        // this lane's frame is consumed: its index in the segment is nf + depth
        const bool mine = alpha ? depth < ntake && gl == (depth == 0 ? 0u : (depth == 1 ? cl1 : (depth == 2 ? cl2 : cl3)))
                                : gl < ntake;
        const u64 fo = sorg + pos;
        const u64 p0 = fo + h.hdr, fe = p0 + h.plen;
        if (mine) {                                                         // consumed frames, in parallel
            if (ST & 2)
                put_item(gptr<u32x4>(A.items + ibase + nf + depth), p0, h.masked ? fe : p0,
                         rotl32(h.key, 8u * (u32)(p0 & 3)));
            if ((ST & 1) && h.ret != 0) ws_store_desc(A.desc + dbase + nf + depth, so + pos, h);
        }
        // the pieces whose first byte lies in a consumed frame point at it: a lane writes its frame's
        // first WALK_PTR_OWN pieces; a longer frame's rest the group's 16 lanes write together
        // (one lane alone would take milliseconds over a multi-GiB frame)
        const u64 pf = first_piece(fo, A.pbase);
        const u64 phi = (fe + (1ull << PIECE_SHIFT) - 1) >> PIECE_SHIFT;   // pieces [pf, phi) start in [fo, fe)
        const u64 pl = phi < pend ? phi : pend;
        if ((ST & 4) && mine) {
            const u64 hown = pf + WALK_PTR_OWN < pl ? (pf + WALK_PTR_OWN) << PIECE_SHIFT : fe;
            put_ptrs(A.ptr, A.pbase, pend, fo, hown, sc, nf + depth);
        }
        bool pending = (ST & 4) && mine && pf + WALK_PTR_OWN < pl;
        while (__ballot(pending)) {
            const u64 gm = (__ballot(pending) >> gb) & gmask;
            const u32 li = gm ? (u32)__builtin_ctzll(gm) : 0u;
            const u32 src = gb + li;
            const u64 a = __shfl(fo, (int)src), b = __shfl(fe, (int)src);
            const u32 kk = nf + (u32)__shfl((int)depth, (int)src);
            if (gl == li) pending = false;
            if (gm) put_ptrs(A.ptr, A.pbase, pend, a, b, sc, kk, WALK_PTR_OWN + gl, WALK_G);
        }
        // the last consumed frame's lane: the stopping lane if it consumed, else the one before it
        const u32 llast = (code_m == 1 || code_m == 2 || mm == G) ? lm
                          : (alpha ? (mm == 1 ? 0u : (mm == 2 ? cl1 : (mm == 3 ? cl2 : cl3))) : (mm ? mm - 1 : 0u));
        const u64 fe_last = __shfl(fe, (int)(gb + llast));
        const u64 pos_m = __shfl(pos, (int)(gb + lm));
        if (ntake) walked_end = fe_last;
        if (!active) continue;
        // (a walk whose next frame would start at or past the segment's end stops now: the next
        // round's lane 0 would find pos >= sl and stop there with status OK)
        if (!alpha && mm == G) {                                            // the whole step continued
            nf += G;
            off += G * g;
            add_len((u32)g);
            if (off < sl) continue;
        } else if (code_m == 1) {                                           // consumed, next length unknown
            nf += mm;
            if (!alpha) {
                if (nf) nonu = true;
                if (mm) add_len((u32)g);
                add_len((u32)ret_m);
                // a step that confirmed one frame of a new length: lengths keep changing
                alpha = mm == 0 && nf > 0 && na >= 2 && A.alpha_ok;
                g = (u32)ret_m;
            } else {
                // a chain of three or more equal lengths: back to stride speculation
                const u32 r0 = (u32)__shfl(h.ret, (int)gb);
                if (mm >= 2 && r0 == (u32)ret_m && (u32)__shfl(h.ret, (int)(gb + cl1)) == r0) {
                    alpha = false;
                    g = (u32)ret_m;
                }
                add_len((u32)ret_m);
            }
            nf += 1;
            off = pos_m + (u32)ret_m;
            if (off < sl) continue;
        } else {
            nf += mm;
            off = pos_m;
            if (code_m == 2) {
                if (ret_m != 0) nf += 1;                                    // ret < 0 keeps its descriptor
                else extra = 1;                                             // ret == 0: unmasked, not counted
                nonu = true;
            }
            status = st_m;
            if (st_m == WEBSOCKET_SEG_ERR_LEN_WRAP) nonu = true;
        }
        active = false;
        // the group's 16 lanes together: the pieces starting in its tail, and past the batch's last
        // segment
        if (ST & 4) {
            const u32 cnt = nf + extra;
            put_ptrs(A.ptr, A.pbase, pend, walked_end, sorg + sl, sc, cnt, gl, G);
            if (sc == A.nseg - 1) put_ptrs(A.ptr, A.pbase, pend, sorg + sl, A.hi + lead0, 0xFFFFFFFFu, 0xFFFFFFFFu, gl, G);
        }
        if (!(ST & 8) && gl == 0 && nf + extra == 0xFFFFFFFFu) *gptr<u32>(A.nwork) = off;   // keeps the walk live
        if ((ST & 8) && gl == 0) {
            const u32 cnt = nf + extra;
            ws_store_res(A.res + sc, off, nf, status);
            *gptr<u32>(A.nwork + sc) = cnt;
            put_item(gptr<u32x4>(reinterpret_cast<u32x4*>(A.segr + sc)), sorg, sorg + sl, cnt);   // WsSegRec
            cnt_out = cnt;
            nonu_out = nonu;
        }
    }
}

// K1: one walk per segment (16 lanes each); counts the segments whose frames are not all of one
// length for the K2 that follows (nonuni, may be null)
#define PSCAN_T 256
__global__ __launch_bounds__(PSCAN_T) void ws_piece_scan_kernel(WalkArgs A, u32* nonuni) {
    const u32 lane = threadIdx.x & 63;
    const u32 s = (blockIdx.x * PSCAN_T + threadIdx.x) / WALK_G;
    u32 cnt = 0;
    bool nonu = false;
    walk_group(A, s, s < A.nseg, lane, cnt, nonu);
    if (nonuni) {                                                           // one atomic per wave, if any
        const u64 b = __ballot(lane % WALK_G == 0 && s < A.nseg && nonu);
        if (lane == 0 && b) atomicAdd(nonuni, (u32)__popcll(b));
    }
}

// K2. Kept configuration (the A/B variants of rounds 1-2 are gone: plain loads/stores,
// exact-byte-only or one-segment whole stores, forced 7-8 waves/SIMD, other window maps —
// all measured slower): nontemporal loads, nontemporal system-coherent (sc1)
// whole-chunk stores (NT 4), chunks wholly inside segments stored whole (byte coverage by the
// visited segments), 2^wshift windows.
template <int NT, int SR>
__global__ __launch_bounds__(PIECE_T) void ws_piece_unmask_kernel(unsigned char* __restrict__ buf,
                                                                  const u64* __restrict__ seg_off,
                                                                  const u64* __restrict__ seg_len, u32 nseg,
                                                                  u32 max_frames, const u32x4* __restrict__ items,
                                                                  const u32* __restrict__ nwork,
                                                                  const u64* __restrict__ ptr,
                                                                  const u32* __restrict__ disorder, u32 gen, u64 pbase,
                                                                  u64 c_lo, u64 c_hi, const u64* __restrict__ desc_base,
                                                                  WebsocketFrameDesc_t* __restrict__ desc,
                                                                  WebsocketSegResult_t* __restrict__ res,
                                                                  u32 wshift, u64 ppw, u64 npieces, u32* nonuni,
                                                                  int* advice, const WsSegRec* __restrict__ segr) {
    const u32 tid = threadIdx.x, lane = tid & 63;
    const u32 wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    // block -> piece: the pieces form 2^wshift windows of ppw pieces streamed side by side
    // (block b takes piece (b mod W) * ppw + b / W); blocks past the last piece load a
    // clamped piece and store nothing
    const u32 bx = blockIdx.x;
    // (round 5: odd windows streamed from their end measured +0.15 % on cfg2 and +0.7 % on cfg3,
    // profiles/r05_piece_dir_place.log)
    const u64 pw = (u64)(bx & ((1u << wshift) - 1u)) * ppw + (bx >> wshift);
    const bool pvalid = pw < npieces;
    const u64 pidx = pvalid ? pw : npieces - 1;
    const u64 pc0 = (pbase + pidx) << (PIECE_SHIFT - 4);                     // first chunk of the piece
    const u64 wc0 = pc0 + (u64)wv * (64 * PIECE_U);                          // this wave's 4 KiB: 256 chunks
    gu32x4* const base = reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(buf) & ~(uintptr_t)15);
    // ---- 1. payload loads (unconditional, clamped to the batch's chunks [c_lo, c_hi))
    u32x4 v[PIECE_U];
#pragma unroll
    for (int u = 0; u < PIECE_U; ++u) {
        const u64 c = wc0 + (u64)(u * 64 + lane);
        v[u] = ld16<NT>(base + (c < c_lo ? c_lo : (c < c_hi ? c : c_hi - 1)));
    }
    // ---- 2. items that touch this wave's range [r0, r1) (origin-relative bytes)
    constexpr long long RW = 64 * PIECE_U * 16;                             // this wave's bytes
    const u64 r0 = wc0 << 4, r1 = r0 + RW;
    const u64 pv = *reinterpret_cast<const __attribute__((address_space(4))) u64*>(
        reinterpret_cast<uintptr_t>(ptr + pidx));
    // the next piece's first item: when it is in the same segment, the items that touch this
    // piece are exactly [k, k_next], so the first load takes only those (long segments would
    // otherwise load 16 per wave however few they need)
    const u64 pn = pidx + 1 < npieces ? *reinterpret_cast<const __attribute__((address_space(4))) u64*>(
                                            reinterpret_cast<uintptr_t>(ptr + pidx + 1))
                                      : PIECE_NONE;
    const u32 ok = *reinterpret_cast<const cu32*>(reinterpret_cast<uintptr_t>(disorder)) != gen;
    u32 cov[PIECE_U];
#pragma unroll
    for (int u = 0; u < PIECE_U; ++u) cov[u] = 0;
    // no early return: an exit branch here would be hoisted above the payload loads
    u32 s = ok && pvalid && pv != PIECE_NONE ? (u32)(pv >> 32) : nseg, k = (u32)pv, step = 16;
    bool exact = false;                                                     // the first load holds them all
    if (s < nseg && pn != PIECE_NONE && (u32)(pn >> 32) == s && (u32)pn >= k && (u32)pn - k < 16u) {
        step = (u32)pn - k + 1;
        exact = true;
    }
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    const int xl = (int)lane * 16;                                          // lane's byte offset in a 1 KiB row
    // Chunks that hold payload bytes and lie wholly inside segments are stored whole
    // (bytes the decode does not change are written back unchanged: one 16-B store
    // instead of byte stores; byte coverage by the visited segments, so chunks spanning
    // two adjacent segments count too); others get exact byte stores.
    u32 segcov[PIECE_U];
#pragma unroll
    for (int u = 0; u < PIECE_U; ++u) segcov[u] = 0;
    bool first = true;
    while (s < nseg) {
        // the segment: SR = K1's 32-B record (one scalar load), else the caller's tables
        u64 slo, shi;
        u32 cnt;
        if (SR) {
            const u32x4 R = *reinterpret_cast<const __attribute__((address_space(4))) u32x4*>(
                reinterpret_cast<uintptr_t>(segr + s));
            const u64 w0 = (u64)R.x | ((u64)R.y << 32), w1 = (u64)R.z | ((u64)R.w << 32);
            slo = w0 & 0xFFFFFFFFFFFFull; shi = w1 & 0xFFFFFFFFFFFFull;
            cnt = (u32)(w0 >> 48) | ((u32)(w1 >> 48) << 16);
        } else {
            // (the raw-stream path) the three loads issued together: the compiler would otherwise sink
            // the second and third below the `slo >= r1` exit, three dependent round trips per wave
            const u64 so = seg_off[s], sl = seg_len[s];
            const u32 nw = nwork[s];
            asm volatile("" ::"s"(so), "s"(sl), "s"(nw));
            slo = so + lead0; shi = slo + sl; cnt = nw;
        }
        if (!first && slo >= r1) break;                                     // the next segment starts past us
        first = false;
        {
            // segment bytes relative to this wave's range, clamped to [-16, RW + 16]
            const long long sa = (long long)(slo - r0), sb = (long long)(shi - r0);
            const int SA = (int)(sa < -16 ? -16 : (sa > RW + 16 ? RW + 16 : sa));
            const int SB = (int)(sb < -16 ? -16 : (sb > RW + 16 ? RW + 16 : sb));
#pragma unroll
            for (int u = 0; u < PIECE_U; ++u) {
                const int x = u * 1024 + xl;
                const int lo = SA > x ? (SA - x < 16 ? SA - x : 16) : 0;
                const int hi = SB > x ? (SB - x < 16 ? SB - x : 16) : 0;
                if (hi > lo) segcov[u] |= (0xFFFFu >> (16 - hi)) & (0xFFFFu << lo);
            }
        }
        if (k < cnt) {
            // items load `step` at a time: 16 first (a 4 KiB wave range rarely needs more), 64
            // after that — all 64 lanes loading would fetch 1 KiB of items per wave in long segments
            const u32 j = k + lane;
            const bool valid = j < cnt && lane < step;
            u32x4 q = {0, 0, 0, 0};
            if (valid) q = items[(u64)s * max_frames + j];
            const u64 w0 = (u64)q.x | ((u64)q.y << 32), w1 = (u64)q.z | ((u64)q.w << 32);
            const u64 P0 = w0 & 0xFFFFFFFFFFFFull, P1 = w1 & 0xFFFFFFFFFFFFull;
            const u32 rk = (u32)(w0 >> 48) | ((u32)(w1 >> 48) << 16);
            // items are in address order: the first one starting at/after r1 ends the scan
            const u64 past = __ballot(valid && P0 >= r1);
            const u32 nlim = past ? (u32)__builtin_ctzll(past) : 64u;
            // wave-relative item range, clamped to [-16, RW + 16] (32-bit from here on)
            const long long ra = (long long)(P0 - r0), rb = (long long)(P1 - r0);
            const int A = (int)(ra < -16 ? -16 : (ra > RW + 16 ? RW + 16 : ra));
            const int B = (int)(rb < -16 ? -16 : (rb > RW + 16 ? RW + 16 : rb));
            u64 hm = __ballot(valid && lane < nlim && P1 > r0 && P0 < P1);
            while (hm) {
                const int i = __builtin_ctzll(hm);
                hm &= hm - 1;
                const int a = __builtin_amdgcn_readlane(A, i), b = __builtin_amdgcn_readlane(B, i);
                const u32 key = (u32)__builtin_amdgcn_readlane((int)rk, i);
#pragma unroll
                for (int u = 0; u < PIECE_U; ++u) {
                    if (b <= u * 1024 || a >= u * 1024 + 1024) continue;       // (uniform) not in row u
                    const int x = u * 1024 + xl;
                    const int lo = a > x ? a - x : 0, hi = b < x + 16 ? b - x : 16;
                    if (hi <= lo) continue;
                    ws_xor_range(key, lo, hi, v[u], cov[u]);                    // unmask in registers
                }
            }
            if (nlim < step || exact) break;                                // reached an item past the range
            if (k + step < cnt) { k += step; step = 64; continue; }         // more items of this segment
        }
        // this segment has no more items: continue with the next one if it starts in range
        ++s;
        k = 0;
        step = 16;
    }
    // ---- 3. store (v[] holds the unmasked bytes): full chunks one 16-B store, edge chunks
    //         exactly the covered bytes
    // NT 4: whole chunks leave as `buffer_store_dwordx4 … nt sc1` through a descriptor over this
    // wave's 4 KiB (round 4: −0.15–0.5 % per step against `global_store … nt` on cfg2, cfg3 and
    // the raw stream, `profiles/r04_k2_store_sc1nt_ab.log`; a one-shot XOR block streams 2.6 %
    // faster that way, `profiles/r04_calib_store_policy.log`)
    [[maybe_unused]] __amdgpu_buffer_rsrc_t wrs;
    if constexpr (NT == 4) wrs = ws_rsrc(reinterpret_cast<uintptr_t>(base + wc0), 64 * PIECE_U * 16);
#pragma unroll
    for (int u = 0; u < PIECE_U; ++u) {
        const u64 c = wc0 + (u64)(u * 64 + lane);
        if (!cov[u] || c < c_lo || c >= c_hi) continue;
        const u32x4 w = v[u];
        if (cov[u] == 0xFFFFu || segcov[u] == 0xFFFFu) {
            if constexpr (NT == 4) st16_sc1nt(w, wrs, (u * 64 + lane) * 16);
            else
                st16<NT>(w, base + c);
        } else {
            ws_store_bytes(reinterpret_cast<gu8*>(base + c), w, cov[u]);
        }
    }
    // K1 found the segments out of buffer order (or outside [lo, hi)): nothing was stored
    // above; the batch is decoded here instead, one wavefront per segment (ws_walk.h)
    if (!ok) {
        for (u32 s2 = blockIdx.x * (PIECE_T / 64) + wv; s2 < nseg; s2 += gridDim.x * (PIECE_T / 64))
            walk_segment<4, NT>(buf, s2, seg_off, seg_len, max_frames, desc_base, desc, res, lane);
    }
    // the host's stride hint for the next call (ws_api.hip): valid while at most 1/32 of the
    // segments had frames of more than one length (K1 has finished: its count is final)
    if (advice && bx == 0 && tid == 0) {
        const u32 n = *gptr<u32>(nonuni);
        *gptr<u32>(nonuni) = 0;
        __hip_atomic_store(advice, ok && (u64)n * 32 <= nseg ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(advice + 1, (int)ws_first_frame_len(buf, seg_off, seg_len, nseg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ws layout: [disorder u32 | nonuni u32 | pad to 16][ptr: npieces u64][nwork: nseg u32][items: nseg*max_frames x 16 B]
// No per-call reset: K1 writes every piece pointer, and marks an unordered batch by
// storing this call's generation number `gen` (never 0) into `disorder`, which the
// workspace owner zeroes once when it allocates the workspace. `nonuni` (K1's count of
// segments with frames of several lengths) rests at zero: K2 reads and clears it.
static u64 piece_count(u64 lo_org, u64 hi_org) {
    return hi_org > lo_org ? ((hi_org - 1) >> PIECE_SHIFT) - (lo_org >> PIECE_SHIFT) + 1 : 0;
}

size_t ws_piece_workspace_bytes(u64 span, u32 nseg, u32 max_frames) {
    const u64 npieces = (span + 15) / (1ull << PIECE_SHIFT) + 2;
    size_t b = (16 + npieces * 8 + 15) & ~(size_t)15;
    b = (b + (size_t)nseg * 4 + 31) & ~(size_t)31;
    b += (size_t)nseg * sizeof(WsSegRec);
    return b + (size_t)nseg * max_frames * 16 + 16;
}

// "scan_alpha": 1 (default) the walk switches to alphabet speculation once lengths keep changing,
// 0 stride speculation only (round 3's walk)
WsOpt ws_scan_alpha{1};

// K1 alone (also the first stage of the reassembly path, ws_reasm.hip). Segments lie in
// [lo, hi) of L.buf. count_nonuniform: K1 counts segments with frames of several lengths
// for the K2 that follows (ws_launch_piece); other users pass false.
static WalkArgs piece_scan_args(const WsLaunch& L, u64 lo, u64 hi, unsigned char* ws, u32 gen, PieceWs& P, u32 g0) {
    const u64 lead0 = reinterpret_cast<uintptr_t>(L.buf) & 15;
    const u64 lo_org = lo + lead0, hi_org = hi + lead0;
    P.npieces = piece_count(lo_org, hi_org);
    P.pbase = lo_org >> PIECE_SHIFT;
    P.c_lo = lo_org >> 4;
    P.c_hi = (hi_org + 15) >> 4;
    P.disorder = reinterpret_cast<u32*>(ws);
    P.nonuni = reinterpret_cast<u32*>(ws) + 1;
    P.ptr = reinterpret_cast<u64*>(ws + 16);
    size_t b = (16 + P.npieces * 8 + 15) & ~(size_t)15;
    P.nwork = reinterpret_cast<u32*>(ws + b);
    b = (b + (size_t)L.nseg * 4 + 31) & ~(size_t)31;
    P.segr = reinterpret_cast<WsSegRec*>(ws + b);
    b += (size_t)L.nseg * sizeof(WsSegRec);
    P.items = reinterpret_cast<u32x4*>(ws + b);
    WalkArgs W;
    W.buf = L.buf; W.seg_off = L.seg_off; W.seg_len = L.seg_len; W.nseg = L.nseg; W.max_frames = L.max_frames;
    W.desc_base = L.desc_base; W.desc = L.desc; W.res = L.res; W.items = P.items; W.ptr = P.ptr; W.nwork = P.nwork;
    W.segr = P.segr; W.disorder = P.disorder; W.gen = gen; W.pbase = P.pbase; W.lo = lo; W.hi = hi;
    W.g0 = g0 < (1u << 31) ? g0 : 0u;
    W.alpha_ok = ws_scan_alpha ? 1u : 0u;
    return W;
}

int ws_launch_piece_scan(const WsLaunch& L, u64 lo, u64 hi, unsigned char* ws, u32 gen, PieceWs* out,
                         bool count_nonuniform, u32 g0) {
    PieceWs P;
    const WalkArgs W = piece_scan_args(L, lo, hi, ws, gen, P, g0);
    const u32 blocks = (u32)(((u64)L.nseg * WALK_G + PSCAN_T - 1) / PSCAN_T);
    hipLaunchKernelGGL(ws_piece_scan_kernel, dim3(blocks), dim3(PSCAN_T), 0, L.stream, W,
                       count_nonuniform ? P.nonuni : nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ws_set_err("ws_piece_scan_kernel launch", e);
    *out = P;
    return 0;
}

#ifdef WS_K1_VARIANTS
// Measurement build only (tools/exp_k1k2.sh compiles this file a second time with it): K1 with a
// subset of its stores (st: the walk_group ST bitmask) or, st = 16, all stores at 8 waves per SIMD
// — the K1 breakdown of round 5. Not in the drop-in library.
template <int ST>
__global__ __launch_bounds__(PSCAN_T) void ws_piece_scan_kernel_st(WalkArgs A, u32* nonuni) {
    const u32 lane = threadIdx.x & 63;
    const u32 s = (blockIdx.x * PSCAN_T + threadIdx.x) / WALK_G;
    u32 cnt = 0;
    bool nonu = false;
    walk_group<ST>(A, s, s < A.nseg, lane, cnt, nonu);
}
__global__ __launch_bounds__(PSCAN_T) __attribute__((amdgpu_waves_per_eu(8, 8))) void ws_piece_scan_kernel_w8(
    WalkArgs A, u32* nonuni) {
    const u32 lane = threadIdx.x & 63;
    const u32 s = (blockIdx.x * PSCAN_T + threadIdx.x) / WALK_G;
    u32 cnt = 0;
    bool nonu = false;
    walk_group<15>(A, s, s < A.nseg, lane, cnt, nonu);
}
int ws_launch_piece_scan_variant(const WsLaunch& L, u64 lo, u64 hi, unsigned char* ws, u32 gen, u32 g0, int st,
                                 PieceWs* out) {
    PieceWs P;
    const WalkArgs W = piece_scan_args(L, lo, hi, ws, gen, P, g0);
    const dim3 g((u32)(((u64)L.nseg * WALK_G + PSCAN_T - 1) / PSCAN_T)), b(PSCAN_T);
    switch (st) {
    case 0: hipLaunchKernelGGL(ws_piece_scan_kernel_st<0>, g, b, 0, L.stream, W, nullptr); break;
    case 1: hipLaunchKernelGGL(ws_piece_scan_kernel_st<1>, g, b, 0, L.stream, W, nullptr); break;
    case 3: hipLaunchKernelGGL(ws_piece_scan_kernel_st<3>, g, b, 0, L.stream, W, nullptr); break;
    case 7: hipLaunchKernelGGL(ws_piece_scan_kernel_st<7>, g, b, 0, L.stream, W, nullptr); break;
    case 8: hipLaunchKernelGGL(ws_piece_scan_kernel_st<8>, g, b, 0, L.stream, W, nullptr); break;
    case 13: hipLaunchKernelGGL(ws_piece_scan_kernel_st<13>, g, b, 0, L.stream, W, nullptr); break;
    case 15: hipLaunchKernelGGL(ws_piece_scan_kernel_st<15>, g, b, 0, L.stream, W, nullptr); break;
    case 16: hipLaunchKernelGGL(ws_piece_scan_kernel_w8, g, b, 0, L.stream, W, nullptr); break;
    default: return -1;
    }
    *out = P;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
#endif

// "piece_lds": bytes of unused dynamic LDS per K2 block, which caps its blocks (= waves per
// SIMD) per CU. 0 (default): the CU's LDS / 7 for frames of <= 16 KiB, else / 6 (ws_piece_dyn_lds).
// K2 needs only 60 VGPRs (8 waves/SIMD would fit); with nontemporal stores it streamed best at 6
// (round 3, profiles/r03_k2_occupancy.log); with the sc1|nt stores (round 4) pieces holding
// several frames gain a seventh block (cfg2 -0.5-1.4 %, cfg2 in 64-frame segments -1.8 %), large
// frames keep 6 (cfg3 +0.6 %, cfg4 +0.75 % at 7), 8 loses 2 % (profiles/r04_k2_occupancy_sc1.log).
// gfx950 (160 KiB per CU): 23,296 B and 27,136 B.
WsOpt ws_piece_lds{0};
WsOpt ws_piece_win{-1};  // "piece_win": log2 of the number of piece windows K2 streams side by side; -1 (default)
                          // 2 for batches of >= 32 GiB, and of >= 16 GiB the previous call advised as frames of
                          // one length, else 1
                          // (piece_wshift)

int ws_piece_dyn_lds(const WsLaunch& L, u64 npieces, u32 g0) {
    const int opt = ws_piece_lds;
    if (opt > 0) return opt <= 65536 ? opt : 65536;
    // 7 blocks per CU for frames of <= 16 KiB (several per piece), 6 for larger ones; the frame
    // length is the previous call's advice when it had frames of one length (g0), else the
    // batch's segment density stands in for it
    const bool seven = g0 >= 2 ? g0 <= 16384u : (u64)L.nseg * 8 >= npieces;
    const int per = L.lds_per_cu / (seven ? 7 : 6);
    return per > 65536 ? 65536 : (per & ~255);
}

// "k2_timing" (measurement only, bench.py): a pair of HIP events is recorded around every
// K2 launch on its stream; websocketframeGpuGetStat("k2_ns") waits for and sums the
// recorded durations, "k2_calls" counts them; setting the option clears the record.
WsOpt ws_k2_timing{0};
static std::vector<hipEvent_t> g_k2ev;    // start, end, start, end, ...
static size_t g_k2n = 0;
static std::mutex g_k2mu;

void ws_k2_timing_reset() {
    std::lock_guard<std::mutex> lk(g_k2mu);
    g_k2n = 0;
}

int ws_k2_stat(unsigned long long* ns, unsigned long long* calls) {
    std::lock_guard<std::mutex> lk(g_k2mu);
    double total = 0.0;
    for (size_t i = 0; i < g_k2n; ++i) {
        float ms = 0.f;
        hipError_t e = hipEventSynchronize(g_k2ev[2 * i + 1]);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, g_k2ev[2 * i], g_k2ev[2 * i + 1]);
        if (e != hipSuccess) return ws_set_err("k2 timing events", e);
        total += ms;
    }
    *ns = (unsigned long long)(total * 1e6);
    *calls = g_k2n;
    return 0;
}

int ws_k2_mark(hipStream_t st, bool end, size_t* slot) {
    std::lock_guard<std::mutex> lk(g_k2mu);
    if (!end) *slot = g_k2n++;
    const size_t i = 2 * *slot + (end ? 1 : 0);
    hipError_t e;
    while (g_k2ev.size() <= i) {
        hipEvent_t ev;
        if ((e = hipEventCreate(&ev)) != hipSuccess) return ws_set_err("hipEventCreate", e);
        g_k2ev.push_back(ev);
    }
    if ((e = hipEventRecord(g_k2ev[i], st)) != hipSuccess) return ws_set_err("hipEventRecord", e);
    return 0;
}

// Windows: round 1 measured two windows half a batch apart against one (cfg4 74 -> 82 %, cfg2 +2 %,
// cfg3 =). Round 5 measured the window count per buffer PLACEMENT (several buffers of one config in
// one process, tools/exp_place_win.py, profiles/r05_place_win.log): one 68.7 GB cfg4 round takes
// 20.6-22.0 ms with two windows depending on where its buffer lies in HBM, 20.6-21.0 with four
// (mean -1.6 to -2.2 %, worst buffer -2.7 to -4.8 %, three processes); cfg2 -0.5 % with four; cfg3
// (mixed lengths) +0.85 % with four. In the bench's own protocol (the same buffer re-decoded) cfg2
// runs 0.4 % slower with four (1.3597-1.3623 against 1.3539-1.3545 ms at 100 steps, processes
// paired over both placements, profiles/r05_win_ab.log) while cfg4 keeps the gain. So four windows
// for batches of >= 1 M pieces (16 GiB) the previous call advised as frames of one length (g0, the
// stride hint), two otherwise (first calls, captured calls, mixed lengths, smaller batches).
// Round 6 (profiles/r06_win_rule_*.json, tools/exp_win_rule.py): first and
// captured calls have no advice, so a 68.7 GB cfg4 round took two windows there and 21.7-22.0 ms
// on its slow placement against 20.98-21.04 with four; four windows from the size alone also for
// cfg3's 23.5 GB cost 0.6-0.9 % (captured and steady). So batches of >= 2 M pieces (32 GiB) take
// four windows whatever the advice, 1-2 M pieces four only when advised as one frame length.
#define PIECE_WIN4_MIN (1ull << 20)
#define PIECE_WIN4_BIG (2ull << 20)
static u32 piece_wshift(u64 npieces, u32 g0, int call_win) {
    int pwin = ws_piece_win;
    if (pwin < 0 && call_win >= 0) pwin = call_win;                      // the caller's choice (raw stream)
    if (pwin < 0) pwin = npieces >= PIECE_WIN4_BIG || (g0 >= 2 && npieces >= PIECE_WIN4_MIN) ? 2 : 1;
    u32 wshift = (u32)(pwin > 6 ? 6 : pwin);
    while (wshift && (npieces >> wshift) < 256) --wshift;                // small batches: one window
    return wshift;
}

// K2 over the pieces of a scanned batch; advice (device view of pinned host memory, may be
// null): K2 turns K1's non-uniform count into the host's stride hint for the next call
std::atomic<unsigned long long> ws_stat_k2_windows{0};   // windows of the most recent K2 launch (stat "k2_windows")
int ws_launch_piece_unmask(const WsLaunch& L, const PieceWs& P, u32 gen, int* advice, u32 g0) {
    if (!P.npieces) return 0;
    size_t tslot = 0;
    int rc;
    const int timing = ws_k2_timing;
    if (timing && (rc = ws_k2_mark(L.stream, false, &tslot))) return rc;
    const u32 wshift = piece_wshift(P.npieces, g0, L.pwin);
    ws_stat_k2_windows = 1ull << wshift;
    const u64 ppw = (P.npieces + (1ull << wshift) - 1) >> wshift;
    const u64 grid = ppw << wshift;
    if (P.segr)
        hipLaunchKernelGGL((ws_piece_unmask_kernel<4, 1>), dim3((u32)grid), dim3(PIECE_T), ws_piece_dyn_lds(L, P.npieces, g0), L.stream,
                           L.buf, L.seg_off, L.seg_len, L.nseg, L.max_frames, P.items, P.nwork, P.ptr, P.disorder, gen,
                           P.pbase, P.c_lo, P.c_hi, L.desc_base, L.desc, L.res, wshift, ppw, (u64)P.npieces, P.nonuni,
                           advice, (const WsSegRec*)P.segr);
    else
        hipLaunchKernelGGL((ws_piece_unmask_kernel<4, 0>), dim3((u32)grid), dim3(PIECE_T), ws_piece_dyn_lds(L, P.npieces, g0), L.stream,
                           L.buf, L.seg_off, L.seg_len, L.nseg, L.max_frames, P.items, P.nwork, P.ptr, P.disorder, gen,
                           P.pbase, P.c_lo, P.c_hi, L.desc_base, L.desc, L.res, wshift, ppw, (u64)P.npieces, P.nonuni,
                           advice, (const WsSegRec*)nullptr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ws_set_err("ws_piece_unmask_kernel launch", e);
    return timing ? ws_k2_mark(L.stream, true, &tslot) : 0;
}

// K1 + K2; K2 also holds the fallback for unordered batches. *fallback_needed: no K2
// was launched (no pieces), so the caller must launch the gated walker itself.
int ws_launch_piece(const WsLaunch& L, u64 lo, u64 hi, unsigned char* ws, u32 gen, int* advice,
                    const u32** disorder_out, bool* fallback_needed, u32 g0) {
    PieceWs P;
    int rc = ws_launch_piece_scan(L, lo, hi, ws, gen, &P, advice != nullptr, g0);
    if (rc) return rc;
    if ((rc = ws_launch_piece_unmask(L, P, gen, advice, g0))) return rc;
    *disorder_out = P.disorder;
    *fallback_needed = P.npieces == 0;
    return 0;
}
