// ws_stream.hip — one raw rx stream of any size (a single connection's inbuf, e.g.
// many GB): frame-boundary discovery on the device without host-supplied offsets
// (SURVEY §8f rank 2), then the piece path's one-shot unmask.
//
// The reactor loop over one buffer (net_reactor.c:515-526) is a serial chain: frame k+1
// starts where frame k ends. Walking it with one lane (or one group, ws_piece.hip) costs
// one dependent load per frame (per G frames with stride speculation). Here the WHOLE
// GRID speculates: from the last confirmed frame (offset P, length g) thread k parses the
// header at P + k*g; the chain is right up to the first thread whose frame is not a
// length-g frame (atomicMin over a packed (k, outcome) word), and every thread below it
// has already written its descriptor, payload item and piece pointers. A stream of
// equal-length frames is confirmed in one pass; each length change costs one more pass.
// Speculative writes past the first stop are overwritten by the next pass (same slots,
// same pieces). Passes are driven from the host (one 8-byte read each); when passes stop
// paying (a pass confirms fewer than 64 frames), the rest of the stream is walked by one
// wavefront in a single launch (ws_stream_walk_kernel: stride speculation over 64
// lanes, no host round trips) — lengths that change every frame are a serial chain.
#include <cstdio>
#include <vector>

#include "ws_common.h"

#define SPASS_T 256
#define PIECE_SHIFT_S 14

// outcome bits packed with the candidate index: k << 36 | code << 34 | stf << 32 | (u32)ret
//   code 1: consumed, length != g   2: consumed, walk ends (ret <= 0)   3: not consumed
//   stf (code 3): 0 OK, 1 MAX_FRAMES, 2 LEN_WRAP; (code 2): 0 ret == 0, 1 ret < 0
__global__ __launch_bounds__(SPASS_T) void ws_stream_pass_kernel(const unsigned char* __restrict__ buf, u64 len,
                                                                 u64 P, u64 g, u32 nf, u32 max_frames, u64 K,
                                                                 WebsocketFrameDesc_t* __restrict__ desc,
                                                                 u32x4* __restrict__ items, u64* __restrict__ ptr,
                                                                 u64 pend, unsigned long long* __restrict__ stop) {
    const u64 k = (u64)blockIdx.x * SPASS_T + threadIdx.x;
    if (k >= K) return;
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    const u64 pos = P + k * g;
    u32 code = 0, stf = 0;
    WsHdr h = {};
    if (pos >= len) code = 3;
    else if ((u64)nf + k >= max_frames) { code = 3; stf = 1; }
    else if (len - pos < 2) code = 3;                                        // websocketframe.c:121
    else {
        const uintptr_t pa = reinterpret_cast<uintptr_t>(buf + pos);
        const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
        u64 h0, h1;
        ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
        h = ws_parse(h0, h1, len - pos);
        if (h.kind == WS_PARSE_INCOMPLETE) code = 3;
        else if (h.kind == WS_PARSE_WRAP) { code = 3; stf = 2; }
        else if (h.ret <= 0) { code = 2; stf = h.ret < 0 ? 1u : 0u; }
        else code = (u64)(u32)h.ret == g ? 0u : 1u;
    }
    if (code == 0 || code == 1 || code == 2) {                               // speculative writes
        const u64 fo = lead0 + pos, p0 = fo + h.hdr, fe = p0 + h.plen;
        const u64 slot = (u64)nf + k;
        const u64 w0 = p0 | ((u64)(rotl32(h.key, 8u * (u32)(p0 & 3)) & 0xFFFFu) << 48);
        const u64 w1 = (h.masked ? fe : p0) | ((u64)(rotl32(h.key, 8u * (u32)(p0 & 3)) >> 16) << 48);
        u32x4 it;
        it.x = (u32)w0; it.y = (u32)(w0 >> 32); it.z = (u32)w1; it.w = (u32)(w1 >> 32);
        *gptr<u32x4>(items + slot) = it;
        for (u64 p = (fo + (1ull << PIECE_SHIFT_S) - 1) >> PIECE_SHIFT_S; (p << PIECE_SHIFT_S) < fe && p < pend; ++p)
            *gptr<u64>(ptr + p) = slot;                                      // segment 0, item `slot`
        if (h.ret != 0) ws_store_desc(desc + slot, pos, h);
    }
    if (code != 0) {
        const unsigned long long word = ((unsigned long long)k << 36) | ((unsigned long long)code << 34) |
                                        ((unsigned long long)stf << 32) | (u32)h.ret;
        atomicMin(stop, word);
    }
}

// Piece pointers [lo, hi) -> val. With lo_from_item / hi_from_item the bound is the
// payload end (P1, origin-relative) of item `item` instead: the extent of a frame whose
// length the host does not know (the loop's last frame when it returned <= 0).
__global__ void ws_stream_ptr_kernel(u64* __restrict__ ptr, u64 pend, u64 lo, u64 hi, u64 val,
                                     const u32x4* __restrict__ items, u64 item, int lo_from_item, int hi_from_item) {
    if (lo_from_item || hi_from_item) {
        const u32x4 it = items[item];
        const u64 p1 = ((u64)it.z | ((u64)it.w << 32)) & 0xFFFFFFFFFFFFull;
        if (lo_from_item) lo = p1;
        if (hi_from_item) hi = p1;
    }
    const u64 p0 = (lo + (1ull << PIECE_SHIFT_S) - 1) >> PIECE_SHIFT_S;
    for (u64 p = p0 + threadIdx.x; (p << PIECE_SHIFT_S) < hi && p < pend; p += blockDim.x) ptr[p] = val;
}

__global__ void ws_stream_res_kernel(u32* __restrict__ nwork, u32 cnt, WebsocketSegResult_t* __restrict__ res,
                                     u64 consumed, u32 nf, int status) {
    nwork[0] = cnt;
    ws_store_res(res, consumed, nf, status);
}

// Frames of the stream starting in [P0, end) from (P0, nf0, g0) by one wavefront: the group
// walk of ws_piece.hip (64 lanes, stride speculation; only consumed frames are written).
// `last`: the walk runs to the stream's end (end == len) and then writes the tail
// pointers, the item count and the segment result; otherwise it stops before the first
// frame starting at or after `end` (another wavefront owns it).
__device__ __forceinline__ void stream_walk(const unsigned char* __restrict__ buf, u64 len, u64 P0, u64 g0, u32 nf0,
                                            u64 end, bool last, u32 max_frames, WebsocketFrameDesc_t* __restrict__ desc,
                                            u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                            u32* __restrict__ nwork, WebsocketSegResult_t* __restrict__ res,
                                            u32 lane, u64* __restrict__ out = nullptr) {
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    const uintptr_t seg = reinterpret_cast<uintptr_t>(buf);
    u64 off = P0, g = g0, walked_end = lead0 + P0;
    u32 nf = nf0, extra = 0;
    int status = WEBSOCKET_SEG_OK;
    bool at_bnd = false;
    for (;;) {
        const u64 pos = off + (u64)lane * g;
        const bool cand = lane == 0 || g > 0;
        const bool eval = cand && pos < len;
        const uintptr_t pa = seg + (eval ? pos : 0);
        const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
        u64 h0, h1;
        ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
        const WsHdr h = ws_parse(h0, h1, eval ? len - pos : 0);
        u32 code = 3, bnd = 0;
        int st = WEBSOCKET_SEG_OK;
        if (cand) {
            if (pos >= len) code = 3;
            else if (pos >= end) { code = 3; bnd = 1; }                      // the next wavefront's frame
            else if (nf + lane >= max_frames) { code = 3; st = WEBSOCKET_SEG_MAX_FRAMES; }
            else if (len - pos < 2) code = 3;                                // websocketframe.c:121
            else if (h.kind == WS_PARSE_INCOMPLETE) code = 3;
            else if (h.kind == WS_PARSE_WRAP) { code = 3; st = WEBSOCKET_SEG_ERR_LEN_WRAP; }
            else if (h.ret <= 0) { code = 2; st = h.ret < 0 ? WEBSOCKET_SEG_ERR_DECODE : WEBSOCKET_SEG_OK; }
            else code = (u64)(u32)h.ret == g ? 0u : 1u;
        }
        const u64 stopm = __ballot(code != 0);
        const u32 mm = stopm ? (u32)__builtin_ctzll(stopm) : 64u;
        const u32 code_m = mm < 64 ? (u32)__builtin_amdgcn_readlane((int)code, (int)mm) : 0u;
        const u32 ntake = mm + ((code_m == 1 || code_m == 2) ? 1u : 0u);
        const u64 fo = lead0 + pos, p0 = fo + h.hdr, fe = p0 + h.plen;
        if (lane < ntake) {
            const u64 w0 = p0 | ((u64)(rotl32(h.key, 8u * (u32)(p0 & 3)) & 0xFFFFu) << 48);
            const u64 w1 = (h.masked ? fe : p0) | ((u64)(rotl32(h.key, 8u * (u32)(p0 & 3)) >> 16) << 48);
            u32x4 it;
            it.x = (u32)w0; it.y = (u32)(w0 >> 32); it.z = (u32)w1; it.w = (u32)(w1 >> 32);
            *gptr<u32x4>(items + nf + lane) = it;
            for (u64 p = (fo + (1ull << PIECE_SHIFT_S) - 1) >> PIECE_SHIFT_S; (p << PIECE_SHIFT_S) < fe && p < pend; ++p)
                *gptr<u64>(ptr + p) = nf + lane;
            if (h.ret != 0) ws_store_desc(desc + nf + lane, pos, h);
        }
        if (ntake) walked_end = __shfl(fe, (int)ntake - 1);
        if (mm == 64) { nf += 64; off += 64 * g; continue; }
        const u64 pos_m = off + (u64)mm * g;
        const int ret_m = __builtin_amdgcn_readlane(h.ret, (int)mm);
        nf += mm;
        if (code_m == 1) { nf += 1; off = pos_m + (u32)ret_m; g = (u32)ret_m; continue; }
        off = pos_m;
        at_bnd = __builtin_amdgcn_readlane((int)bnd, (int)mm) != 0;
        if (code_m == 2) {
            if (ret_m != 0) nf += 1;
            else extra = 1;
        }
        status = __builtin_amdgcn_readlane(st, (int)mm);
        break;
    }
    // `out` (a walk of one chunk): {next entry, its frame index, 1 if the stream's walk ended
    // here}; a walk that ended here finishes the stream as the last one does
    if (out && lane == 0) {
        out[0] = off;
        out[1] = nf;
        out[2] = at_bnd ? 0 : 1;
    }
    if (!last && (at_bnd || !out)) return;
    const u32 cnt = nf + extra;
    for (u64 p = ((walked_end + (1ull << PIECE_SHIFT_S) - 1) >> PIECE_SHIFT_S) + lane;
         (p << PIECE_SHIFT_S) < lead0 + len && p < pend; p += 64)
        ptr[p] = cnt;
    if (lane == 0) {
        nwork[0] = cnt;
        ws_store_res(res, off, nf, status);
    }
}

// The rest of the stream from (P0, nf0, g0) by one wavefront (lengths that keep changing)
__global__ __launch_bounds__(64) void ws_stream_walk_kernel(const unsigned char* __restrict__ buf, u64 len, u64 P0,
                                                            u64 g0, u32 nf0, u32 max_frames,
                                                            WebsocketFrameDesc_t* __restrict__ desc,
                                                            u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                                            u32* __restrict__ nwork,
                                                            WebsocketSegResult_t* __restrict__ res) {
    stream_walk(buf, len, P0, g0, nf0, len, true, max_frames, desc, items, ptr, pend, nwork, res, threadIdx.x);
}

// One chunk [P0, end) walked by one wavefront when the chunk-parallel records have no link
// (see below): reports the next entry in out[0..2]
__global__ __launch_bounds__(64) void ws_rw_chunk_kernel(const unsigned char* __restrict__ buf, u64 len, u64 P0,
                                                         u32 nf0, u64 end, u32 max_frames,
                                                         WebsocketFrameDesc_t* __restrict__ desc,
                                                         u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                                         u32* __restrict__ nwork, WebsocketSegResult_t* __restrict__ res,
                                                         u64* __restrict__ out) {
    stream_walk(buf, len, P0, 0, nf0, end, false, max_frames, desc, items, ptr, pend, nwork, res, threadIdx.x, out);
}

// ---------------------------------------------------------------------------------------------
// Chunk-parallel walk for long streams whose frame lengths keep changing (the reactor
// loop is a serial chain; one wavefront walks it at ~1 frame per dependent load).
//   sample: one wavefront walks the first RW_SAMPLE bytes (ws_rw_chunk_kernel), which also
//      gives the mean wire length; the rest of the stream [P, len) is cut into chunks of C
//      bytes (about 512 frames each) and the true chain enters chunk c at its first frame
//      start at or after the chunk's first byte, i.e. inside the chunk's first H bytes
//      (8-16 mean frames) unless a frame longer than that covers them;
//   spec (ws_rw_spec_kernel): every position of those windows whose header looks like a
//      client frame (RSV clear, a defined opcode, MASK set when the stream's frames are
//      masked) runs the reactor's rules from there, dropping out at the first implausible
//      header (a wrong start lands on garbage within a step or two; the true chain of a
//      client stream never does), and records where it leaves its chunk or where the
//      stream's walk ends. Every true frame start of the window survives (a suffix of the
//      chain), so a chunk keeps up to RW_S0 records of walks that leave it;
//   host: from P, follow the records chunk by chunk (exact: each record IS the reference
//      loop from its start); a chunk with no record at the chain's entry (a frame longer
//      than the window, an implausible frame, more survivors than slots) is walked by one
//      wavefront that reports the next entry;
//   emit (ws_rw_emit_kernel): one wavefront per chunk on the chain writes its frames
//      (stream_walk from the chain's frame index), the last one also the tail, count and
//      result.
// Every byte decision is made by the reference rules; speculation only picks where to start.
#define RW_CMAX (4ull << 20)
#define RW_CMIN (64ull << 10)
#define RW_HMAX (128u << 10)
#define RW_HMIN (4u << 10)
#define RW_SAMPLE (256ull << 10)
#define RW_S0 40          // records per chunk of walks that leave it (~8-16 true frame starts)
#define RW_S1 8           // ... of walks that end the stream in it
#define RW_SLOTS (RW_S0 + RW_S1)
#define RW_SLAST 4096     // walks that end the stream in the last chunk
#define RW_MAXSTEPS 4096

struct RwRec {            // one surviving walk from chunk start + start
    u32 start;
    u32 cs;               // frames consumed | status << 31 (0 left the chunk, 1 the stream's walk ends)
    u64 exit;             // the next frame start (status 0) or where the walk ended
};

// b23: header bytes 2 and 3 (the top of a 64-bit length, which a real frame leaves zero:
// a random 64-bit length reads as an incomplete frame and would crowd the records)
__device__ __forceinline__ bool rw_plausible(u32 b0, u32 b1, u32 b23, bool need_mask) {
    const u32 op = b0 & 15u;
    return !(b0 & 0x70u) && (op <= 2u || (op >= 8u && op <= 10u)) && (!need_mask || (b1 & 0x80u)) &&
           ((b1 & 0x7Fu) != 127u || b23 == 0u);
}

// one thread per 16 window positions (aligned loads); walks its plausible positions
__global__ __launch_bounds__(256) void ws_rw_spec_kernel(const unsigned char* __restrict__ buf, u64 len, u64 P,
                                                         u64 C, u32 H, u32 nchunks, u32 need_mask,
                                                         RwRec* __restrict__ recs, u32* __restrict__ nrec) {
    const u64 t = (u64)blockIdx.x * 256 + threadIdx.x;
    const u32 per = H / 16;
    const u64 c = t / per;
    if (c >= nchunks) return;
    const uintptr_t origin = reinterpret_cast<uintptr_t>(buf);
    const u64 cs0 = P + c * C, cend = cs0 + C;
    const uintptr_t a = ((origin + cs0) & ~(uintptr_t)15) + (t % per) * 16;
    if (a >= origin + len) return;                                           // reads stay within len + pad
    const u32x4 x0 = reinterpret_cast<const gu32x4*>(a)[0], x1 = reinterpret_cast<const gu32x4*>(a)[1];
    const u32 w[5] = {x0.x, x0.y, x0.z, x0.w, x1.x};
    u32 cands = 0;
#pragma unroll
    for (u32 k = 0; k < 16; ++k) {
        const u32 b0 = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const u32 b1 = (w[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xFFu;
        const u32 b2 = (w[(k + 2) >> 2] >> (8 * ((k + 2) & 3))) & 0xFFu;
        const u32 b3 = (w[(k + 3) >> 2] >> (8 * ((k + 3) & 3))) & 0xFFu;
        cands |= (rw_plausible(b0, b1, b2 | b3, need_mask) ? 1u : 0u) << k;
    }
    while (cands) {
        const u32 k = (u32)__builtin_ctz(cands);
        cands &= cands - 1;
        const u64 start = a + k - origin;
        if (start < cs0 || start >= len) continue;
        u64 pos = start;
        u32 cnt = 0, st = 0;
        bool alive = true;
        for (u32 step = 0;; ++step) {
            if (pos >= cend) break;                                          // left the chunk
            if (step >= RW_MAXSTEPS) { alive = false; break; }
            if (pos >= len || len - pos < 2) { st = 1; break; }              // websocketframe.c:121
            const uintptr_t pa = origin + pos;
            const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
            u64 h0, h1;
            ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
            if (!rw_plausible((u32)h0 & 0xFFu, (u32)(h0 >> 8) & 0xFFu, (u32)(h0 >> 16) & 0xFFFFu, need_mask)) {
                alive = false;
                break;
            }
            const WsHdr h = ws_parse(h0, h1, len - pos);
            if (h.kind != WS_PARSE_FRAME || h.ret <= 0) { st = 1; break; }  // the stream's walk ends here
            pos += (u32)h.ret;
            ++cnt;
        }
        if (!alive) continue;
        // the last chunk's window lies near the stream's end, where wrong starts read as
        // incomplete frames: its walks that end get a pool of their own
        const bool lastc = c + 1 == nchunks;
        const u32 slot = atomicAdd(nrec + 2 * c + st, 1u);
        if (slot >= (st ? (lastc ? RW_SLAST : RW_S1) : RW_S0)) continue;
        RwRec r;
        r.start = (u32)(start - cs0);
        r.cs = cnt | (st << 31);
        r.exit = pos;
        recs[st && lastc ? (u64)nchunks * RW_SLOTS + slot : c * RW_SLOTS + (st ? RW_S0 : 0) + slot] = r;
    }
}

// emit: one wavefront per chain chunk: tab[b] = {entry, end, nf0, last}
__global__ __launch_bounds__(64) void ws_rw_emit_kernel(const unsigned char* __restrict__ buf, u64 len, u32 max_frames,
                                                        const u64* __restrict__ tab,
                                                        WebsocketFrameDesc_t* __restrict__ desc,
                                                        u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                                        u32* __restrict__ nwork, WebsocketSegResult_t* __restrict__ res) {
    const u64* t = tab + 4 * blockIdx.x;
    stream_walk(buf, len, t[0], 0, (u32)t[2], t[1], t[3] != 0, max_frames, desc, items, ptr, pend, nwork, res,
                threadIdx.x);
}

int ws_launch_piece_unmask(const WsLaunch& L, const PieceWs& P, int nt, u32 gen);

#define RW_MIN (16ull << 20)      // streams shorter than this after the passes: one wavefront walks
int ws_stream_rw = 1;            // "stream_rw": 1 chunk-parallel walk for long streams, 0 one wavefront
extern int ws_dbg_flags;
unsigned long long ws_stat_rw_chunks = 0;       // chunks written from records (last call)
unsigned long long ws_stat_rw_chunk_walks = 0;  // chunks walked by one wavefront without a record

// grow-only scratch for the chunk-parallel walk (per device): device records + counters,
// and a pinned host copy of them
struct RwScratch {
    void* d = nullptr;
    size_t d_bytes = 0;
    void* h = nullptr;
    size_t h_bytes = 0;
};
static RwScratch g_rw[64];

static int rw_scratch(size_t dbytes, size_t hbytes, hipStream_t st, RwScratch** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return ws_set_err("hipGetDevice", e);
    if (dev < 0 || dev >= 64) return ws_set_err("device index", hipErrorInvalidDevice);
    RwScratch& s = g_rw[dev];
    if (s.d_bytes < dbytes || s.h_bytes < hbytes) {
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return ws_set_err("hipStreamSynchronize", e);
    }
    if (s.d_bytes < dbytes) {
        if (s.d) (void)hipFree(s.d);
        s.d = nullptr;
        s.d_bytes = 0;
        if ((e = hipMalloc(&s.d, dbytes)) != hipSuccess) return ws_set_err("hipMalloc(stream scratch)", e);
        s.d_bytes = dbytes;
    }
    if (s.h_bytes < hbytes) {
        if (s.h) (void)hipHostFree(s.h);
        s.h = nullptr;
        s.h_bytes = 0;
        if ((e = hipHostMalloc(&s.h, hbytes, hipHostMallocDefault)) != hipSuccess)
            return ws_set_err("hipHostMalloc(stream scratch)", e);
        s.h_bytes = hbytes;
    }
    *out = &s;
    return 0;
}

static u64 rw_pow2_clamp(u64 x, u64 lo, u64 hi) {
    u64 v = lo;
    while (v < x && v < hi) v <<= 1;
    return v;
}

// The chunk-parallel walk of [P, len) with nf frames before P (see above). Launches the
// emit kernels and, for chunks without a link, one-wavefront chunk walks; the last of
// them writes the tail pointers, item count and segment result.
static int rw_walk(unsigned char* d_buf, u64 len, u64 P, u32 nf, u32 max_frames, WebsocketFrameDesc_t* d_desc,
                   const PieceWs& Pw, WebsocketSegResult_t* d_res, hipStream_t st) {
    hipError_t e;
    const u64 nchunks_max = (len - P + RW_CMIN - 1) / RW_CMIN;
    const size_t b_recs = ((size_t)(nchunks_max * RW_SLOTS + RW_SLAST) * sizeof(RwRec) + 255) & ~(size_t)255;
    const size_t b_nrec = ((size_t)nchunks_max * 8 + 255) & ~(size_t)255;
    const size_t b_tab = ((size_t)nchunks_max * 32 + 255) & ~(size_t)255;
    RwScratch* S = nullptr;
    int rc = rw_scratch(b_recs + b_nrec + b_tab + 256, b_recs + b_nrec + 256, st, &S);
    if (rc) return rc;
    unsigned char* w = reinterpret_cast<unsigned char*>(S->d);
    RwRec* recs = reinterpret_cast<RwRec*>(w);
    u32* nrec = reinterpret_cast<u32*>(w + b_recs);
    u64* tab = reinterpret_cast<u64*>(w + b_recs + b_nrec);
    u64* wout = reinterpret_cast<u64*>(w + b_recs + b_nrec + b_tab);
    unsigned char* hw = reinterpret_cast<unsigned char*>(S->h);
    RwRec* hr = reinterpret_cast<RwRec*>(hw);
    u32* hn = reinterpret_cast<u32*>(hw + b_recs);
    u64* ho = reinterpret_cast<u64*>(hw + b_recs + b_nrec);                // chunk-walk reports, header bytes
    ws_stat_rw_chunk_walks = 0;
    ws_stat_rw_chunks = 0;
    // one chunk [ent, end) by one wavefront: the next entry, or the stream finished
    auto chunk_walk = [&](u64 ent, u32 nfc, u64 end, u64& next, u32& nfn) -> int {
        ++ws_stat_rw_chunk_walks;
        hipLaunchKernelGGL(ws_rw_chunk_kernel, dim3(1), dim3(64), 0, st, d_buf, len, ent, nfc, end < len ? end : len,
                           max_frames, d_desc, Pw.items, Pw.ptr, Pw.npieces, Pw.nwork, d_res, wout);
        hipError_t e2 = hipGetLastError();
        if (e2 != hipSuccess) return ws_set_err("ws_rw_chunk_kernel launch", e2);
        if ((e2 = hipMemcpyAsync(ho, wout, 24, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (e2 = hipStreamSynchronize(st)) != hipSuccess)
            return ws_set_err("stream chunk walk", e2);
        next = ho[0];
        nfn = (u32)ho[1];
        return ho[2] ? 1 : 0;
    };
    // sample: the first RW_SAMPLE bytes, and the mean wire length
    u64 P1 = 0;
    u32 nf1 = 0;
    if ((rc = chunk_walk(P, nf, P + RW_SAMPLE, P1, nf1))) return rc < 0 ? rc : 0;
    ws_stat_rw_chunk_walks = 0;                                              // not counting the sample
    const u64 mean = nf1 > nf ? (P1 - P) / (nf1 - nf) : (P1 - P);
    P = P1;
    nf = nf1;
    const u64 C = rw_pow2_clamp(mean * 512, RW_CMIN, RW_CMAX);
    const u32 H = (u32)rw_pow2_clamp(mean * 8, RW_HMIN, C / 2 < RW_HMAX ? C / 2 : RW_HMAX);
    const u64 nchunks = (len - P + C - 1) / C;
    // the stream's frames are masked if the one at P is (client streams): candidates must be too
    unsigned char* hb = reinterpret_cast<unsigned char*>(ho + 4);
    hb[1] = 0;
    if ((e = hipMemcpyAsync(hb, d_buf + P, 2, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipMemsetAsync(nrec, 0, nchunks * 8, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return ws_set_err("stream walk setup", e);
    const u32 need_mask = (hb[1] & 0x80u) ? 1u : 0u;
    const u64 threads = nchunks * (H / 16);
    hipLaunchKernelGGL(ws_rw_spec_kernel, dim3((u32)((threads + 255) / 256)), dim3(256), 0, st, d_buf, len, P, C, H,
                       (u32)nchunks, need_mask, recs, nrec);
    if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_rw_spec_kernel launch", e);
    if ((e = hipMemcpyAsync(hn, nrec, nchunks * 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipMemcpyAsync(hr, recs, nchunks * RW_SLOTS * sizeof(RwRec), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipMemcpyAsync(hr + nchunks * RW_SLOTS, recs + nchunks * RW_SLOTS,
                            (size_t)RW_SLAST * sizeof(RwRec), hipMemcpyDeviceToHost, st)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return ws_set_err("stream walk records", e);
    // follow the chain from P: exact, every record is the reference loop from its start
    std::vector<u64> ht;
    u64 ent = P;
    u32 nfc = nf;
    for (bool last = false; !last;) {
        const u64 c = (ent - P) / C, cs0 = P + c * C;
        const RwRec* r = nullptr;
        if (c < nchunks && ent - cs0 < H) {
            const u32 so = (u32)(ent - cs0);
            for (u32 k = 0; k < hn[2 * c] && k < RW_S0; ++k)
                if (hr[c * RW_SLOTS + k].start == so) { r = &hr[c * RW_SLOTS + k]; break; }
            const bool lastc = c + 1 == nchunks;
            const RwRec* r1 = lastc ? hr + nchunks * RW_SLOTS : hr + c * RW_SLOTS + RW_S0;
            for (u32 k = 0; !r && k < hn[2 * c + 1] && k < (lastc ? RW_SLAST : RW_S1); ++k)
                if (r1[k].start == so) { r = &r1[k]; break; }
        }
        if (r) {
            const u32 cnt = r->cs & 0x7FFFFFFFu;
            last = (r->cs >> 31) != 0 || r->exit >= len || (u64)nfc + cnt >= max_frames;
            ht.push_back(ent);
            ht.push_back(last ? len : r->exit);
            ht.push_back(nfc);
            ht.push_back(last ? 1 : 0);
            nfc += cnt;
            ent = r->exit;
            continue;
        }
        if ((ws_dbg_flags & 16) && ws_stat_rw_chunk_walks < 6 && c < nchunks) {
            fprintf(stderr, "rw: chunk %llu/%llu C %llu H %u entry +%llu n0 %u n1 %u:", (unsigned long long)c,
                    (unsigned long long)nchunks, (unsigned long long)C, H, (unsigned long long)(ent - cs0),
                    hn[2 * c], hn[2 * c + 1]);
            for (u32 k = 0; k < hn[2 * c] && k < RW_S0; ++k)
                fprintf(stderr, " [%u %u]", hr[c * RW_SLOTS + k].start, hr[c * RW_SLOTS + k].cs);
            fprintf(stderr, "\n");
        }
        u64 nx = 0;
        u32 nfn = 0;
        if ((rc = chunk_walk(ent, nfc, cs0 + C, nx, nfn)) < 0) return rc;
        last = rc == 1;                                                      // it finished the stream
        ent = nx;
        nfc = nfn;
    }
    const u32 nb = (u32)(ht.size() / 4);
    ws_stat_rw_chunks = nb;
    if (nb) {
        if ((e = hipMemcpyAsync(tab, ht.data(), ht.size() * 8, hipMemcpyHostToDevice, st)) != hipSuccess)
            return ws_set_err("hipMemcpyAsync(stream chain)", e);
        hipLaunchKernelGGL(ws_rw_emit_kernel, dim3(nb), dim3(64), 0, st, d_buf, len, max_frames, tab, d_desc,
                           Pw.items, Pw.ptr, Pw.npieces, Pw.nwork, d_res);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_rw_emit_kernel launch", e);
    }
    // `ht` is pageable host memory read by the copy above: complete it before returning
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return ws_set_err("hipStreamSynchronize", e);
    return 0;
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeStreamDecodeDevice(unsigned char* d_buf, unsigned long long len,
                                                                   unsigned int max_frames,
                                                                   WebsocketFrameDesc_t* d_desc,
                                                                   WebsocketSegResult_t* d_res, void* hip_stream) {
    if (!d_buf || !d_desc || !d_res || max_frames == 0) return ws_set_msg("websocketframeStreamDecodeDevice: invalid argument");
    if ((reinterpret_cast<uintptr_t>(d_desc) | reinterpret_cast<uintptr_t>(d_res)) & 15)
        return ws_set_msg("websocketframeStreamDecodeDevice: d_desc/d_res not 16-B aligned");
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    hipError_t e;
    // workspace: the piece path's layout for one segment [0, len), plus the stop word and the
    // segment's (offset, length) pair for the unmask kernel
    const size_t pws = ws_piece_workspace_bytes(len, 1, max_frames);
    void* ws = nullptr;
    int rc = ws_device_workspace(pws + 256, st, &ws);
    if (rc) return rc;
    unsigned char* w8 = reinterpret_cast<unsigned char*>(ws);
    unsigned long long* d_stop = reinterpret_cast<unsigned long long*>(w8 + ((pws + 63) & ~(size_t)63));
    u64* d_seg = reinterpret_cast<u64*>(d_stop + 2);                        // [0] offset 0, [1] length
    const u64 seg[2] = {0, len};
    if ((e = hipMemcpyAsync(d_seg, seg, sizeof(seg), hipMemcpyHostToDevice, st)) != hipSuccess)
        return ws_set_err("hipMemcpyAsync(segment)", e);
    WsLaunch L;
    L.buf = d_buf; L.seg_off = d_seg; L.seg_len = d_seg + 1; L.nseg = 1; L.max_frames = max_frames;
    L.desc_base = nullptr; L.desc = d_desc; L.res = d_res; L.stream = st; L.cus = 0;
    PieceWs Pw;
    const u32 gen = ws_next_gen();
    // the piece-path views of the workspace (no kernel launched: lo == hi == 0 segments walk)
    {
        const u64 lead0 = reinterpret_cast<uintptr_t>(d_buf) & 15;
        Pw.npieces = len + lead0 ? ((len + lead0 - 1) >> PIECE_SHIFT_S) + 1 : 0;
        Pw.pbase = 0;
        Pw.c_lo = 0;
        Pw.c_hi = (len + lead0 + 15) >> 4;
        Pw.disorder = reinterpret_cast<u32*>(w8);
        Pw.ptr = reinterpret_cast<u64*>(w8 + 16);
        size_t b = (16 + Pw.npieces * 8 + 15) & ~(size_t)15;
        Pw.nwork = reinterpret_cast<u32*>(w8 + b);
        b = (b + 4 + 15) & ~(size_t)15;
        Pw.items = reinterpret_cast<u32x4*>(w8 + b);
    }
    const u64 lead0 = reinterpret_cast<uintptr_t>(d_buf) & 15;
    auto set_ptrs = [&](u64 lo, u64 hi, u64 val, u64 item, int lo_it, int hi_it) -> int {
        hipLaunchKernelGGL(ws_stream_ptr_kernel, dim3(1), dim3(256), 0, st, Pw.ptr, Pw.npieces, lo, hi, val, Pw.items,
                           item, lo_it, hi_it);
        hipError_t e2 = hipGetLastError();
        return e2 == hipSuccess ? 0 : ws_set_err("ws_stream_ptr_kernel launch", e2);
    };
    u64 P = 0, g = 0;
    u32 nf = 0, extra = 0, short_passes = 0;
    int status = WEBSOCKET_SEG_OK;
    bool walked = false;
    bool probe = true;                       // after a length change: a short pass first (a stream
                                             // whose lengths keep changing never pays a full one)
    for (;;) {
        const u64 remaining = len - P;
        u64 K = g ? remaining / g + 1 : 1;                                   // candidates this pass
        if (K > (u64)max_frames - nf + 1) K = (u64)max_frames - nf + 1;
        if (K > (probe ? (1ull << 12) : (1ull << 26))) K = probe ? (1ull << 12) : (1ull << 26);
        const unsigned long long none = ~0ull;
        if ((e = hipMemcpyAsync(d_stop, &none, 8, hipMemcpyHostToDevice, st)) != hipSuccess)
            return ws_set_err("hipMemcpyAsync(stop)", e);
        hipLaunchKernelGGL(ws_stream_pass_kernel, dim3((u32)((K + SPASS_T - 1) / SPASS_T)), dim3(SPASS_T), 0, st, d_buf,
                           (u64)len, P, g, nf, max_frames, K, d_desc, Pw.items, Pw.ptr, Pw.npieces, d_stop);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_stream_pass_kernel launch", e);
        unsigned long long word = 0;
        if ((e = hipMemcpyAsync(&word, d_stop, 8, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return ws_set_err("hipMemcpyAsync(stop D2H)", e);
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return ws_set_err("hipStreamSynchronize", e);
        if (word == ~0ull) {                                                 // all K candidates were g-frames
            nf += (u32)K;
            P += K * g;
            short_passes = 0;
            probe = false;
            continue;
        }
        probe = true;
        const u64 m = word >> 36;
        const u32 code = (u32)(word >> 34) & 3u, stf = (u32)(word >> 32) & 3u;
        const int ret = (int)(u32)word;
        const u64 pos_m = P + m * g;
        const u64 slot_m = (u64)nf + m;
        nf += (u32)m;
        if (code == 1) {
            // frame m is longer than g: later candidates may have written pointers inside it
            if ((rc = set_ptrs(lead0 + pos_m, lead0 + pos_m + (u32)ret, slot_m, 0, 0, 0))) return rc;
            nf += 1;
            P = pos_m + (u32)ret;
            g = (u32)ret;
            if (P >= len) break;                                             // consumed the whole stream
            if (m < 64 && ++short_passes >= 2) {                             // lengths keep changing:
                if (ws_stream_rw && len - P >= RW_MIN) {                     // chunk-parallel walk
                    if ((rc = rw_walk(d_buf, len, P, nf, max_frames, d_desc, Pw, d_res, st))) return rc;
                } else {                                                     // one wavefront
                    hipLaunchKernelGGL(ws_stream_walk_kernel, dim3(1), dim3(64), 0, st, d_buf, (u64)len, P, g, nf,
                                       max_frames, d_desc, Pw.items, Pw.ptr, Pw.npieces, Pw.nwork, d_res);
                    if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_stream_walk_kernel launch", e);
                }
                walked = true;                                               // it writes result and tail
                break;
            }
            continue;
        }
        P = pos_m;
        if (code == 2) {                                                     // ret <= 0: unmasked, walk ends
            if (ret != 0) { nf += 1; status = WEBSOCKET_SEG_ERR_DECODE; }
            else extra = 1;
            if ((rc = set_ptrs(lead0 + pos_m, 0, slot_m, slot_m, 0, 1))) return rc;       // its payload
            if ((rc = set_ptrs(0, lead0 + len, (u64)nf + extra, slot_m, 1, 0))) return rc;  // the rest
        } else {
            status = stf == 1 ? WEBSOCKET_SEG_MAX_FRAMES : (stf == 2 ? WEBSOCKET_SEG_ERR_LEN_WRAP : WEBSOCKET_SEG_OK);
            if ((rc = set_ptrs(lead0 + pos_m, lead0 + len, nf, 0, 0, 0))) return rc;
        }
        break;
    }
    if (!walked) {
        hipLaunchKernelGGL(ws_stream_res_kernel, dim3(1), dim3(1), 0, st, Pw.nwork, nf + extra, d_res,
                           P < len ? P : (u64)len, nf, status);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_stream_res_kernel launch", e);
    }
    if ((e = hipMemsetAsync(Pw.disorder, 0, 4, st)) != hipSuccess) return ws_set_err("hipMemsetAsync", e);
    return ws_launch_piece_unmask(L, Pw, 1, gen);
}
