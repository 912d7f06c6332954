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
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "ws_common.h"

#define SPASS_T 256
#define PIECE_SHIFT_S WS_PIECE_SHIFT

// outcome bits packed with the candidate index: k << 36 | code << 34 | stf << 32 | (u32)ret
//   code 1: consumed, length != g   2: consumed, walk ends (ret <= 0)   3: not consumed
//   stf (code 3): 0 OK, 1 MAX_FRAMES, 2 LEN_WRAP; (code 2): 0 ret == 0, 1 ret < 0
__device__ __forceinline__ void stream_pass_one(const unsigned char* __restrict__ buf, u64 len, u64 P, u64 g, u32 nf,
                                                u32 max_frames, u64 k, WebsocketFrameDesc_t* __restrict__ desc,
                                                u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                                unsigned long long* __restrict__ stop) {
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
        atomicMax(stop, ~word);                                              // the first stop, inverted
    }
}

// The pass loop's state, device-resident (the first bytes of the calling stream's auxiliary
// workspace): the host never has to read it, so a decode of any stream can be one
// asynchronous launch sequence. It RESTS at zero between calls — stop words 0 (= no stop:
// they hold ~word, merged with atomicMax), ticket 0 — so a call needs no init kernel: the
// first round starts from (P, nf) = (0, 0) without reading it, and every resolve leaves the
// stop words and the ticket at zero again.
#define SD_PASSES 0u      // the grid passes go on
#define SD_WALK 1u        // lengths keep changing: the rest is walked (chunk-parallel or one wavefront)
#define SD_DONE 2u        // result, item count and tail pointers are written
#define SD_PROBE_K 4096ull
#define SD_KMAX (1ull << 26)
struct SdState {
    u64 P;                           // next frame offset (every frame before it is confirmed)
    u64 g;                           // the last confirmed frame's length
    unsigned long long stop[2];      // pass A / pass B: ~(packed first stop), 0: none
    u32 ticket;                      // resolve blocks done (the last one writes the state)
    u32 nf, extra, short_passes, phase;
    int status;
    u32 walk_hint;                   // captured calls: the last chunk walk's hint (next replay: no rounds)
};
static_assert(sizeof(SdState) <= 128, "stream state");
struct SdMirror {                    // pinned host copy of the state after a resolve (eager calls)
    u64 P, g;
    u32 nf, phase, gen;
    u32 walk_hint;                   // the last chunk walk's sample: lengths kept changing (next call: no rounds)
};

// reset of a state left dirty by a call that failed between its launches (rare)
__global__ void ws_stream_init_kernel(SdState* __restrict__ sd) {
    sd->stop[0] = sd->stop[1] = 0;
    sd->ticket = 0;
}

// the stride at P: the length of the frame there (0 when it is not a complete frame with a
// positive return: then only candidate 0 exists), and the candidate count of a pass
__device__ __forceinline__ void sd_stride(const unsigned char* __restrict__ buf, u64 len, u64 P, u32 nf,
                                          u32 max_frames, u64& g, u64& K) {
    g = 0;
    if (P < len && len - P >= 2) {
        const uintptr_t pa = reinterpret_cast<uintptr_t>(buf + P);
        const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
        u64 h0, h1;
        ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
        const WsHdr h = ws_parse(h0, h1, len - P);
        if (h.kind == WS_PARSE_FRAME && h.ret > 0) g = (u32)h.ret;
    }
    u64 kf = g ? (len - P) / g + 1 : 1;
    if (kf > (u64)max_frames - nf + 1) kf = (u64)max_frames - nf + 1;
    K = kf < SD_KMAX ? kf : SD_KMAX;
}

// One pass of the loop: part 0 (A) takes candidates [0, SD_PROBE_K), part 1 (B) the rest
// and runs only if A confirmed all of its candidates. From the last confirmed frame
// (P, nf) thread k parses the header at P + k*g (g: the length of the frame at P);
// candidates are ordered, so the pair is exactly one pass over [0, K). `first`: the call's
// first round, from (0, 0) — its pass A also writes the unmask's segment pair and clears
// the unmask's gate word.
__global__ __launch_bounds__(SPASS_T) void ws_stream_pass_kernel(const unsigned char* __restrict__ buf, u64 len,
                                                                 u32 max_frames, int part, int first,
                                                                 WebsocketFrameDesc_t* __restrict__ desc,
                                                                 u32x4* __restrict__ items, u64* __restrict__ ptr,
                                                                 u64 pend, SdState* __restrict__ sd,
                                                                 u64* __restrict__ seg, u32* __restrict__ disorder,
                                                                 int dev_hint) {
    if (dev_hint && sd->walk_hint) return;                                   // the chunk walk starts at 0
    if (first && part == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
        seg[0] = 0;
        seg[1] = len;
        *disorder = 0;
    }
    if ((!first && sd->phase != SD_PASSES) || (part == 1 && sd->stop[0] != 0)) return;   // the same for every block
    const u64 P = first ? 0 : sd->P;
    const u32 nf = first ? 0 : sd->nf;
    u64 g, K;
    sd_stride(buf, len, P, nf, max_frames, g, K);
    const u64 k0 = part ? SD_PROBE_K : 0, k1 = part ? K : (K < SD_PROBE_K ? K : SD_PROBE_K);
    for (u64 k = k0 + (u64)blockIdx.x * SPASS_T + threadIdx.x; k < k1; k += (u64)gridDim.x * SPASS_T)
        stream_pass_one(buf, len, P, g, nf, max_frames, k, desc, items, ptr, pend, &sd->stop[part]);
}

// Frames of the stream starting in [P0, end) from (P0, nf0, g0) by one wavefront: the group
// walk of ws_piece.hip (stride speculation; only consumed frames are written). The
// speculative width adapts: 64 lanes while runs of equal lengths hold, 2 (k + 1) lanes after a
// length change at lane k (at least 4), doubling after every step whose lanes all confirmed —
// on lengths that change every frame a step loads 4 header lines instead of 64.
// `last`: the walk runs to the stream's end (end == len) and then writes the tail
// pointers, the item count and the segment result; otherwise it stops before the first
// frame starting at or after `end` (another wavefront owns it).
struct SwOut {            // where a stream_walk stopped: the next frame, its index, 1 if the walk ended
    u64 next;
    u32 nf, ended;
    u32 steps;            // header rounds the walk took (a run of equal frames takes one per 64)
    u32 maxlen;           // the longest frame it took (wire bytes; only when asked: want_max)
    u32 cnt;              // the item count a finishing walk writes (frames + an unconsumed ret == 0 frame)
};
__device__ __forceinline__ SwOut stream_walk(const unsigned char* __restrict__ buf, u64 len, u64 P0, u64 g0, u32 nf0,
                                            u64 end, bool last, u32 max_frames, WebsocketFrameDesc_t* __restrict__ desc,
                                            u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                            u32* __restrict__ nwork, WebsocketSegResult_t* __restrict__ res,
                                            u32 lane, u64* __restrict__ out = nullptr, bool want_max = false) {
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    const uintptr_t seg = reinterpret_cast<uintptr_t>(buf);
    u64 off = P0, g = g0, walked_end = lead0 + P0;
    u32 nf = nf0, extra = 0;
    int status = WEBSOCKET_SEG_OK;
    bool at_bnd = false;
    u32 steps = 0, mx = 0, w = 64;
    for (;;) {
        ++steps;
        const u32 wl = g > 0 ? w : 1u;                                      // lanes evaluated
        const u64 pos = off + (u64)lane * g;
        const bool cand = lane < wl;
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
        const u64 stopm = __ballot(cand && code != 0);
        const u32 mm = stopm ? (u32)__builtin_ctzll(stopm) : wl;
        const u32 code_m = stopm ? (u32)__builtin_amdgcn_readlane((int)code, (int)mm) : 0u;
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
        if (want_max && lane < ntake && h.ret > 0 && (u32)h.ret > mx) mx = (u32)h.ret;
        if (!stopm) {                                                        // every evaluated lane confirmed
            nf += wl;
            off += (u64)wl * g;
            w = w < 32 ? 2 * w : 64;
            continue;
        }
        const u64 pos_m = off + (u64)mm * g;
        const int ret_m = __builtin_amdgcn_readlane(h.ret, (int)mm);
        nf += mm;
        if (code_m == 1) {                                                   // (g 0: the first frame, no history)
            nf += 1;
            off = pos_m + (u32)ret_m;
            w = g == 0 ? 64u : (mm < 2 ? 4u : (mm < 32 ? 2 * (mm + 1) : 64u));
            g = (u32)ret_m;
            continue;
        }
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
    SwOut r;
    r.next = off;
    r.nf = nf;
    r.ended = at_bnd ? 0u : 1u;
    r.steps = steps;
    r.maxlen = 0;
    r.cnt = nf + extra;
    if (want_max) {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const u32 o2 = (u32)__shfl_xor((int)mx, d);
            mx = o2 > mx ? o2 : mx;
        }
        r.maxlen = mx;
    }
    if (!last && (at_bnd || !out)) return r;
    const u32 cnt = nf + extra;
    for (u64 p = ((walked_end + (1ull << PIECE_SHIFT_S) - 1) >> PIECE_SHIFT_S) + lane;
         (p << PIECE_SHIFT_S) < lead0 + len && p < pend; p += 64)
        ptr[p] = cnt;
    if (lane == 0) {
        nwork[0] = cnt;
        ws_store_res(res, off, nf, status);
    }
    return r;
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

// After a pass pair: its stop applied to the state (the host loop of earlier versions, in
// net_reactor.c:515-526 order): advance past a run of g-frames, take a frame of another
// length (a new stride; its pieces point at it again, later candidates may have written
// them), or end the walk (ret <= 0, not consumed, max frames: the rest of the pieces point
// past the items) and write the result. A pass that found a new length within its first 64
// candidates twice hands the rest to a walk (SD_WALK). Every block derives the same
// outcome and writes its share of the piece pointers; the last block to finish (ticket)
// writes the state, after every block has read it, and resets the stop words. `finish`
// (the last round of a call that does not read the state back): that block's first wave
// also walks whatever is left, one wavefront from (P, g, nf) to the end. `mirror` (eager
// calls): the state is published to pinned host memory, tagged with the call's `gen`.
__global__ __launch_bounds__(SPASS_T) void ws_stream_resolve_kernel(const unsigned char* __restrict__ buf, u64 len,
                                                                    u32 max_frames, int first, int finish,
                                                                    WebsocketFrameDesc_t* __restrict__ desc,
                                                                    u32x4* __restrict__ items, u64* __restrict__ ptr,
                                                                    u64 pend, SdState* __restrict__ sd,
                                                                    u32* __restrict__ nwork,
                                                                    WebsocketSegResult_t* __restrict__ res,
                                                                    SdMirror* __restrict__ mirror, u32 gen,
                                                                    int dev_hint) {
    __shared__ u64 f_lo[2], f_hi[2], f_val[2];
    __shared__ int s_last;
    if (dev_hint && sd->walk_hint) return;
    if (!first && sd->phase != SD_PASSES) {                                  // nothing left to resolve
        if (finish && blockIdx.x == 0 && threadIdx.x < 64 && sd->phase != SD_DONE)
            stream_walk(buf, len, sd->P, sd->g, sd->nf, len, true, max_frames, desc, items, ptr, pend, nwork, res,
                        threadIdx.x);
        return;
    }
    const u64 P = first ? 0 : sd->P;
    const u32 nf = first ? 0 : sd->nf;
    const unsigned long long word = sd->stop[0] ? ~sd->stop[0] : ~sd->stop[1];   // candidates are ordered
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    u64 g, K;
    sd_stride(buf, len, P, nf, max_frames, g, K);
    u64 P2 = P + K * g, g2 = g;
    u32 nf2 = nf + (u32)K, extra = 0, short_passes = 0, phase = SD_PASSES;
    int status = WEBSOCKET_SEG_OK;
    if (threadIdx.x == 0) {
        f_lo[0] = f_hi[0] = f_lo[1] = f_hi[1] = 0;
        f_val[0] = f_val[1] = 0;
    }
    __syncthreads();
    if (word != ~0ull) {
        const u64 m = word >> 36;
        const u32 code = (u32)(word >> 34) & 3u, stf = (u32)(word >> 32) & 3u;
        const int ret = (int)(u32)word;
        const u64 pos_m = P + m * g;
        const u64 slot_m = (u64)nf + m;
        nf2 = nf + (u32)m;
        P2 = pos_m;
        short_passes = first ? 0u : sd->short_passes;
        phase = SD_DONE;
        if (code == 1) {
            if (threadIdx.x == 0) { f_lo[0] = lead0 + pos_m; f_hi[0] = lead0 + pos_m + (u32)ret; f_val[0] = slot_m; }
            nf2 += 1;
            P2 = pos_m + (u32)ret;
            g2 = (u32)ret;
            if (P2 < len) {                                                  // else: consumed the whole stream
                phase = SD_PASSES;
                if (m < 64 && ++short_passes >= 2) phase = SD_WALK;
            }
        } else if (code == 2) {                                              // ret <= 0: unmasked, walk ends
            if (ret != 0) { nf2 += 1; status = WEBSOCKET_SEG_ERR_DECODE; }
            else extra = 1;
            // its payload extent: the header at pos_m again (the buffer is not written yet)
            const uintptr_t pa = reinterpret_cast<uintptr_t>(buf + pos_m);
            const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
            u64 h0, h1;
            ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
            const WsHdr h = ws_parse(h0, h1, len - pos_m);
            const u64 p1 = lead0 + pos_m + h.hdr + (h.masked ? h.plen : 0);
            if (threadIdx.x == 0) {
                f_lo[0] = lead0 + pos_m; f_hi[0] = p1; f_val[0] = slot_m;
                f_lo[1] = p1; f_hi[1] = lead0 + len; f_val[1] = (u64)nf2 + extra;
            }
        } else {
            status = stf == 1 ? WEBSOCKET_SEG_MAX_FRAMES : (stf == 2 ? WEBSOCKET_SEG_ERR_LEN_WRAP : WEBSOCKET_SEG_OK);
            if (threadIdx.x == 0) { f_lo[0] = lead0 + pos_m; f_hi[0] = lead0 + len; f_val[0] = nf2; }
        }
    }
    __syncthreads();
    const u64 t0 = (u64)blockIdx.x * SPASS_T + threadIdx.x, ts = (u64)gridDim.x * SPASS_T;
#pragma unroll
    for (int f = 0; f < 2; ++f)
        for (u64 p = ((f_lo[f] + (1ull << PIECE_SHIFT_S) - 1) >> PIECE_SHIFT_S) + t0; (p << PIECE_SHIFT_S) < f_hi[f] && p < pend;
             p += ts)
            ptr[p] = f_val[f];
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&sd->ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x == 0) {
        sd->ticket = 0;
        sd->stop[0] = sd->stop[1] = 0;
        sd->P = P2;
        sd->g = g2;
        sd->nf = nf2;
        sd->short_passes = short_passes;
        sd->phase = phase;
        if (phase == SD_DONE) {
            sd->extra = extra;
            sd->status = status;
            nwork[0] = nf2 + extra;
            ws_store_res(res, P2 < len ? P2 : len, nf2, status);
        }
        if (mirror) {
            mirror->P = P2;
            mirror->g = g2;
            mirror->nf = nf2;
            mirror->phase = phase;
            __threadfence_system();
            __hip_atomic_store(&mirror->gen, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // the rest of a stream whose lengths keep changing (or whose rounds ran out): one wavefront
    if (finish && phase != SD_DONE && threadIdx.x < 64)
        stream_walk(buf, len, P2, g2, nf2, len, true, max_frames, desc, items, ptr, pend, nwork, res, threadIdx.x);
}

// Whatever an eager call's rounds left, when the chunk-parallel walk does not apply: one
// wavefront walks from the state's (P, g, nf) to the end
__global__ __launch_bounds__(64) void ws_stream_finish_kernel(const unsigned char* __restrict__ buf, u64 len,
                                                              u32 max_frames, WebsocketFrameDesc_t* __restrict__ desc,
                                                              u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                                              u32* __restrict__ nwork,
                                                              WebsocketSegResult_t* __restrict__ res,
                                                              const SdState* __restrict__ sd) {
    if (sd->phase == SD_DONE) return;
    stream_walk(buf, len, sd->P, sd->g, sd->nf, len, true, max_frames, desc, items, ptr, pend, nwork, res, threadIdx.x);
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
#define RW_CMAX (16ull << 20)
#define RW_CMIN (64ull << 10)
#define RW_HMAX (128u << 10)
#define RW_HMIN (4u << 10)
#define RW_SAMPLE (256ull << 10)
#define RW_S0 40          // records per chunk of walks that leave it (~8-16 true frame starts)
#define RW_S1 8           // ... of walks that end the stream in it
#define RW_SLOTS (RW_S0 + RW_S1)
#define RW_SLAST 4096     // walks that end the stream in the last chunk
#define RW_MAXSTEPS 65536
#define RW_TPOS 64        // window positions per thread
#define RW_D 4            // distinct window exits per chunk walked on (phase B owners)
#define RW_STG 4096       // largest staging list per owner (frame offsets); the call's is stgn
#define RW_MIN (512ull << 10)     // streams shorter than this after the passes: one wavefront walks
#define RW_MIN_FRAMES 256         // ... and, after the sample, fewer frames than this (by the mean)
// captured (device-planned) calls: R1 and R2 grid-stride grids, blocks of 256 (round 5: R1
// 4096 -> 16384 blocks 176.8 -> 160.8 us, R2 4096 -> 8192 42.9 -> 36.9 us on cfg3,
// profiles/r05_stream_grid_ab.log)
#define RW_R1_GRID 16384
#define RW_R2_GRID 8192
#define RW_WCAP 256       // R1: candidates of a wave spread over its lanes (more: lane by lane)

__host__ __device__ static u64 rw_pow2_clamp(u64 x, u64 lo, u64 hi) {
    u64 v = lo;
    while (v < x && v < hi) v <<= 1;
    return v;
}

// The window at each chunk's start must hold a frame start of the chain: any window longer
// than every frame does. 4 mean frames or the sample's longest frame + 4 KiB, whichever is
// larger, in 4 KiB steps, within [RW_HMIN, min(C / 2, RW_HMAX)] (round 3: 8 mean frames
// rounded up to a power of two; cfg3 128 -> 92 KiB, stream 8.32-8.36 -> 8.19 ms eager,
// profiles/r04_stream_rw_ab.log)
__device__ static u32 rw_window(u64 mean, u32 maxlen, u64 C) {
    // (round 5: 0, 2 or 4 mean frames measured the same on one buffer, R1 unchanged at 247 us)
    const u64 hi = C / 2 < RW_HMAX ? C / 2 : RW_HMAX;
    u64 h = mean * 4 > (u64)maxlen + 4096 ? mean * 4 : (u64)maxlen + 4096;
    h = (h + 4095) & ~4095ull;
    return (u32)(h < RW_HMIN ? RW_HMIN : (h > hi ? hi : h));
}

struct RwRec {            // phase A: one surviving walk from chunk start + start
    u32 start;
    u32 cs;               // frames consumed | status << 31 (0 left the window, 1 the stream's walk ends)
    u64 exit;             // the next frame start (status 0) or where the walk ended
};

struct RwOwn {            // phase B: the walk from a window exit to the chunk's end
    u64 exit;             // the next frame start (left the chunk) or where the stream's walk ends
    u32 cs;               // frames | status << 31
    u32 dead;             // 1: an implausible header (not the chain)
    u64 over;             // the (stgn+1)-th frame's start when more than stgn frames
    u64 pad;
};

// The walk's geometry chosen on the device (captured calls: the host cannot read the sample):
// R1-R3, the linker and the emit take it from here; scratch is sized for the caps at capture.
// Round 6: the rest of the stream after the sample is one to RW_NP PARTS, each a chunk grid of
// its own. With a split (stream_split), part 0 = [P, B1) in small chunks (its owner walks are
// short: it is the walk K2's first launch waits for), the last part = [B_last, len) in large
// chunks, and (stream_split2) a middle part; the parts after part 0 are walked on a side stream
// beside K2's launches over the earlier parts' pieces. Chunk arrays are indexed by the global
// chunk g = cbase + local index; per-part lists start at their bases.
struct RwPart {
    u64 P;                // the part's chunk grid origin
    u64 C;                // its chunk bytes
    u32 H, n, cbase, capc; // window bytes, chunks, first global chunk, candidates per chunk
    u32 stgn, pad;        // staging per owner
    u64 stg_base, cand_base;  // where its staging and candidate lists start (entries)
};
#define RW_NP 3           // parts of a split walk at most
struct RwPlan {
    RwPart pt[RW_NP];     // parts past nparts empty (n = 0)
    u32 nchunks;          // sum of the parts' chunks (global chunk count)
    u32 need_mask, active, nf;   // nf: frames before pt[0].P
    u32 nparts, seen_max; // seen_max: the longest frame the previous walk on this stream wrote (emit, linker)
    u32 nrows[RW_NP], linked[RW_NP];   // emit rows of each part (rows at tab[cbase + r]); linked: rows final
    u64 sample_out[4];    // stream_walk's report of the sample / of a linked chunk walk
    // the hand-off into part k (k >= 1): the chain's entry, the frames before it, and its state —
    // 0 not yet, 1 part k continues at in_ent[k], 2 the walk ended before part k
    u64 in_ent[RW_NP];
    u32 in_nf[RW_NP], in_state[RW_NP];
    u32 nw[RW_NP];        // the item count K2's launch k reads (k < nparts - 1): every item it may need is written
};
static_assert(sizeof(RwPlan) <= WS_AUX_ZERO - WS_AUX_HEAD, "RwPlan lies in the zeroed aux range (WS_AUX_ZERO)");

// the walk ended in part `part` with `cnt` items: every later K2 launch reads the final count, every
// later part is a no-op (one thread)
__device__ __forceinline__ void rw_end_counts(RwPlan* plan, int part, u32 cnt) {
    for (int k = part; k < RW_NP; ++k) plan->nw[k] = cnt;
}
__device__ __forceinline__ void rw_end_states(RwPlan* plan, int part) {
    for (int k = part + 1; k < RW_NP; ++k) plan->in_state[k] = 2;
}
// part `part` hands the chain over to the next part at `ent` with `nf` frames before it (one thread)
__device__ __forceinline__ void rw_hand_over(RwPlan* plan, int part, u64 ent, u32 nf) {
    plan->in_ent[part + 1] = ent;
    plan->in_nf[part + 1] = nf;
    plan->nw[part] = nf;
    plan->in_state[part + 1] = 1;
}

// a kernel's chunk grid: the plan's part (device-planned calls) or the host's arguments
struct RwGeo {
    u64 P, C;
    u32 H, n, cbase, capc, stgn, nall, need_mask;
    u64 stg_base, cand_base;
};
__device__ __forceinline__ RwGeo rw_geo(const RwPlan* plan, int part, u64 P, u64 C, u32 H, u32 nchunks, u32 capc,
                                        u32 stgn, u32 need_mask) {
    RwGeo G;
    if (plan) {
        const RwPart& t = plan->pt[part];
        G.P = t.P; G.C = t.C; G.H = t.H; G.n = t.n; G.cbase = t.cbase; G.capc = t.capc; G.stgn = t.stgn;
        G.nall = plan->nchunks; G.need_mask = plan->need_mask; G.stg_base = t.stg_base; G.cand_base = t.cand_base;
    } else {
        G.P = P; G.C = C; G.H = H; G.n = nchunks; G.cbase = 0; G.capc = capc; G.stgn = stgn; G.nall = nchunks;
        G.need_mask = need_mask; G.stg_base = 0; G.cand_base = 0;
    }
    return G;
}

// a wavefront's longest frame -> the plan's seen_max (the next call's windows cover it)
__device__ __forceinline__ void rw_note_max(const RwPlan* plan, u32 mx, u32 lane) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const u32 o = (u32)__shfl_xor((int)mx, d);
        mx = o > mx ? o : mx;
    }
    if (plan && lane == 0 && mx) atomicMax(const_cast<u32*>(&plan->seen_max), mx);
}

// b23: header bytes 2 and 3 (the top of a 64-bit length, which a real frame leaves zero:
// a random 64-bit length reads as an incomplete frame and would crowd the records)
__device__ __forceinline__ bool rw_plausible(u32 b0, u32 b1, u32 b23, bool need_mask) {
    const u32 op = b0 & 15u;
    return !(b0 & 0x70u) && (op <= 2u || (op >= 8u && op <= 10u)) && (!need_mask || (b1 & 0x80u)) &&
           ((b1 & 0x7Fu) != 127u || b23 == 0u);
}

// One speculative step at pos: 0 frame (pos advanced), 1 the stream's walk ends at pos,
// 2 implausible header (a wrong start)
__device__ __forceinline__ u32 rw_step(uintptr_t origin, u64 len, u64& pos, bool need_mask) {
    if (pos >= len || len - pos < 2) return 1;                               // websocketframe.c:121
    const uintptr_t pa = origin + pos;
    const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
    u64 h0, h1;
    ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
    if (!rw_plausible((u32)h0 & 0xFFu, (u32)(h0 >> 8) & 0xFFu, (u32)(h0 >> 16) & 0xFFFFu, need_mask)) return 2;
    const WsHdr h = ws_parse(h0, h1, len - pos);
    if (h.kind != WS_PARSE_FRAME || h.ret <= 0) return 1;
    pos += (u32)h.ret;
    return 0;
}

// R1 (candidates): one thread per RW_TPOS window positions (aligned 16-B loads); the
// plausible positions of a wavefront are appended to its chunk's list (capc slots) with
// one atomic per wave on the chunk's counter
// (lanes are dense in R2: a wrong start costs one lane-slot, not a wavefront-slot).
// A candidate whose frame is followed by an implausible header inside its chunk is dropped
// here (R2 would drop it at that step: its second header), so the list holds only starts that
// survive two headers (cfg3: R2 150 -> 24 us, R1 + R2 279 -> 154 us with the windows below)
__global__ __launch_bounds__(256) void ws_rw_cand_kernel(const unsigned char* __restrict__ buf, u64 len, u64 P,
                                                         u64 C, u32 H, u32 nchunks, u32 need_mask,
                                                         u64* __restrict__ cand, u32* __restrict__ nrec, u32 capc,
                                                         const RwPlan* __restrict__ plan, int part) {
    if (plan && !plan->active) return;
    const RwGeo G = rw_geo(plan, part, P, C, H, nchunks, capc, 0, need_mask);   // geometry from the device
    P = G.P; C = G.C; H = G.H; need_mask = G.need_mask; capc = G.capc;
    const u32 lane = threadIdx.x & 63;
    __shared__ unsigned short s_cand[256 / 64][RW_WCAP];                     // a wave's candidates (position in its 4 KiB)
    const u32 per = H / RW_TPOS;                                             // a multiple of 64: one
    // grid-stride (a captured call's grid is sized for the largest geometry); a whole
    // wavefront takes the same iterations
    for (u64 t = (u64)blockIdx.x * 256 + threadIdx.x;; t += (u64)gridDim.x * 256) {
    const u64 c = t / per;                                                   // chunk per wavefront (local)
    if (c >= G.n) return;
    const u64 gc = G.cbase + c;                                              // ... global
    const uintptr_t origin = reinterpret_cast<uintptr_t>(buf);
    const u64 cs0 = P + c * C;
    const uintptr_t a = ((origin + cs0) & ~(uintptr_t)15) + (t % per) * RW_TPOS;
    u64 cands = 0;
    if (a < origin + len) {
        // the thread's 64 positions and the 3 bytes after them: chunks 0..4 (chunk m only where
        // the scalar version read it, a + 16 m < origin + len + 16; else chunk 0, masked below)
        u32 w[4 * (RW_TPOS / 16) + 4];
#pragma unroll
        for (u32 m = 0; m <= RW_TPOS / 16; ++m) {
            const u32x4 x = reinterpret_cast<const gu32x4*>(a)[a + 16 * m < origin + len + 16 ? m : 0];
            w[4 * m] = x.x; w[4 * m + 1] = x.y; w[4 * m + 2] = x.z; w[4 * m + 3] = x.w;
        }
        // rw_plausible for 4 positions at once (SWAR: byte lane i = position 4q + i); the
        // per-byte tests leave their verdict in bit 7 of each byte
        const u32 H7 = 0x80808080u;
        auto zb = [](u32 x) -> u32 { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u; };  // byte == 0
#pragma unroll
        for (u32 q = 0; q < RW_TPOS / 4; ++q) {
            const u32 B0 = w[q], B1 = __builtin_amdgcn_alignbyte(w[q + 1], w[q], 1);
            const u32 B2 = __builtin_amdgcn_alignbyte(w[q + 1], w[q], 2), B3 = __builtin_amdgcn_alignbyte(w[q + 1], w[q], 3);
            const u32 rsv = zb(B0 & 0x70707070u);                                      // RSV bits clear
            const u32 opc = ~(((B0 & 0x07070707u) + 0x05050505u) << 4) & H7;        // opcode & 7 <= 2
            const u32 msk = need_mask ? (B1 & H7) : H7;                              // MASK when client
            const u32 l64 = ~zb((B1 & 0x7F7F7F7Fu) ^ 0x7F7F7F7Fu) | zb(B2 | B3);     // len 127: top bytes 0
            const u32 ok = rsv & opc & msk & l64 & H7;
            const u32 bits = (((ok >> 7) * 0x00204081u) >> 21) & 15u;               // bit 8i+7 -> bit i
            cands |= (u64)bits << (4 * q);
        }
        // positions inside [cs0, len) only
        const u64 p0 = a - origin;
        const u64 lo = cs0 > p0 ? cs0 - p0 : 0, hi = len - p0;                     // p0 < len
        u64 rm = hi >= 64 ? ~0ull : (1ull << hi) - 1;
        rm &= lo >= 64 ? 0ull : ~0ull << lo;
        cands &= rm;
    }
    // Each candidate is checked by its frame and the header after it (two dependent loads). Round 4
    // did that per lane, so a wave waited for its busiest lane's chain (≈ 5-6 candidates of 64
    // positions); round 5 spreads the wave's candidates over its 64 lanes through LDS, so a wave
    // takes ceil(candidates / 64) chains (round 4's per-lane batching of four measured no faster).
    const u32 wv = threadIdx.x >> 6;
    const u32 n = (u32)__builtin_popcountll(cands);
    u32 incl = n;                                                            // wavefront inclusive scan
#pragma unroll
    for (u32 d = 1; d < 64; d <<= 1) {
        const u32 v = (u32)__shfl_up((int)incl, d);
        if (lane >= d) incl += v;
    }
    const u32 total = (u32)__shfl((int)incl, 63);
    u64 rest = cands;                                                        // not staged (overflow)
    for (u32 o = incl - n; rest && o < RW_WCAP; ++o) {
        s_cand[wv][o] = (unsigned short)((lane << 6) | (u32)__builtin_ctzll(rest));
        rest &= rest - 1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const u64 pw0 = (a - origin) - (u64)lane * RW_TPOS;                      // lane 0's first position
    const u64 cend = cs0 + C;
    u64* cl = cand + G.cand_base + c * capc;
    const u32 staged = total < RW_WCAP ? total : RW_WCAP;
    // one verdict per lane per pass: survivors appended to the chunk's list (one atomic per pass)
    auto verdict = [&](bool have, u64 pos0) {
        bool keep = false;
        if (have) {
            u64 pos = pos0;
            keep = !(rw_step(origin, len, pos, need_mask) == 0 && pos < cend &&
                     rw_step(origin, len, pos, need_mask) == 2);
        }
        const u64 km = __ballot(keep);
        const u32 cnt = (u32)__builtin_popcountll(km);
        u32 ob = 0;
        if (lane == 0 && cnt) ob = atomicAdd(nrec + 4 * gc + 2, cnt);        // the chunk's counter
        ob = (u32)__shfl((int)ob, 0);
        if (keep) {
            const u32 o = ob + (u32)__builtin_popcountll(km & ((1ull << lane) - 1));
            if (o < capc) cl[o] = pos0;
        }
    };
    for (u32 r = 0; r < staged; r += 64) {
        const u32 idx = r + lane;
        const bool have = idx < staged;
        verdict(have, have ? pw0 + s_cand[wv][idx] : 0);
    }
    // a wave with more than RW_WCAP candidates: the rest lane by lane
    while (__ballot(rest != 0)) {
        const bool have = rest != 0;
        const u32 k = have ? (u32)__builtin_ctzll(rest) : 0u;
        rest &= rest ? rest - 1 : 0ull;
        verdict(have, (a - origin) + k);
    }
    __builtin_amdgcn_wave_barrier();                                         // s_cand reads before the next pass's writes
    }
}

// R2 (window walks): one lane per candidate (grid-stride), the walk to the window's end
// -> an A record {start, frames, exit_w}; a walk that left the window claims exit_w in
// dx[] (one walk per distinct exit: merged walks share it) for R3
__global__ __launch_bounds__(256) void ws_rw_spec_kernel(const unsigned char* __restrict__ buf, u64 len, u64 P,
                                                         u64 C, u32 H, u32 nchunks, u32 need_mask,
                                                         const u64* __restrict__ cand, u32 capc,
                                                         RwRec* __restrict__ recs, u32* __restrict__ nrec,
                                                         unsigned long long* __restrict__ dx,
                                                         const RwPlan* __restrict__ plan, int part) {
    if (plan && !plan->active) return;
    const RwGeo G = rw_geo(plan, part, P, C, H, nchunks, capc, 0, need_mask);
    P = G.P; C = G.C; H = G.H; need_mask = G.need_mask; capc = G.capc;
    nchunks = G.nall;                                                        // (the last chunk's pool)
    const uintptr_t origin = reinterpret_cast<uintptr_t>(buf);
    const u64 n = (u64)G.n * capc;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) {
        const u64 cl = i / capc, c = G.cbase + cl;                           // local, global chunk
        if (i - cl * capc >= nrec[4 * c + 2]) continue;                     // past the chunk's candidates
        const u64 start = cand[G.cand_base + i];
        const u64 cs0 = P + cl * C, cend = cs0 + C, wend = cs0 + H;
        u64 pos = start;
        u32 cnt = 0, r = 0;
        while (pos < wend && (r = rw_step(origin, len, pos, need_mask)) == 0) ++cnt;
        if (r == 2) continue;                                                // a wrong start
        if (r == 0) {
            // a wrong start just before the window's end crosses it in one jump: a few more
            // plausible headers past it before the walk may claim its exit
            u64 vp = pos;
            u32 vr = 0;
            for (u32 v = 0; v < 3 && vp < cend && (vr = rw_step(origin, len, vp, need_mask)) == 0; ++v) {
            }
            if (vr == 2) continue;
        }
        const u32 st = r;                                                    // 1: the walk ends in the window
        // the last chunk's window lies near the stream's end, where wrong starts read as
        // incomplete frames: its walks that end get a pool of their own
        const bool lastc = c + 1 == nchunks;
        const u32 slot = atomicAdd(nrec + 4 * c + st, 1u);
        if (slot < (st ? (lastc ? RW_SLAST : RW_S1) : RW_S0)) {
            RwRec rr;
            rr.start = (u32)(start - cs0);
            rr.cs = cnt | (st << 31);
            rr.exit = pos;
            recs[st && lastc ? (u64)nchunks * RW_SLOTS + slot : c * RW_SLOTS + (st ? RW_S0 : 0) + slot] = rr;
        }
        if (st) continue;
        for (u32 d = 0; d < RW_D; ++d) {
            const unsigned long long old = atomicCAS(dx + c * RW_D + d, 0ull, (unsigned long long)pos);
            if (old == 0ull || old == pos) break;
        }
    }
}

// R3 (chunk walks): one lane per claimed window exit, the walk to the chunk's end; the
// offsets of the frames it passes go to the staging list (the emit writes them in parallel)
#define RW_OWN_T 64       // one wavefront per block: the owner walks spread over every CU
__global__ __launch_bounds__(RW_OWN_T) void ws_rw_own_kernel(const unsigned char* __restrict__ buf, u64 len, u64 P, u64 C,
                                                        u32 nchunks, u32 need_mask,
                                                        const unsigned long long* __restrict__ dx,
                                                        RwOwn* __restrict__ own, u32* __restrict__ stg, u32 stgn,
                                                        const RwPlan* __restrict__ plan, int part) {
    if (plan && !plan->active) return;
    const RwGeo G = rw_geo(plan, part, P, C, 0, nchunks, 0, stgn, need_mask);
    P = G.P; C = G.C; need_mask = G.need_mask; stgn = G.stgn;
    const u64 ol = (u64)blockIdx.x * RW_OWN_T + threadIdx.x;                 // local owner index
    if (ol >= (u64)G.n * RW_D) return;
    const u64 oi = (u64)G.cbase * RW_D + ol;                                 // global
    u64 pos = dx[oi];
    if (!pos) return;
    const uintptr_t origin = reinterpret_cast<uintptr_t>(buf);
    const u64 c = ol / RW_D, cs0 = P + c * C, cend = cs0 + C;
    u32* sl = stg + G.stg_base + ol * stgn;
    u32 nb = 0, r = 0;
    u64 over = 0;
    while (pos < cend) {
        if (nb < stgn) sl[nb] = (u32)(pos - cs0);
        else if (nb == stgn) over = pos;
        if ((r = rw_step(origin, len, pos, need_mask)) != 0) break;
        ++nb;
        if (nb > RW_MAXSTEPS) { r = 2; break; }
    }
    RwOwn ow;
    ow.exit = pos;
    ow.cs = nb | ((r == 1 ? 1u : 0u) << 31);
    ow.dead = r == 2 ? 1u : 0u;
    ow.over = over;
    ow.pad = 0;
    own[oi] = ow;
}

// emit: one wavefront per chain chunk, tab[b] = {entry, exit_w, nf0, cnt_w, owner, n_par,
// last, cs0}: the window prefix [entry, exit_w) by the group walk, then n_par staged
// frames in parallel (lane i: frame i, i + 64, ...), then the group walk from the next
// frame to the chunk's exit (or, last, to the stream's end: tail, count, result).
// owner == ~0: the whole rest from entry by the group walk (a chain ending in the window).
__global__ __launch_bounds__(64) void ws_rw_emit_kernel(const unsigned char* __restrict__ buf, u64 len, u32 max_frames,
                                                        const u64* __restrict__ tab, const RwOwn* __restrict__ own,
                                                        const u32* __restrict__ stg, u32 stgn,
                                                        WebsocketFrameDesc_t* __restrict__ desc,
                                                        u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                                        u32* __restrict__ nwork, WebsocketSegResult_t* __restrict__ res,
                                                        RwPlan* __restrict__ plan, int part) {
    u64 row = blockIdx.x, obase = 0, sbase = 0;
    if (plan) {                                                              // rows written by the linker
        if (!plan->active || blockIdx.x >= plan->nrows[part] || (part >= 1 && plan->in_state[part] != 1)) return;
        const RwPart& pt = plan->pt[part];
        stgn = pt.stgn;
        row += pt.cbase;                                                     // the part's rows start at its first chunk
        obase = (u64)pt.cbase * RW_D;
        sbase = pt.stg_base;
    }
    const u64* t = tab + 8 * row;
    const u64 ent = t[0], exit_w = t[1], nf0 = t[2], cnt_w = t[3], oi = t[4], n_par = t[5], cs0 = t[7];
    const bool last = t[6] != 0;
    const u32 lane = threadIdx.x;
    // the row that ends the walk also writes the count K2's launches from this part on read
    auto note_end = [&](const SwOut& o) {
        if (plan && last && lane == 0) rw_end_counts(plan, part, o.cnt);
    };
    if (oi == ~0ull) {
        const SwOut o = stream_walk(buf, len, ent, 0, (u32)nf0, len, true, max_frames, desc, items, ptr, pend, nwork,
                                    res, lane, nullptr, plan != nullptr);
        rw_note_max(plan, o.maxlen, lane);
        note_end(o);
        return;
    }
    const SwOut o1 = stream_walk(buf, len, ent, 0, (u32)nf0, exit_w, false, max_frames, desc, items, ptr, pend, nwork,
                                 res, lane, nullptr, plan != nullptr);
    u32 mx = o1.maxlen;
    const RwOwn ow = own[oi];
    const u32* sl = stg + sbase + (oi - obase) * stgn;
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    const uintptr_t origin = reinterpret_cast<uintptr_t>(buf);
    for (u64 i = lane; i < n_par; i += 64) {
        const u64 pos = cs0 + sl[i];
        const uintptr_t pa = origin + pos;
        const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
        u64 h0, h1;
        ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
        const WsHdr h = ws_parse(h0, h1, len - pos);                         // a frame (the owner walked it)
        if ((u32)h.ret > mx) mx = (u32)h.ret;
        const u64 slot = nf0 + cnt_w + i;
        const u64 fo = lead0 + pos, p0 = fo + h.hdr, fe = p0 + h.plen;
        const u64 w0 = p0 | ((u64)(rotl32(h.key, 8u * (u32)(p0 & 3)) & 0xFFFFu) << 48);
        const u64 w1 = (h.masked ? fe : p0) | ((u64)(rotl32(h.key, 8u * (u32)(p0 & 3)) >> 16) << 48);
        u32x4 it;
        it.x = (u32)w0; it.y = (u32)(w0 >> 32); it.z = (u32)w1; it.w = (u32)(w1 >> 32);
        *gptr<u32x4>(items + slot) = it;
        for (u64 p = (fo + (1ull << PIECE_SHIFT_S) - 1) >> PIECE_SHIFT_S; (p << PIECE_SHIFT_S) < fe && p < pend; ++p)
            *gptr<u64>(ptr + p) = slot;
        ws_store_desc(desc + slot, pos, h);
    }
    const u64 nb = ow.cs & 0x7FFFFFFFu;
    const u64 staged = nb < stgn ? nb : stgn;
    const u64 next = n_par < staged ? cs0 + sl[n_par] : (n_par == nb ? ow.exit : ow.over);
    const SwOut o2 = stream_walk(buf, len, next, 0, (u32)(nf0 + cnt_w + n_par), last ? len : ow.exit, last, max_frames,
                                 desc, items, ptr, pend, nwork, res, lane, nullptr, plan != nullptr);
    rw_note_max(plan, o2.maxlen > mx ? o2.maxlen : mx, lane);
    note_end(o2);
}

// ---- the chunk-parallel walk inside a captured call (no host reads): the plan kernel
// walks the sample and picks the geometry, R1-R3 read it, the linker follows the records
// on the device (the host loop of rw_walk, one wavefront), the emit writes the chain.
#define RW_CAP_CHUNKS 32768u   // a captured call's chunk-count cap (the smallest chunk follows)
#define RW_CAP_STGN 1024u      // ... and staging per owner

__global__ __launch_bounds__(64) void ws_rw_plan_kernel(const unsigned char* __restrict__ buf, u64 len, u32 max_frames,
                                                        SdState* __restrict__ sd, RwPlan* __restrict__ plan,
                                                        u64 cmin, u64 cmax, u32 nchunks_cap, u64 cand_cap, u64 stg_cap,
                                                        WebsocketFrameDesc_t* __restrict__ desc,
                                                        u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                                        u32* __restrict__ nwork, WebsocketSegResult_t* __restrict__ res,
                                                        int fresh, u64* __restrict__ seg, u32* __restrict__ disorder,
                                                        SdMirror* __restrict__ mirror, u64 split_x0, u64 split_x1,
                                                        u32 c0_shift, u32 c1_shift) {
    const u32 lane = threadIdx.x;
    // the previous device walk's longest frame: 0 before the first (the plan lies in the WS_AUX_ZERO range,
    // zeroed when the aux buffer is allocated or a capture adopts the slot; the host-linked walk's
    // scratch starts after it, rw_scratch)
    const u32 seen = plan->seen_max;
    // fresh 2 (captured calls): the previous replay's hint decides, as the passes saw it
    const int dev = fresh == 2;
    if (dev) fresh = sd->walk_hint != 0;
    // the walk is finished before any part: K2's first launch reads the final count
    auto finished = [&](u32 cnt) {
        if (lane == 0) {
            plan->active = 0;
            rw_end_counts(plan, 0, cnt);
            rw_end_states(plan, -1);
        }
    };
    if (!fresh && sd->phase == SD_DONE) {                                    // the passes finished it
        finished(nwork[0]);
        return;
    }
    // fresh: no pass rounds ran (the previous chunk walk on this stream saw lengths that keep
    // changing): the walk starts at (0, 0), and this kernel does the first round's chores — the
    // unmask's segment pair and gate word, and the pieces before the first frame
    const u64 P = fresh ? 0 : sd->P;
    const u32 nf = fresh ? 0 : sd->nf;
    if (fresh && lane == 0) {
        seg[0] = 0;
        seg[1] = len;
        *disorder = 0;
        if (reinterpret_cast<uintptr_t>(buf) & 15) ptr[0] = 0;               // piece 0 starts before the frame
    }
    // the sample (a walk that ends in it finishes the stream: `out` given)
    const u64 send = len - P > RW_SAMPLE ? P + RW_SAMPLE : len;
    const SwOut o = stream_walk(buf, len, P, fresh ? 0 : sd->g, nf, send, false, max_frames, desc, items, ptr, pend,
                                nwork, res, lane, plan->sample_out, true);
    // the next call on this stream skips the pass rounds unless the sample looks like runs of
    // equal lengths (>= 3 frames and >= 4 per header round, the round that met the sample's end
    // not counted) or the stream ended in it
    if (lane == 0) {
        const u64 fr = o.nf - nf, st = o.steps > 1 ? o.steps - 1 : 1;
        const u32 hint = !o.ended && !(fr >= 3 && fr >= 4 * st) ? 1u : 0u;
        if (mirror) __hip_atomic_store(&mirror->walk_hint, hint, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (dev) sd->walk_hint = hint;                                       // read by the next replay
    }
    if (o.ended) {
        finished(o.cnt);
        return;
    }
    const u64 P1 = o.next;
    const u64 mean = o.nf > nf ? (P1 - P) / (o.nf - nf) : (P1 - P);
    if ((len - P1) / (mean ? mean : 1) < RW_MIN_FRAMES) {                   // a short rest: this wavefront
        const SwOut o3 = stream_walk(buf, len, P1, 0, o.nf, len, true, max_frames, desc, items, ptr, pend, nwork, res,
                                     lane);
        finished(o3.cnt);
        return;
    }
    const u32 seenm = o.maxlen > seen ? o.maxlen : seen;
    u64 C = rw_pow2_clamp(mean * 1024, cmin > RW_CMIN ? cmin : RW_CMIN, cmin > cmax ? cmin : cmax);
    // split (split_x0 / split_x1: the first bytes K2's second / third launch own; 0 = none): part k
    // ends at the first chunk start at or past split_x_k; part 0's chunks are C >> c0_shift, a middle
    // part's C >> c1_shift (at least twice the window a frame start needs), the last part's C
    const u64 hneed = rw_window(mean, seenm, 4 * (u64)RW_HMAX);
    const u64 xs[RW_NP - 1] = {split_x0, split_x1};
    const u32 shifts[RW_NP - 1] = {c0_shift, c1_shift};
    u64 Pk[RW_NP], Ck[RW_NP], nk[RW_NP];
    u32 np = 1;
    for (;;) {
        u64 B = P1, tot = 0;
        np = 0;
        for (u32 k = 0; k < RW_NP; ++k) {
            const bool lastp = k + 1 == RW_NP || !xs[k] || xs[k] >= len;
            u64 Cx = C;
            if (!lastp) {
                const u64 want = (C >> shifts[k]) > 2 * hneed ? (C >> shifts[k]) : 2 * hneed;
                Cx = rw_pow2_clamp(want, RW_CMIN, C);
            }
            u64 E = len;
            if (!lastp) {
                E = xs[k] > B ? B + (xs[k] - B + Cx - 1) / Cx * Cx : B;
                if (E >= len) E = len;
            }
            Pk[k] = B; Ck[k] = Cx; nk[k] = E > B ? (E - B + Cx - 1) / Cx : 0;
            tot += nk[k];
            ++np;
            B = E;
            if (lastp || E >= len) break;
        }
        // fit the caps (cmin makes the chunk count fit; the smallest staging and candidate lists too)
        if (tot <= nchunks_cap && tot * RW_D * 64 <= stg_cap && tot * 64 <= cand_cap) break;
        C <<= 1;
    }
    u64 Hk[RW_NP], stgk[RW_NP], capk[RW_NP];
    u64 stg_need = 0, cand_need = 0;
    for (u32 k = 0; k < np; ++k) {
        Hk[k] = rw_window(mean, seenm, Ck[k]);
        stgk[k] = rw_pow2_clamp(2 * Ck[k] / (mean ? mean : 1), 256, RW_CAP_STGN);
        capk[k] = Hk[k] / 32;
    }
    for (;;) {                                                               // shrink staging / candidates to the caps
        stg_need = cand_need = 0;
        bool can = false;
        for (u32 k = 0; k < np; ++k) {
            stg_need += nk[k] * RW_D * stgk[k];
            cand_need += nk[k] * capk[k];
            can = can || stgk[k] > 64 || capk[k] > 64;
        }
        if ((stg_need <= stg_cap && cand_need <= cand_cap) || !can) break;
        for (u32 k = 0; k < np; ++k) {
            if (stg_need > stg_cap && stgk[k] > 64) stgk[k] >>= 1;
            if (cand_need > cand_cap && capk[k] > 64) capk[k] >>= 1;
        }
    }
    if (lane == 0) {
        u64 cb = 0, sb = 0, cdb = 0;
        for (u32 k = 0; k < RW_NP; ++k) {
            RwPart& t = plan->pt[k];
            if (k < np) {
                t.P = Pk[k]; t.C = Ck[k]; t.H = (u32)Hk[k]; t.n = (u32)nk[k]; t.cbase = (u32)cb; t.capc = (u32)capk[k];
                t.stgn = (u32)stgk[k]; t.stg_base = sb; t.cand_base = cdb;
                cb += nk[k]; sb += nk[k] * RW_D * stgk[k]; cdb += nk[k] * capk[k];
            } else {
                t.P = len; t.C = C; t.H = RW_HMIN; t.n = 0; t.cbase = (u32)cb; t.capc = 64; t.stgn = 64;
                t.stg_base = sb; t.cand_base = cdb;
            }
            plan->nrows[k] = 0;
            plan->linked[k] = 0;
            plan->in_ent[k] = 0;
            plan->in_nf[k] = 0;
            plan->in_state[k] = 0;
            plan->nw[k] = 0;
        }
        plan->nchunks = (u32)cb;
        plan->nparts = np;
        plan->need_mask = (buf[P1 + 1] & 0x80u) ? 1u : 0u;                   // client frames: masked
        plan->nf = o.nf;
        plan->seen_max = 0;                 // this call's emit and linker fill it in
        plan->active = 1;
        rw_end_states(plan, (int)np - 1);   // parts past the last one are no-ops
    }
}

// ---- The captured call's linker, chunk-parallel (the common case; ws_rw_link_kernel below
// stays as the exact serial fallback). The chain's entry into chunk c is the exit of chunk
// c-1's owner walk on the chain; wrong starts inside a window either die (an implausible
// header: owner dead) or merge with the chain, so the live owners of a chunk nearly always
// agree on ONE exit, and then the entry into chunk c is known without the chain before it.
// ws_rw_plink_kernel (one wavefront per chunk): entry = that common exit (chunk 0: the
// plan's P), its record, its owner; ws_rw_pscan_kernel (one block): the frame counts'
// prefix sum up to the first chunk that ends the walk, and the emit rows exactly as the
// serial linker writes them. Anything else — live owners that disagree, an entry outside
// its window or without a record or owner, a frame spanning a whole chunk, max_frames
// reached before the chain's last chunk, no chunk ending the walk — leaves nrows at 0 and
// the serial linker runs.
struct RwLink {
    u64 ent, rexit;
    u32 cnt_w, nb, oi, flags;       // flags: 1 valid, 2 the walk ends in the window, 4 the chain ends here
};

__global__ __launch_bounds__(64) void ws_rw_plink_kernel(u64 len, const RwPlan* __restrict__ plan,
                                                         const RwRec* __restrict__ recs, const u32* __restrict__ nrec,
                                                         const unsigned long long* __restrict__ dx,
                                                         const RwOwn* __restrict__ own, RwLink* __restrict__ lk,
                                                         int part) {
    const u32 lane = threadIdx.x, cl = blockIdx.x;                           // local chunk
    if (!plan->active || cl >= plan->pt[part].n || (part >= 1 && plan->in_state[part] != 1)) return;
    const RwPart& pt = plan->pt[part];
    const u64 P = pt.P, C = pt.C;
    const u32 H = pt.H, nchunks = plan->nchunks;
    const u64 c = (u64)pt.cbase + cl;                                        // global chunk
    const u64 cs0 = P + (u64)cl * C;
    const bool lastc = c + 1 == nchunks;
    // the next chunk's size (a part's last chunk: the next part's first)
    const u64 Cn = (cl + 1 == pt.n && part + 1 < (int)plan->nparts) ? plan->pt[part + 1].C : C;
    auto rl64 = [](u64 v, int i) -> u64 {
        return (u64)(u32)__builtin_amdgcn_readlane((int)(u32)v, i) |
               ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), i) << 32);
    };
    // the entry: the common exit of chunk c-1's live owners; a part's first chunk: the part's
    // origin (part 0) or the previous part's hand-off (the chain's exact entry)
    u64 ent = part == 0 ? P : plan->in_ent[part];
    bool ok = true;
    if (cl) {
        const u64 oi = (c - 1) * RW_D + (lane & (RW_D - 1));
        const u64 d = dx[oi];
        const RwOwn o = own[oi];
        const bool live = lane < RW_D && d != 0 && !o.dead;
        const u64 m = __ballot(live);
        if (!m) {
            ok = false;
        } else {
            ent = rl64(o.exit, __builtin_ctzll(m));
            ok = __ballot(live && o.exit != ent) == 0;
        }
    }
    ok = ok && ent >= cs0 && ent - cs0 < H && (lastc || ent - cs0 < C);
    RwLink L = {ent, 0, 0, 0, 0, 0};
    if (ok) {
        const u32 so = (u32)(ent - cs0);
        const u32 n0 = nrec[4 * c], n1 = nrec[4 * c + 1];
        const u32 na = n0 < RW_S0 ? n0 : RW_S0;
        const RwRec q = recs[c * RW_SLOTS + (lane < RW_S0 ? lane : 0)];
        u64 m = __ballot(lane < na && q.start == so);
        u32 rcs = 0;
        u64 rexit = 0;
        bool found = false;
        if (m) {
            const int i = __builtin_ctzll(m);
            rcs = (u32)__builtin_amdgcn_readlane((int)q.cs, i);
            rexit = rl64(q.exit, i);
            found = true;
        } else {                                                             // walks that end the stream
            const RwRec* r1 = lastc ? recs + (u64)nchunks * RW_SLOTS : recs + c * RW_SLOTS + RW_S0;
            const u32 nb1 = lastc ? (n1 < RW_SLAST ? n1 : RW_SLAST) : (n1 < RW_S1 ? n1 : RW_S1);
            for (u32 k0 = 0; k0 < nb1 && !found; k0 += 64) {
                RwRec q1 = {};
                if (k0 + lane < nb1) q1 = r1[k0 + lane];
                const u64 m1 = __ballot(k0 + lane < nb1 && q1.start == so);
                if (m1) {
                    const int i = __builtin_ctzll(m1);
                    rcs = (u32)__builtin_amdgcn_readlane((int)q1.cs, i);
                    rexit = rl64(q1.exit, i);
                    found = true;
                }
            }
        }
        if (found) {
            L.cnt_w = rcs & 0x7FFFFFFFu;
            L.rexit = rexit;
            if (rcs >> 31) {
                L.flags = 1 | 2 | 4;                                         // the walk ends in the window
            } else {
                const u64 oi = c * RW_D + (lane & (RW_D - 1));
                const u64 d = dx[oi];
                const RwOwn o = own[oi];
                const u64 mo = __ballot(lane < RW_D && d == rexit);
                if (mo) {
                    const int i = __builtin_ctzll(mo);
                    const u32 dead = (u32)__builtin_amdgcn_readlane((int)o.dead, i);
                    const u32 ocs = (u32)__builtin_amdgcn_readlane((int)o.cs, i);
                    const u64 oexit = rl64(o.exit, i);
                    const bool ends = (ocs >> 31) != 0 || oexit >= len;
                    if (!dead && (ends || (oexit >= cs0 + C && oexit - (cs0 + C) < Cn && !lastc))) {
                        L.nb = ocs & 0x7FFFFFFFu;
                        L.oi = (u32)(c * RW_D + (u64)i);
                        L.flags = 1 | (ends ? 4 : 0);
                    }
                }
            }
        }
    }
    if (lane == 0) lk[c] = L;
}

// one block of RW_PS_T threads: the prefix sum of the chain's frame counts and the emit rows
#define RW_PS_T 1024
__global__ __launch_bounds__(RW_PS_T) void ws_rw_pscan_kernel(u32 max_frames, RwPlan* __restrict__ plan,
                                                             const RwLink* __restrict__ lk, u64* __restrict__ tab,
                                                             const RwOwn* __restrict__ own, int part) {
    __shared__ u32 s_stop;
    __shared__ u32 s_bad;
    __shared__ u64 s_wsum[RW_PS_T / 64];
    __shared__ u64 s_carry;
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (!plan->active || (part >= 1 && plan->in_state[part] != 1)) return;
    const RwPart& pt = plan->pt[part];
    const u32 n = pt.n, cb = pt.cbase, stgn = pt.stgn;
    // a part of a split hands the chain over to the next part when no chunk of it ends the walk
    const bool has_next = part + 1 < (int)plan->nparts;
    if (tid == 0) { s_stop = n; s_bad = 0; s_carry = part == 0 ? plan->nf : plan->in_nf[part]; }
    __syncthreads();
    // the first chunk that is invalid or ends the chain
    for (u32 c = tid; c < n; c += RW_PS_T) {
        const u32 f = lk[cb + c].flags;
        if (!(f & 1) || (f & 4)) atomicMin(&s_stop, c);
    }
    __syncthreads();
    const u32 stop = s_stop;
    if (stop >= n ? !has_next : !(lk[cb + stop].flags & 1)) return;         // the serial linker runs
    // frame counts of chunks [0, stop): nfc before each, max_frames never reached on the way
    for (u32 t0 = 0; t0 <= stop; t0 += RW_PS_T) {
        const u32 c = t0 + tid;
        RwLink L = {};
        if (c <= stop && c < n) L = lk[cb + c];
        const u64 cnt = c < stop ? (u64)L.cnt_w + L.nb : 0;
        u64 x = cnt;                                                         // inclusive wave scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u64 y = (u64)__shfl_up((long long)x, d);
            if (lane >= (u32)d) x += y;
        }
        if (lane == 63) s_wsum[wv] = x;
        __syncthreads();
        u64 before = s_carry;
        for (u32 w = 0; w < wv; ++w) before += s_wsum[w];
        const u64 nfc = before + x - cnt;
        const u64 cs0 = pt.P + (u64)c * pt.C;
        if (c < stop) {
            if (nfc + cnt >= max_frames) s_bad = 1;                         // max_frames mid-chain: serial
            u64* t = tab + 8 * ((u64)cb + c);
            const u64 n_par = L.nb < stgn ? L.nb : stgn;
            t[0] = L.ent; t[1] = L.rexit; t[2] = nfc; t[3] = L.cnt_w; t[4] = L.oi; t[5] = n_par; t[6] = 0;
            t[7] = cs0;
        } else if (c == stop && stop < n) {
            u64* t = tab + 8 * ((u64)cb + c);
            if ((L.flags & 2) || nfc + L.cnt_w >= max_frames) {             // ends in the window: group walk
                t[0] = L.ent; t[1] = 0; t[2] = nfc; t[3] = 0; t[4] = ~0ull; t[5] = 0; t[6] = 1; t[7] = cs0;
            } else {
                u64 n_par = L.nb < stgn ? L.nb : stgn;
                if (nfc + L.cnt_w + n_par > max_frames) n_par = max_frames - nfc - L.cnt_w;
                t[0] = L.ent; t[1] = L.rexit; t[2] = nfc; t[3] = L.cnt_w; t[4] = L.oi; t[5] = n_par; t[6] = 1;
                t[7] = cs0;
            }
        }
        __syncthreads();
        if (tid == RW_PS_T - 1) s_carry = before + x;
        __syncthreads();
    }
    if (tid == 0 && !s_bad) {
        if (stop < n) {                                                      // the walk ends in this part
            plan->nrows[part] = stop + 1;
            rw_end_states(plan, part);                                       // (counts: the last row's emit)
        } else {                                                             // this part hands over
            plan->nrows[part] = n;
            // (an empty part passes its own entry on: the plan's P for part 0, the hand-off into it else)
            rw_hand_over(plan, part, n ? own[lk[cb + n - 1].oi].exit : (part == 0 ? pt.P : plan->in_ent[part]),
                         (u32)s_carry);
        }
        plan->linked[part] = 1;
    }
}


// The linker: from the plan's entry, chunk by chunk, the record whose start is the entry
// (A records, then the walks that end the stream), its window exit's owner walk, one
// emit row per chunk; a chunk without a usable record is walked here by this wavefront
// (stream_walk writes its frames; a walk that ends the stream finishes it). Bounded by
// the chunk count (every step moves the entry forward).
__global__ __launch_bounds__(64) void ws_rw_link_kernel(const unsigned char* __restrict__ buf, u64 len, u32 max_frames,
                                                        RwPlan* __restrict__ plan, const RwRec* __restrict__ recs,
                                                        const u32* __restrict__ nrec,
                                                        const unsigned long long* __restrict__ dx,
                                                        const RwOwn* __restrict__ own, u64* __restrict__ tab,
                                                        WebsocketFrameDesc_t* __restrict__ desc,
                                                        u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                                        u32* __restrict__ nwork, WebsocketSegResult_t* __restrict__ res,
                                                        int part) {
    const u32 lane = threadIdx.x;
    if (!plan->active || plan->linked[part] || (part >= 1 && plan->in_state[part] != 1)) return;   // linked by pscan
    const RwPart& pt = plan->pt[part];
    const u64 P = pt.P, C = pt.C;
    const u32 H = pt.H, nchunks = plan->nchunks, stgn = pt.stgn, np = pt.n, cb = pt.cbase;
    // a part of a split stops where the next part begins and hands the chain over
    const bool has_next = part + 1 < (int)plan->nparts;
    const u64 Pb = has_next ? plan->pt[part + 1].P : len;
    u64 ent = part == 0 ? P : plan->in_ent[part];
    u32 nfc = part == 0 ? plan->nf : plan->in_nf[part], rows = 0;
    bool last = false;
    u32 cnt_end = 0;                                                         // the count a finishing walk wrote
    bool ended_walk = false;
    auto row = [&](u64 a0, u64 a1, u64 a2, u64 a3, u64 a4, u64 a5, u64 a6, u64 a7) {
        if (lane == 0) {
            u64* t = tab + 8 * ((u64)cb + rows);
            t[0] = a0; t[1] = a1; t[2] = a2; t[3] = a3; t[4] = a4; t[5] = a5; t[6] = a6; t[7] = a7;
        }
        ++rows;
    };
    // The records of RW_LK consecutive chunks are loaded in one round (the chain almost always
    // moves to the next chunk), then taken one chunk at a time; a chain that leaves that run
    // (a skipped chunk, a chunk walked here) reloads at its new chunk.
    constexpr u32 RW_LK = 8;
    u32 steps = 0, mx = 0;
    while (!last && ent < len && steps <= np + 1 && !(has_next && ent >= Pb)) {
        const u64 c0 = (ent - P) / C;                                        // local chunk
        // lane l < RW_LK: the record counts of chunk c0 + l (read back per chunk by readlane)
        u32 n0v = 0, n1v = 0;
        {
            const u64 cl = c0 + (lane < RW_LK ? lane : 0);
            const u64 cc = cb + (cl < np ? cl : (np ? np - 1 : 0));
            n0v = nrec[4 * cc];
            n1v = nrec[4 * cc + 1];
        }
        RwRec q[RW_LK];
        unsigned long long dd[RW_LK];
        RwOwn oo[RW_LK];
#pragma unroll
        for (u32 k = 0; k < RW_LK; ++k) {                                   // clamped: in-range loads
            const u64 cc = cb + (c0 + k < np ? c0 + k : (np ? np - 1 : 0));
            q[k] = recs[cc * RW_SLOTS + (lane < RW_S0 ? lane : 0)];
            dd[k] = dx[cc * RW_D + (lane & (RW_D - 1))];
            oo[k] = own[cc * RW_D + (lane & (RW_D - 1))];
        }
        bool reload = false;
#pragma unroll
        for (u32 k = 0; k < RW_LK; ++k) {
            if (reload || last || ent >= len || (has_next && ent >= Pb)) break;
            const u64 c = (ent - P) / C, cs0 = P + c * C;                    // local chunk
            if (c != c0 + k) break;                                          // left the run: reload
            ++steps;
            bool found = false;
            RwRec r = {};
            const u64 gcx = (u64)cb + c;                                     // global chunk
            if (c < np && ent - cs0 < H) {
                const u32 so = (u32)(ent - cs0);
                const bool lastc = gcx + 1 == nchunks;
                const u32 n0k = (u32)__builtin_amdgcn_readlane((int)n0v, (int)k);
                const u32 n1k = (u32)__builtin_amdgcn_readlane((int)n1v, (int)k);
                const u32 na = n0k < RW_S0 ? n0k : RW_S0;
                const u64 m = __ballot(lane < na && q[k].start == so);
                if (m) {
                    const int i = __builtin_ctzll(m);
                    r.start = so;
                    r.cs = (u32)__builtin_amdgcn_readlane((int)q[k].cs, i);
                    r.exit = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)q[k].exit, i)) |
                             ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(q[k].exit >> 32), i) << 32);
                    found = true;
                } else {                                                     // walks that end the stream
                    const RwRec* r1 = lastc ? recs + (u64)nchunks * RW_SLOTS : recs + gcx * RW_SLOTS + RW_S0;
                    const u32 nb1 = lastc ? (n1k < RW_SLAST ? n1k : RW_SLAST) : (n1k < RW_S1 ? n1k : RW_S1);
                    for (u32 k0 = 0; k0 < nb1 && !found; k0 += 64) {
                        RwRec q1 = {};
                        if (k0 + lane < nb1) q1 = r1[k0 + lane];
                        const u64 m1 = __ballot(k0 + lane < nb1 && q1.start == so);
                        if (m1) {
                            const int i = __builtin_ctzll(m1);
                            r.start = so;
                            r.cs = (u32)__builtin_amdgcn_readlane((int)q1.cs, i);
                            r.exit = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)q1.exit, i)) |
                                     ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(q1.exit >> 32), i) << 32);
                            found = true;
                        }
                    }
                }
            }
            const u32 cnt_w = found ? (r.cs & 0x7FFFFFFFu) : 0u;
            if (found && ((r.cs >> 31) || (u64)nfc + cnt_w >= max_frames)) { // ends in the window: group walk
                row(ent, 0, nfc, 0, ~0ull, 0, 1, cs0);
                last = true;
                break;
            }
            if (found) {
                // the owner walk of this exit (at most RW_D distinct exits per chunk)
                const u64 mo = __ballot(lane < RW_D && dd[k] == r.exit);
                if (mo) {
                    const int i = __builtin_ctzll(mo);
                    const u32 dead = (u32)__builtin_amdgcn_readlane((int)oo[k].dead, i);
                    if (!dead) {
                        const u32 ocs = (u32)__builtin_amdgcn_readlane((int)oo[k].cs, i);
                        const u64 oexit = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)oo[k].exit, i)) |
                                          ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(oo[k].exit >> 32), i) << 32);
                        const u32 nb = ocs & 0x7FFFFFFFu;
                        last = (ocs >> 31) != 0 || oexit >= len || (u64)nfc + cnt_w + nb >= max_frames;
                        u64 n_par = nb < stgn ? nb : stgn;
                        if (last && (u64)nfc + cnt_w + n_par > max_frames) n_par = max_frames - nfc - cnt_w;
                        row(ent, r.exit, nfc, cnt_w, gcx * RW_D + (u64)i, n_par, last ? 1ull : 0ull, cs0);
                        nfc += cnt_w + nb;
                        ent = oexit;
                        continue;
                    }
                }
            }
            // no usable record: this wavefront walks the chunk (writing its frames)
            const SwOut o = stream_walk(buf, len, ent, 0, nfc, cs0 + C < len ? cs0 + C : len, false, max_frames, desc,
                                        items, ptr, pend, nwork, res, lane, plan->sample_out, true);
            if (o.maxlen > mx) mx = o.maxlen;
            if (o.ended) { last = true; ended_walk = true; cnt_end = o.cnt; break; }   // (it finished the stream)
            if (o.next <= ent) { steps = np + 2; break; }                    // (cannot happen: no progress)
            ent = o.next;
            nfc = o.nf;
            reload = true;                                                   // its frames may cross chunks
        }
    }
    const bool handoff = !last && has_next && ent >= Pb && ent < len;
    if (!last && !handoff) {                                                 // safety: walk whatever is left
        const SwOut o = stream_walk(buf, len, ent, 0, nfc, len, true, max_frames, desc, items, ptr, pend, nwork, res,
                                    lane, nullptr, true);
        if (o.maxlen > mx) mx = o.maxlen;
        ended_walk = true;
        cnt_end = o.cnt;
    }
    rw_note_max(plan, mx, lane);
    if (lane == 0) {
        plan->nrows[part] = rows;
        if (handoff) {
            rw_hand_over(plan, part, ent, nfc);
        } else {
            rw_end_states(plan, part);
            if (ended_walk) rw_end_counts(plan, part, cnt_end);              // (else: the last row's emit writes them)
        }
        plan->linked[part] = 1;
    }
}

WsOpt ws_stream_rw{1};          // "stream_rw": chunk-parallel walk for long streams, linked on the device
                                // (1) or by the host (2, eager calls), 0 one wavefront
WsOpt ws_stream_rw_cmax{22};    // "stream_rw_cmax": log2 of the largest chunk (cfg3: 4 MiB 8.11-8.13 ms
                                // against 8.19-8.21 at 8 MiB and 8.14-8.15 at 2 MiB, profiles/r04_stream_cmax_ab.log)
WsOpt ws_stream_rounds{4};      // "stream_rounds": pass rounds (A + B) enqueued per state read
WsOpt ws_stream_plink{1};       // "stream_plink": captured calls link the chunk records in parallel (0: serial only)
WsOpt ws_stream_split{8};       // "stream_split": eager device-planned walks: K2's first launch takes this many 256ths
                                // of the pieces, the walk past them runs beside it on a side stream (0: no split)
WsOpt ws_stream_split_wait{0};  // "stream_split_wait": part 1's walk starts after the plan (0), part 0's owner
                                // walks (1) or part 0's emit (2)
WsOpt ws_stream_side_prio{0};   // "stream_side_prio": the split walk's side stream priority: 0 default, 1 least, 2 greatest
                                // (a stream of the least priority measured 7.82-7.85 ms against 7.91 on a fresh process,
                                // but 8.24 against 7.61 after the host path's three pipeline streams: its walk then waited
                                // for the first unmask launch; the greatest 10.14 — profiles/r06_stream_side_prio.log)
WsOpt ws_stream_split2{48};     // "stream_split2": a third part — K2's second launch ends at this many 256ths of the
                                // pieces (> stream_split; 0: two parts). Three parts 8 / 48 with part 0 in chunks of
                                // C / 8 and the middle in C / 4: 7.53-7.56 ms against 7.57-7.59 for two parts 24 in
                                // C / 4 (cfg3, profiles/r06_stream_split_ab.log)
WsOpt ws_stream_split_capture{1};   // "stream_split_capture": split captured calls too (their side stream
                                    // becomes a graph branch, run beside the unmask: cfg3 replays 7.60 ms
                                    // against 7.84 unsplit, profiles/r06_stream_split_ab.log ab_gcap)
WsOpt ws_stream_win{2};         // "stream_win": log2 of the piece windows of a raw-stream call's unmask launches
                                // (-1: the batch rule); four windows: cfg3 7.41 against 7.54 ms with two
                                // (profiles/r06_stream_win_ab.log)
WsOpt ws_stream_c1{2};          // "stream_c1": a middle part's chunks are the last part's chunk >> this
WsOpt ws_stream_c0{3};          // "stream_c0": part 0's chunks are the usual chunk >> this (at least twice its window)
std::atomic<unsigned long long> ws_stat_rw_chunks{0};       // chunks written from records (last call)
std::atomic<unsigned long long> ws_stat_stream_skips{0};    // eager calls that skipped the pass rounds (since load)
std::atomic<unsigned long long> ws_stat_rw_chunk_walks{0};  // chunks walked by one wavefront without a record

// scratch for the chunk-parallel walk: the call's slot's auxiliary workspace (device
// records + counters, and a pinned host copy of them), so concurrent calls on different
// streams never share it (the walk runs in eager calls only)
struct RwScratch {
    void* d = nullptr;
    void* h = nullptr;
};

// (the aux head holds the pass loop's state and the 256 B after it the device walk's plan,
// RwPlan: the host-linked walk's device scratch starts after both, so a slot that serves both
// kinds of call never hands the plan this walk's leftovers — ADVICE r05)
static int rw_scratch(WsSlot& slot, size_t dbytes, size_t hbytes, RwScratch* out) {
    WsAux A;
    const int rc = slot.aux(WS_AUX_ZERO + dbytes, WS_AUX_HEAD + hbytes, &A);
    if (rc) return rc;
    out->d = reinterpret_cast<unsigned char*>(A.d) + WS_AUX_ZERO;
    out->h = reinterpret_cast<unsigned char*>(A.h) + WS_AUX_HEAD;
    return 0;
}


// The chunk-parallel walk of [P, len) with nf frames before P (see above). Launches the
// emit kernels and, for chunks without a link, one-wavefront chunk walks; the last of
// them writes the tail pointers, item count and segment result.
static int rw_walk(WsSlot& slot, unsigned char* d_buf, u64 len, u64 P, u32 nf, u32 max_frames,
                   WebsocketFrameDesc_t* d_desc, const PieceWs& Pw, WebsocketSegResult_t* d_res, hipStream_t st) {
    hipError_t e;
    int rc;
    ws_stat_rw_chunk_walks = 0;
    ws_stat_rw_chunks = 0;
    RwScratch S;
    u64* wout = nullptr;       // chunk-walk report (device) and its pinned copy
    u64* ho = nullptr;
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
    if ((rc = rw_scratch(slot, 256, 256, &S))) return rc;
    wout = reinterpret_cast<u64*>(S.d);
    ho = reinterpret_cast<u64*>(S.h);
    u64 P1 = 0;
    u32 nf1 = 0;
    if ((rc = chunk_walk(P, nf, P + RW_SAMPLE, P1, nf1))) return rc < 0 ? rc : 0;
    ws_stat_rw_chunk_walks = 0;                                              // not counting the sample
    const u64 mean = nf1 > nf ? (P1 - P) / (nf1 - nf) : (P1 - P);
    P = P1;
    nf = nf1;
    if ((len - P) / (mean ? mean : 1) < RW_MIN_FRAMES) {                    // a short rest: one wavefront
        hipLaunchKernelGGL(ws_stream_walk_kernel, dim3(1), dim3(64), 0, st, d_buf, len, P, (u64)0, nf, max_frames,
                           d_desc, Pw.items, Pw.ptr, Pw.npieces, Pw.nwork, d_res);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_stream_walk_kernel launch", e);
        return 0;
    }
    const int cmax_log = ws_stream_rw_cmax;                                  // one read per call
    const u64 cmax = cmax_log >= 16 && cmax_log <= 26 ? 1ull << cmax_log : RW_CMAX;
    const u64 C = rw_pow2_clamp(mean * 1024, RW_CMIN, cmax);
    const u32 H = (u32)rw_pow2_clamp(mean * 8, RW_HMIN, C / 2 < RW_HMAX ? C / 2 : RW_HMAX);
    const u64 nchunks = (len - P + C - 1) / C;
    const size_t b_recs = ((size_t)(nchunks * RW_SLOTS + RW_SLAST) * sizeof(RwRec) + 255) & ~(size_t)255;
    const size_t b_nrec = ((size_t)nchunks * 16 + 255) & ~(size_t)255;     // per chunk: n0, n1, candidates
    const size_t b_dx = ((size_t)nchunks * RW_D * 8 + 255) & ~(size_t)255;
    const size_t b_own = ((size_t)nchunks * RW_D * sizeof(RwOwn) + 255) & ~(size_t)255;
    const size_t b_tab = ((size_t)nchunks * 64 + 255) & ~(size_t)255;
    // staging: about twice the chunk's mean frame count (frames past it are walked by the emit)
    const u32 stgn = (u32)rw_pow2_clamp(2 * C / (mean ? mean : 1), 256, RW_STG);
    const size_t b_stg = (size_t)nchunks * RW_D * stgn * 4;
    const u32 capc = H / 32;                                                 // candidates: 1/32 of a window
    const size_t b_cand = (size_t)nchunks * capc * 8;
    const size_t b_host = b_recs + b_nrec + b_dx + 256 + b_own;              // copied back
    if ((rc = rw_scratch(slot, 256 + b_host + b_tab + b_stg + b_cand, 256 + b_host, &S))) return rc;
    unsigned char* w = reinterpret_cast<unsigned char*>(S.d);
    unsigned char* hw = reinterpret_cast<unsigned char*>(S.h);
    wout = reinterpret_cast<u64*>(w);
    ho = reinterpret_cast<u64*>(hw);
    RwRec* recs = reinterpret_cast<RwRec*>(w + 256);
    u32* nrec = reinterpret_cast<u32*>(w + 256 + b_recs);
    unsigned long long* dx = reinterpret_cast<unsigned long long*>(w + 256 + b_recs + b_nrec);
    RwOwn* own = reinterpret_cast<RwOwn*>(w + 256 + b_recs + b_nrec + b_dx + 256);
    u64* tab = reinterpret_cast<u64*>(w + 256 + b_host);
    u32* stg = reinterpret_cast<u32*>(w + 256 + b_host + b_tab);
    u64* cand = reinterpret_cast<u64*>(w + 256 + b_host + b_tab + b_stg);
    const RwRec* hr = reinterpret_cast<const RwRec*>(hw + 256);
    const u32* hn = reinterpret_cast<const u32*>(hw + 256 + b_recs);
    const u64* hdx = reinterpret_cast<const u64*>(hw + 256 + b_recs + b_nrec);
    const RwOwn* hown = reinterpret_cast<const RwOwn*>(hw + 256 + b_recs + b_nrec + b_dx + 256);
    // the stream's frames are masked if the one at P is (client streams): candidates must be too
    unsigned char* hb = reinterpret_cast<unsigned char*>(ho + 4);
    hb[1] = 0;
    if ((e = hipMemcpyAsync(hb, d_buf + P, 2, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipMemsetAsync(nrec, 0, b_nrec + b_dx + 256, st)) != hipSuccess ||  // counters, claimed exits
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return ws_set_err("stream walk setup", e);
    const u32 need_mask = (hb[1] & 0x80u) ? 1u : 0u;
    const u64 threads = nchunks * (H / RW_TPOS);
    hipLaunchKernelGGL(ws_rw_cand_kernel, dim3((u32)((threads + 255) / 256)), dim3(256), 0, st, d_buf, len, P, C, H,
                       (u32)nchunks, need_mask, cand, nrec, capc, (const RwPlan*)nullptr, 0);
    if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_rw_cand_kernel launch", e);
    const u32 r2_blocks = (u32)std::min<u64>((nchunks * capc + 255) / 256, 4096);  // grid-stride
    hipLaunchKernelGGL(ws_rw_spec_kernel, dim3(r2_blocks), dim3(256), 0, st, d_buf, len, P, C, H, (u32)nchunks,
                       need_mask, cand, capc, recs, nrec, dx, (const RwPlan*)nullptr, 0);
    if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_rw_spec_kernel launch", e);
    hipLaunchKernelGGL(ws_rw_own_kernel, dim3((u32)((nchunks * RW_D + RW_OWN_T - 1) / RW_OWN_T)), dim3(RW_OWN_T), 0, st, d_buf, len, P,
                       C, (u32)nchunks, need_mask, dx, own, stg, stgn, (const RwPlan*)nullptr, 0);
    if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_rw_own_kernel launch", e);
    if ((e = hipMemcpyAsync(hw + 256, w + 256, b_host, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return ws_set_err("stream walk records", e);
    // follow the chain from P: exact, every record is the reference loop from its start
    std::vector<u64> ht;
    u64 ent = P;
    u32 nfc = nf;
    ht.reserve(nchunks * 8 + 8);
    for (bool last = false; !last;) {
        const u64 c = (ent - P) / C, cs0 = P + c * C;
        if (c + 3 < nchunks) {                                               // the chain is sequential:
            const u64 cp = c + 3;                                            // hide the host's cache misses
            __builtin_prefetch(hn + 4 * cp);
            for (u32 k = 0; k < 4; ++k) __builtin_prefetch(hr + cp * RW_SLOTS + 4 * k);
            __builtin_prefetch(hdx + cp * RW_D);
            __builtin_prefetch(hown + cp * RW_D);
            __builtin_prefetch(hown + cp * RW_D + 2);
        }
        const RwRec* r = nullptr;
        if (c < nchunks && ent - cs0 < H) {
            const u32 so = (u32)(ent - cs0);
            for (u32 k = 0; k < hn[4 * c] && k < RW_S0; ++k)
                if (hr[c * RW_SLOTS + k].start == so) { r = &hr[c * RW_SLOTS + k]; break; }
            const bool lastc = c + 1 == nchunks;
            const RwRec* r1 = lastc ? hr + nchunks * RW_SLOTS : hr + c * RW_SLOTS + RW_S0;
            for (u32 k = 0; !r && k < hn[4 * c + 1] && k < (lastc ? RW_SLAST : RW_S1); ++k)
                if (r1[k].start == so) { r = &r1[k]; break; }
        }
        const RwOwn* ow = nullptr;
        u64 oi = ~0ull;
        if (r && !(r->cs >> 31))
            for (u32 d = 0; d < RW_D; ++d)
                if (hdx[c * RW_D + d] == r->exit) {
                    oi = c * RW_D + d;
                    ow = hown[oi].dead ? nullptr : &hown[oi];
                    break;
                }
        const u32 cnt_w = r ? (r->cs & 0x7FFFFFFFu) : 0u;
        if (r && ((r->cs >> 31) || (u64)nfc + cnt_w >= max_frames)) {      // ends in the window: group walk
            const u64 row[8] = {ent, 0, nfc, 0, ~0ull, 0, 1, cs0};
            ht.insert(ht.end(), row, row + 8);
            break;
        }
        if (ow) {
            const u32 nb = ow->cs & 0x7FFFFFFFu;
            last = (ow->cs >> 31) != 0 || ow->exit >= len || (u64)nfc + cnt_w + nb >= max_frames;
            u64 n_par = nb < stgn ? nb : stgn;
            if (last && (u64)nfc + cnt_w + n_par > max_frames) n_par = max_frames - nfc - cnt_w;
            const u64 row[8] = {ent, r->exit, nfc, cnt_w, oi, n_par, last ? 1ull : 0ull, cs0};
            ht.insert(ht.end(), row, row + 8);
            nfc += cnt_w + nb;
            ent = ow->exit;
            continue;
        }
        u64 nx = 0;
        u32 nfn = 0;
        if ((rc = chunk_walk(ent, nfc, cs0 + C, nx, nfn)) < 0) return rc;
        last = rc == 1;                                                      // it finished the stream
        ent = nx;
        nfc = nfn;
    }
    const u32 nblk = (u32)(ht.size() / 8);
    ws_stat_rw_chunks = nblk;
    if (nblk) {
        if ((e = hipMemcpyAsync(tab, ht.data(), ht.size() * 8, hipMemcpyHostToDevice, st)) != hipSuccess)
            return ws_set_err("hipMemcpyAsync(stream chain)", e);
        hipLaunchKernelGGL(ws_rw_emit_kernel, dim3(nblk), dim3(64), 0, st, d_buf, len, max_frames, tab, own, stg, stgn,
                           d_desc, Pw.items, Pw.ptr, Pw.npieces, Pw.nwork, d_res, (RwPlan*)nullptr, 0);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_rw_emit_kernel launch", e);
    }
    // `ht` is pageable host memory read by the copy above: complete it before returning
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return ws_set_err("hipStreamSynchronize", e);
    return 0;
}

// A captured call's chunk-parallel walk: scratch sized from the stream length (caps), the
// geometry chosen on the device (ws_rw_plan_kernel). Layout after the aux head.
struct RwDevLayout {
    u64 cmin, nch_cap, cand_cap, stg_cap;
    size_t o_plan, o_recs, o_nrec, o_dx, o_own, o_tab, o_stg, o_cand, o_lk, bytes, zero_bytes;
};
static RwDevLayout rw_dev_layout(u64 len) {
    RwDevLayout L;
    L.cmin = RW_CMIN;
    while ((len + L.cmin - 1) / L.cmin + 2 > RW_CAP_CHUNKS) L.cmin <<= 1;
    L.nch_cap = (len + L.cmin - 1) / L.cmin + 2;
    L.cand_cap = std::min<u64>(L.nch_cap * (RW_HMAX / 32), len / 1024 + 65536);
    L.stg_cap = std::min<u64>(L.nch_cap * RW_D * RW_CAP_STGN, len / 256 + 65536);
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o = 0;
    L.o_plan = o; o += up(sizeof(RwPlan));
    L.o_nrec = o; o += up(L.nch_cap * 16);                                   // zeroed: counters,
    L.o_dx = o; o += up(L.nch_cap * RW_D * 8);                               // claimed exits
    L.zero_bytes = o - L.o_nrec;
    L.o_recs = o; o += up((L.nch_cap * RW_SLOTS + RW_SLAST) * sizeof(RwRec));
    L.o_own = o; o += up(L.nch_cap * RW_D * sizeof(RwOwn));
    L.o_tab = o; o += up((L.nch_cap + 2) * 64);
    L.o_stg = o; o += up(L.stg_cap * 4);
    L.o_cand = o; o += up(L.cand_cap * 8);
    L.o_lk = o; o += up(L.nch_cap * sizeof(RwLink));
    L.bytes = o;
    return L;
}

// The split of a device-planned walk (round 6): K2 runs as one launch per
// part (pieces [0, p[0]), [p[0], p[1]), ..., [p[last], npieces)), and the walk of each part after
// part 0 runs on a side stream while the earlier launches stream. Side-stream work joins the
// caller's stream through events (a capture forks and joins through them too: the side stream's
// work becomes a graph branch, option stream_split_capture).
struct RwSplit {
    u32 ncut = 0;                // K2 cut points (parts - 1); 0 = no split
    u64 p[RW_NP - 1] = {};       // the cuts (pieces)
    u64 x[RW_NP - 1] = {};       // the first stream byte of the piece at each cut
    hipStream_t side = nullptr;
    hipEvent_t ev[RW_NP + 1] = {};   // side start, part 0 done, part 1 done, ...
    int wait = 0;                // part 1's R1-R3 start after: 0 the plan, 1 part 0's R3, 2 part 0's emit
    u32 shift[RW_NP - 1] = {2, 1};   // part 0's / a middle part's chunks: C >> shift
};

static int rw_walk_device(unsigned char* d_buf, u64 len, u32 max_frames, WebsocketFrameDesc_t* d_desc,
                          const PieceWs& Pw, WebsocketSegResult_t* d_res, hipStream_t st, SdState* sd,
                          unsigned char* w, const RwDevLayout& L, int fresh = 0, u64* d_seg = nullptr,
                          SdMirror* mirror = nullptr, const RwSplit* sp = nullptr) {
    RwPlan* plan = reinterpret_cast<RwPlan*>(w + L.o_plan);
    u32* nrec = reinterpret_cast<u32*>(w + L.o_nrec);
    unsigned long long* dx = reinterpret_cast<unsigned long long*>(w + L.o_dx);
    RwRec* recs = reinterpret_cast<RwRec*>(w + L.o_recs);
    RwOwn* own = reinterpret_cast<RwOwn*>(w + L.o_own);
    u64* tab = reinterpret_cast<u64*>(w + L.o_tab);
    u32* stg = reinterpret_cast<u32*>(w + L.o_stg);
    u64* cand = reinterpret_cast<u64*>(w + L.o_cand);
    RwLink* lk = reinterpret_cast<RwLink*>(w + L.o_lk);
    const int cmax_log = ws_stream_rw_cmax;                                  // one read per call
    const bool split = sp && sp->ncut;
    // a split walk's last part runs beside K2: chunks twice the usual largest (fewer windows for R1 to
    // scan beside the stream; its longer owner walks are hidden), the earlier parts' that >> shift
    const u64 cmax = std::min<u64>((cmax_log >= 16 && cmax_log <= 26 ? 1ull << cmax_log : RW_CMAX) << (split ? 1 : 0),
                                   RW_CMAX);
    hipError_t e = hipMemsetAsync(nrec, 0, L.zero_bytes, st);
    if (e != hipSuccess) return ws_set_err("hipMemsetAsync(stream walk counters)", e);
    hipLaunchKernelGGL(ws_rw_plan_kernel, dim3(1), dim3(64), 0, st, d_buf, len, max_frames, sd, plan, L.cmin, cmax,
                       (u32)L.nch_cap, L.cand_cap, L.stg_cap, d_desc, Pw.items, Pw.ptr, Pw.npieces, Pw.nwork, d_res,
                       fresh, d_seg, Pw.disorder, mirror, split ? sp->x[0] : 0ull, split && sp->ncut > 1 ? sp->x[1] : 0ull,
                       split ? sp->shift[0] : 0u, split ? sp->shift[1] : 0u);
    // one part's candidate, window and owner walks; its linking and emit
    auto rwalk = [&](hipStream_t s, int part) {
        // R1 and R2 grid-stride, R3 one lane per (chunk, exit): grids for the caps
        hipLaunchKernelGGL(ws_rw_cand_kernel, dim3(RW_R1_GRID), dim3(256), 0, s, d_buf, len, (u64)0, (u64)1, (u32)64, 0u,
                           0u, cand, nrec, 0u, (const RwPlan*)plan, part);
        hipLaunchKernelGGL(ws_rw_spec_kernel, dim3(RW_R2_GRID), dim3(256), 0, s, d_buf, len, (u64)0, (u64)1, (u32)64, 0u,
                           0u, (const u64*)cand, 0u, recs, nrec, dx, (const RwPlan*)plan, part);
        hipLaunchKernelGGL(ws_rw_own_kernel, dim3((u32)((L.nch_cap * RW_D + RW_OWN_T - 1) / RW_OWN_T)), dim3(RW_OWN_T), 0,
                           s, d_buf, len, (u64)0, (u64)1, 0u, 0u, (const unsigned long long*)dx, own, stg, 0u,
                           (const RwPlan*)plan, part);
    };
    auto rlink = [&](hipStream_t s, int part) {
        if (ws_stream_plink) {      // the chunk-parallel linker; the serial one below exits if it linked
            hipLaunchKernelGGL(ws_rw_plink_kernel, dim3((u32)L.nch_cap), dim3(64), 0, s, len, (const RwPlan*)plan,
                               (const RwRec*)recs, (const u32*)nrec, (const unsigned long long*)dx, (const RwOwn*)own,
                               lk, part);
            hipLaunchKernelGGL(ws_rw_pscan_kernel, dim3(1), dim3(RW_PS_T), 0, s, max_frames, plan, (const RwLink*)lk, tab,
                               (const RwOwn*)own, part);
        }
        hipLaunchKernelGGL(ws_rw_link_kernel, dim3(1), dim3(64), 0, s, d_buf, len, max_frames, plan, (const RwRec*)recs,
                           (const u32*)nrec, (const unsigned long long*)dx, (const RwOwn*)own, tab, d_desc, Pw.items,
                           Pw.ptr, Pw.npieces, Pw.nwork, d_res, part);
        hipLaunchKernelGGL(ws_rw_emit_kernel, dim3((u32)(L.nch_cap + 2)), dim3(64), 0, s, d_buf, len, max_frames,
                           (const u64*)tab, (const RwOwn*)own, (const u32*)stg, 0u, d_desc, Pw.items, Pw.ptr,
                           Pw.npieces, Pw.nwork, d_res, plan, part);
    };
    if (!split) {
        rwalk(st, 0);
        rlink(st, 0);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("stream walk (device) launch", e);
        return 0;
    }
#define RW_TRY(call, what) do { if ((e = (call)) != hipSuccess) return ws_set_err(what, e); } while (0)
    if (sp->wait == 0) {
        RW_TRY(hipEventRecord(sp->ev[0], st), "hipEventRecord(stream split)");
        RW_TRY(hipStreamWaitEvent(sp->side, sp->ev[0], 0), "hipStreamWaitEvent(stream split)");
        rwalk(sp->side, 1);
    }
    rwalk(st, 0);
    if (sp->wait == 1) {
        RW_TRY(hipEventRecord(sp->ev[0], st), "hipEventRecord(stream split)");
        RW_TRY(hipStreamWaitEvent(sp->side, sp->ev[0], 0), "hipStreamWaitEvent(stream split)");
        rwalk(sp->side, 1);
    }
    rlink(st, 0);
    RW_TRY(hipEventRecord(sp->ev[1], st), "hipEventRecord(stream split)");
    RW_TRY(hipStreamWaitEvent(sp->side, sp->ev[1], 0), "hipStreamWaitEvent(stream split)");
    if (sp->wait >= 2) rwalk(sp->side, 1);
    rlink(sp->side, 1);
    RW_TRY(hipEventRecord(sp->ev[2], sp->side), "hipEventRecord(stream split)");
    for (u32 k = 2; k <= sp->ncut; ++k) {                                    // later parts, one after the other
        rwalk(sp->side, (int)k);
        rlink(sp->side, (int)k);
        RW_TRY(hipEventRecord(sp->ev[k + 1], sp->side), "hipEventRecord(stream split)");
    }
#undef RW_TRY
    if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("stream walk (device) launch", e);
    return 0;
}

// K2 after a device-planned walk: one launch, or (split) one launch per part's pieces — launch k
// (pieces [p[k-1], p[k])) with the item count part k left in the plan, once part k is emitted; the
// last launch with the stream's final count
std::atomic<unsigned long long> ws_stat_stream_splits{0};   // raw-stream calls whose K2 ran split (since load)
static int rw_unmask(const WsLaunch& L, const PieceWs& Pw, u32 gen, const RwSplit* sp, const RwPlan* plan) {
    if (!sp || !sp->ncut) return ws_launch_piece_unmask(L, Pw, gen);
    ++ws_stat_stream_splits;
    const u64 cpp = 1ull << (PIECE_SHIFT_S - 4);                             // 16-B chunks per piece
    for (u32 k = 0; k <= sp->ncut; ++k) {
        const u64 a = k ? sp->p[k - 1] : 0, b = k < sp->ncut ? sp->p[k] : Pw.npieces;
        if (k) {
            hipError_t e = hipStreamWaitEvent(L.stream, sp->ev[k + 1], 0);
            if (e != hipSuccess) return ws_set_err("hipStreamWaitEvent(stream split join)", e);
        }
        if (b <= a) continue;
        PieceWs A = Pw;
        A.ptr = Pw.ptr + a;
        A.pbase = Pw.pbase + a;
        A.npieces = b - a;
        A.c_lo = std::max<u64>(Pw.c_lo, a * cpp);
        A.c_hi = k < sp->ncut ? std::min<u64>(Pw.c_hi, b * cpp) : Pw.c_hi;
        if (k < sp->ncut) A.nwork = const_cast<u32*>(&plan->nw[k]);
        const int rc = ws_launch_piece_unmask(L, A, gen);
        if (rc) return rc;
    }
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
    // workspace: the piece path's layout for one segment [0, len), then the segment's
    // (offset, length) pair for the unmask kernel; the pass loop's state rests in the head
    // of the stream's auxiliary workspace
    const size_t pws = ws_piece_workspace_bytes(len, 1, max_frames);
    void* ws = nullptr;
    WsSlot slot;                              // every buffer of this call comes from one pinned slot
    int rc = slot.acquire(st);
    if (rc || (rc = slot.workspace(pws + 64, 16, &ws))) return rc;
    unsigned char* w8 = reinterpret_cast<unsigned char*>(ws);
    u64* d_seg = reinterpret_cast<u64*>(w8 + ((pws + 15) & ~(size_t)15));    // [0] offset 0, [1] length
    const bool capture = ws_capturing(st);
    // An eager call on a stream long enough for the chunk-parallel walk reads the state after
    // every round (published by the resolve kernel into pinned host memory, no copy): another
    // round while rounds pay, the chunk-parallel walk once lengths keep changing. A captured
    // call (and any shorter stream) never reads it: `nr` rounds, the last one's resolve also
    // walks whatever is left with one wavefront.
    const int rw_opt = ws_stream_rw;                                         // one read per call
    const bool rw = rw_opt != 0;
    const bool host_rw = rw && len >= RW_MIN && !capture;
    // a captured call on a long stream runs the chunk-parallel walk on the device (its
    // scratch, sized from the length, follows the state in the aux workspace); so does an
    // eager call once its published state says the lengths keep changing (stream_rw 1), unless
    // stream_rw 2 asks for the host to follow the chunk records (round 2's eager form)
    const bool dev_rw = rw && len >= RW_MIN && capture;
    const bool dev_layout = rw && len >= RW_MIN && (capture || rw_opt == 1);
    const RwDevLayout RL = dev_layout ? rw_dev_layout(len) : RwDevLayout{};
    WsAux A;
    if ((rc = slot.aux(WS_AUX_HEAD + (dev_layout ? RL.bytes : 0), host_rw ? WS_AUX_HEAD : 0, &A))) return rc;
    SdState* sd = reinterpret_cast<SdState*>(A.d);
    SdMirror* hm = host_rw ? reinterpret_cast<SdMirror*>(A.h) : nullptr;
    SdMirror* dm = host_rw ? reinterpret_cast<SdMirror*>(A.h_dev) : nullptr;
    WsLaunch L;
    L.buf = d_buf; L.seg_off = d_seg; L.seg_len = d_seg + 1; L.nseg = 1; L.max_frames = max_frames;
    L.desc_base = nullptr; L.desc = d_desc; L.res = d_res; L.stream = st;
    L.cus = slot.cus; L.lds_per_cu = slot.lds;
    L.pwin = ws_stream_win;
    PieceWs Pw;
    const u32 gen = ws_next_gen();
    // the piece-path views of the workspace
    {
        const u64 lead0 = reinterpret_cast<uintptr_t>(d_buf) & 15;
        Pw.npieces = len + lead0 ? ((len + lead0 - 1) >> PIECE_SHIFT_S) + 1 : 0;
        Pw.pbase = 0;
        Pw.c_lo = 0;
        Pw.c_hi = (len + lead0 + 15) >> 4;
        Pw.disorder = reinterpret_cast<u32*>(w8);
        Pw.nonuni = reinterpret_cast<u32*>(w8) + 1;
        Pw.ptr = reinterpret_cast<u64*>(w8 + 16);
        size_t b = (16 + Pw.npieces * 8 + 15) & ~(size_t)15;
        Pw.nwork = reinterpret_cast<u32*>(w8 + b);
        b = (b + 4 + 15) & ~(size_t)15;
        Pw.items = reinterpret_cast<u32x4*>(w8 + b);
    }
    if (!*A.state_ok) {                       // a previous call stopped between its launches
        hipLaunchKernelGGL(ws_stream_init_kernel, dim3(1), dim3(1), 0, st, sd);
        if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_stream_init_kernel launch", e);
    }
    *A.state_ok = false;
    // pass B's grid: every candidate a stream of this length and max_frames can have, grid-stride
    u64 kmax = std::min<u64>(std::min<u64>(len / 2 + 1, (u64)max_frames + 1), SD_KMAX);
    const u32 b_blocks = (u32)std::max<u64>(1, std::min<u64>((kmax + SPASS_T - 1) / SPASS_T, 8192));
    int round = 0;
    auto rounds = [&](int n, bool finish_last, u32 tag, int dev_hint) -> int {
        for (int r = 0; r < n; ++r, ++round) {
            const int first = round == 0, fin = finish_last && r == n - 1;
            hipLaunchKernelGGL(ws_stream_pass_kernel, dim3(SD_PROBE_K / SPASS_T), dim3(SPASS_T), 0, st, d_buf, (u64)len,
                               max_frames, 0, first, d_desc, Pw.items, Pw.ptr, Pw.npieces, sd, d_seg, Pw.disorder,
                               dev_hint);
            hipLaunchKernelGGL(ws_stream_pass_kernel, dim3(b_blocks), dim3(SPASS_T), 0, st, d_buf, (u64)len, max_frames,
                               1, first, d_desc, Pw.items, Pw.ptr, Pw.npieces, sd, d_seg, Pw.disorder, dev_hint);
            hipLaunchKernelGGL(ws_stream_resolve_kernel, dim3(64), dim3(SPASS_T), 0, st, d_buf, (u64)len, max_frames,
                               first, fin, d_desc, Pw.items, Pw.ptr, Pw.npieces, sd, Pw.nwork, d_res, dm, tag, dev_hint);
        }
        const hipError_t e2 = hipGetLastError();
        return e2 == hipSuccess ? 0 : ws_set_err("ws_stream_pass_kernel launch", e2);
    };
    const int nr0 = ws_stream_rounds, nr = nr0 >= 1 && nr0 <= 64 ? nr0 : 4;
    // the split of a device-planned walk (RwSplit): K2's first launch owns pieces [0, p0)
    RwSplit SP;
    unsigned char* const rw_w = reinterpret_cast<unsigned char*>(A.d) + WS_AUX_HEAD;
    const RwPlan* const rw_plan = reinterpret_cast<const RwPlan*>(rw_w + RL.o_plan);
    // (captured calls too unless stream_split_capture is 0: the side stream's work becomes a graph
    // branch, which the runtime runs beside the unmask's launches)
    if (dev_layout && (!capture || ws_stream_split_capture)) {
        const int spl = ws_stream_split, spl2 = ws_stream_split2, sw = ws_stream_split_wait;   // one read each
        const int c0 = ws_stream_c0, c1 = ws_stream_c1, pr = ws_stream_side_prio;
        if (spl > 0 && spl < 256 && Pw.npieces >= 3) {
            const u64 lead0 = reinterpret_cast<uintptr_t>(d_buf) & 15;
            SP.p[0] = std::max<u64>(1, Pw.npieces * (u64)spl / 256);
            SP.ncut = 1;
            if (spl2 > spl && spl2 < 256) {
                const u64 p1 = Pw.npieces * (u64)spl2 / 256;
                if (p1 > SP.p[0] && p1 < Pw.npieces) SP.p[SP.ncut++] = p1;
            }
            for (u32 k = 0; k < SP.ncut; ++k) SP.x[k] = (SP.p[k] << PIECE_SHIFT_S) - lead0;
            SP.wait = sw >= 0 && sw <= 2 ? sw : 0;
            SP.shift[0] = c0 >= 0 && c0 <= 6 ? (u32)c0 : 2u;
            SP.shift[1] = c1 >= 0 && c1 <= 6 ? (u32)c1 : 1u;
            if ((rc = slot.side(&SP.side, SP.ev, pr >= 0 && pr <= 2 ? pr : 0))) return rc;
        }
    }
    if (dev_rw) {
        // a replay whose previous replay's chunk walk saw lengths that keep changing skips the
        // rounds on the device (they exit at once) and the plan kernel starts the walk at 0
        if ((rc = rounds(nr, false, 0, 1))) return rc;
        if ((rc = rw_walk_device(d_buf, len, max_frames, d_desc, Pw, d_res, st, sd, rw_w, RL, 2, d_seg, nullptr, &SP)))
            return rc;
        *A.state_ok = true;
        return rw_unmask(L, Pw, gen, &SP, rw_plan);
    }
    if (!host_rw) {
        if ((rc = rounds(nr, true, 0, 0))) return rc;
        *A.state_ok = true;
        return ws_launch_piece_unmask(L, Pw, gen);
    }
    // eager: one round, then follow the published state
    auto published = [&](u32 tag) -> int {
        for (u64 it = 0;; ++it) {
            if (__atomic_load_n(&hm->gen, __ATOMIC_ACQUIRE) == tag) return 0;
            if ((it & 1023) == 1023) {
                const hipError_t q = hipStreamQuery(st);
                if (q == hipSuccess) {
                    if (__atomic_load_n(&hm->gen, __ATOMIC_ACQUIRE) == tag) return 0;
                    return ws_set_msg("websocketframeStreamDecodeDevice: pass state not published");
                }
                if (q != hipErrorNotReady) return ws_set_err("stream state wait", q);
            }
            __builtin_ia32_pause();
        }
    };
    // the previous chunk walk on this stream saw lengths that keep changing: no pass rounds and
    // no wait for their published state — the device walk starts at 0 (its plan kernel re-checks
    // the lengths on its sample and tells the next call)
    if (rw_opt == 1 && __atomic_load_n(&hm->walk_hint, __ATOMIC_RELAXED) == 1) {
        ++ws_stat_stream_skips;
        *A.state_ok = true;
        if ((rc = rw_walk_device(d_buf, len, max_frames, d_desc, Pw, d_res, st, sd, rw_w, RL, 1, d_seg, dm, &SP)))
            return rc;
        return rw_unmask(L, Pw, gen, &SP, rw_plan);
    }
    u32 tag = ws_next_gen();
    if ((rc = rounds(1, false, tag, 0)) || (rc = published(tag))) return rc;
    while (hm->phase == SD_PASSES) {
        tag = ws_next_gen();
        if ((rc = rounds(1, false, tag, 0)) || (rc = published(tag))) return rc;
    }
    *A.state_ok = true;
    if (hm->phase != SD_DONE) {
        const u64 P = hm->P;
        const u32 nf = hm->nf;
        if (len - P >= RW_MIN && rw_opt == 1) {                              // lengths keep changing:
            if ((rc = rw_walk_device(d_buf, len, max_frames, d_desc, Pw, d_res, st, sd, rw_w, RL, 0, d_seg, dm,
                                     &SP)))                                  // the device walks
                return rc;
            return rw_unmask(L, Pw, gen, &SP, rw_plan);
        } else if (len - P >= RW_MIN) {                                      // ... the host follows
            if ((rc = rw_walk(slot, d_buf, len, P, nf, max_frames, d_desc, Pw, d_res, st))) return rc;
        } else {
            hipLaunchKernelGGL(ws_stream_finish_kernel, dim3(1), dim3(64), 0, st, d_buf, (u64)len, max_frames, d_desc,
                               Pw.items, Pw.ptr, Pw.npieces, Pw.nwork, d_res, sd);
            if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_stream_finish_kernel launch", e);
        }
    }
    return ws_launch_piece_unmask(L, Pw, gen);
}
