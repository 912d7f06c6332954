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

// The rest of the stream from (P0, nf0, g0) by one wavefront: the group walk of
// ws_piece.hip (64 lanes, stride speculation; only consumed frames are written), then the
// tail pointers, the item count and the segment result.
__global__ __launch_bounds__(64) void ws_stream_walk_kernel(const unsigned char* __restrict__ buf, u64 len, u64 P0,
                                                            u64 g0, u32 nf0, u32 max_frames,
                                                            WebsocketFrameDesc_t* __restrict__ desc,
                                                            u32x4* __restrict__ items, u64* __restrict__ ptr, u64 pend,
                                                            u32* __restrict__ nwork,
                                                            WebsocketSegResult_t* __restrict__ res) {
    const u32 lane = threadIdx.x;
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    const uintptr_t seg = reinterpret_cast<uintptr_t>(buf);
    u64 off = P0, g = g0, walked_end = lead0 + P0;
    u32 nf = nf0, extra = 0;
    int status = WEBSOCKET_SEG_OK;
    for (;;) {
        const u64 pos = off + (u64)lane * g;
        const bool cand = lane == 0 || g > 0;
        const bool eval = cand && pos < len;
        const uintptr_t pa = seg + (eval ? pos : 0);
        const gu32x4* q = reinterpret_cast<const gu32x4*>(pa & ~(uintptr_t)15);
        u64 h0, h1;
        ws_hdr_from32(q[0], q[1], (u32)(pa & 15), h0, h1);
        const WsHdr h = ws_parse(h0, h1, eval ? len - pos : 0);
        u32 code = 3;
        int st = WEBSOCKET_SEG_OK;
        if (cand) {
            if (pos >= len) code = 3;
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
        if (code_m == 2) {
            if (ret_m != 0) nf += 1;
            else extra = 1;
        }
        status = __builtin_amdgcn_readlane(st, (int)mm);
        break;
    }
    const u32 cnt = nf + extra;
    for (u64 p = ((walked_end + (1ull << PIECE_SHIFT_S) - 1) >> PIECE_SHIFT_S) + lane;
         (p << PIECE_SHIFT_S) < lead0 + len && p < pend; p += 64)
        ptr[p] = cnt;
    if (lane == 0) {
        nwork[0] = cnt;
        ws_store_res(res, off, nf, status);
    }
}

int ws_launch_piece_unmask(const WsLaunch& L, const PieceWs& P, int nt, u32 gen);

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
    for (;;) {
        const u64 remaining = len - P;
        u64 K = g ? remaining / g + 1 : 1;                                   // candidates this pass
        if (K > (u64)max_frames - nf + 1) K = (u64)max_frames - nf + 1;
        if (K > (1ull << 26)) K = 1ull << 26;
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
            continue;
        }
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
                hipLaunchKernelGGL(ws_stream_walk_kernel, dim3(1), dim3(64), 0, st, d_buf, (u64)len, P, g, nf,
                                   max_frames, d_desc, Pw.items, Pw.ptr, Pw.npieces, Pw.nwork, d_res);
                if ((e = hipGetLastError()) != hipSuccess) return ws_set_err("ws_stream_walk_kernel launch", e);
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
