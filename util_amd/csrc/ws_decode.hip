// ws_decode.hip — MI355X (gfx950) batch decode of WebSocket frames.
//
// Replaces, for device-resident batches, the reactor's rx hot loop
// (src/component/net_reactor.c:515-526) calling websocketframeDecode
// (src/crt/protocol/websocketframe.c:112-165) once per frame. Semantics are the
// reference's, bit for bit, including its quirks (u64 length-sum wrap at :149,
// int truncation of the return at :164, unvalidated opcode/RSV bits).
//
// Design:
//   * One wavefront owns one rx segment at a time (a connection's inbuf) and
//     walks its frames in order, exactly like the reactor loop. Header parsing
//     is wave-uniform scalar work: 5 lanes fetch the <=14 header bytes as
//     aligned dwords, v_readlane moves them to SGPRs, SALU decodes them.
//   * The payload is unmasked by the whole wave with 16-byte coalesced
//     loads/stores over the 16-B-aligned interior of the payload; the key is
//     rotated once per frame by (payload_start & 3) so every dword of a chunk
//     takes the same 32-bit mask. The <=15 unaligned bytes at each payload end
//     are done by 32 lanes with byte loads/stores, so bytes outside the
//     payload (headers, neighbouring frames/segments) are never written: no
//     read-modify-write races between waves.
//   * The next frame's header words are fetched together with the current
//     payload, so a frame costs one memory round trip per wave; thousands of
//     resident waves keep HBM busy.
//   * Only the frame's own bytes are read once and the payload written once:
//     algorithmic traffic = Σ wire + Σ payload.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/wsframe_amd.h"
#include "ws_synth.h"

typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// cache policy of the payload stream (A/B-able): 0 plain, 1 nontemporal loads+stores, 2 nt stores
template <int NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
    if constexpr (NT == 1) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int NT>
__device__ __forceinline__ void st16(u32x4 v, u32x4* p) {
    if constexpr (NT >= 1) __builtin_nontemporal_store(v, p);
    else *p = v;
}

#define WS_WAVES_PER_BLOCK 4
#define WS_BLOCK (64 * WS_WAVES_PER_BLOCK)

static __thread char g_last_error[256];

static int set_err(const char* what, hipError_t e) {
    snprintf(g_last_error, sizeof(g_last_error), "%s: %s", what, hipGetErrorString(e));
    return -(int)(e ? e : 1);
}

extern "C" WSFRAME_AMD_EXPORT const char* websocketframeGpuLastError(void) { return g_last_error; }

// ---------------------------------------------------------------------------------------------
// device helpers

// Header dword k (k = lane < 5) of the aligned window starting at floor4(p).
// Only dwords that contain at least one byte < end are read (never faults: an
// aligned dword with one valid byte lies in a mapped page).
__device__ __forceinline__ u32 load_header_dword(const unsigned char* p, const unsigned char* end, u32 lane) {
    const u32* q = reinterpret_cast<const u32*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    u32 v = 0;
    if (lane < 5 && reinterpret_cast<const unsigned char*>(q + lane) < end) v = __builtin_nontemporal_load(q + lane);
    return v;
}

__device__ __forceinline__ u32 rotl32(u32 x, u32 r) { return r ? (x << r) | (x >> (32 - r)) : x; }

// Unmask payload bytes [P0, P1) (absolute addresses) with LE key K, in place.
template <int U, int NT>
__device__ __forceinline__ void unmask_payload(unsigned char* P0, unsigned char* P1, u32 K, u32 lane) {
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(P0), a1 = reinterpret_cast<uintptr_t>(P1);
    const uintptr_t A = (a0 + 15) & ~(uintptr_t)15, B = a1 & ~(uintptr_t)15;
    // interior: 16-B aligned chunks, every dword takes the same rotated key
    if (A < B) {
        const u32 R = rotl32(K, 8u * (u32)(a0 & 3));
        u32x4* pa = reinterpret_cast<u32x4*>(A);
        const u64 n = (u64)(B - A) >> 4;
        for (u64 c0 = 0; c0 < n; c0 += 64 * U) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u64 c = c0 + (u64)(u * 64 + lane);
                if (c < n) v[u] = ld16<NT>(pa + c);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u64 c = c0 + (u64)(u * 64 + lane);
                if (c < n) {
                    st16<NT>(v[u] ^ R, pa + c);
                }
            }
        }
    }
    // edges: head [a0, min(A, a1)) on lanes 0-15, tail [max(A, B), a1) on lanes 16-31
    const uintptr_t head_end = A < a1 ? A : a1;
    const uintptr_t tail_beg = A > B ? A : B;
    uintptr_t x = 0;
    bool act = false;
    if (lane < 16) { x = a0 + lane; act = x < head_end; }
    else if (lane < 32) { x = tail_beg + (lane - 16); act = x < a1; }
    if (act) {
        unsigned char* px = reinterpret_cast<unsigned char*>(x);
        const u32 kb = (K >> (8u * (u32)((x - a0) & 3))) & 0xFFu;
        *px = (unsigned char)(*px ^ kb);
    }
}

// ---------------------------------------------------------------------------------------------
// the decode kernel: one wave per segment (grid-stride over segments)

template <int U, int NT>
__global__ __launch_bounds__(WS_BLOCK) void ws_decode_segments_kernel(
    unsigned char* __restrict__ buf, const u64* __restrict__ seg_off, const u64* __restrict__ seg_len, u32 nseg,
    u32 max_frames, const u64* __restrict__ desc_base, WebsocketFrameDesc_t* __restrict__ desc,
    WebsocketSegResult_t* __restrict__ res) {
    const u32 lane = threadIdx.x & 63;
    const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u32 nwaves = gridDim.x * WS_WAVES_PER_BLOCK;

    for (u32 s = blockIdx.x * WS_WAVES_PER_BLOCK + wave; s < nseg; s += nwaves) {
        const u64 so = seg_off[s], sl = seg_len[s];
        const u64 dbase = desc_base ? desc_base[s] : (u64)s * max_frames;
        unsigned char* const seg = buf + so;
        unsigned char* const end = seg + sl;
        u64 off = 0;
        u32 nf = 0;
        int status = WEBSOCKET_SEG_OK;
        u32 hv = load_header_dword(seg, end, lane);

        while (off < sl) {
            if (nf >= max_frames) { status = WEBSOCKET_SEG_MAX_FRAMES; break; }
            const u64 avail = sl - off;
            if (avail < 2) break;                                           // websocketframe.c:121
            unsigned char* const p = seg + off;
            // ---- header bytes 0..15 into two u64 (SGPRs)
            const u64 lo = (u64)(u32)__builtin_amdgcn_readlane(hv, 0) | ((u64)(u32)__builtin_amdgcn_readlane(hv, 1) << 32);
            const u64 mi = (u64)(u32)__builtin_amdgcn_readlane(hv, 2) | ((u64)(u32)__builtin_amdgcn_readlane(hv, 3) << 32);
            const u64 hi = (u64)(u32)__builtin_amdgcn_readlane(hv, 4);
            const u32 sh = 8u * (u32)(reinterpret_cast<uintptr_t>(p) & 3);
            const u64 h0 = sh ? (lo >> sh) | (mi << (64 - sh)) : lo;           // bytes 0..7
            const u64 h1 = sh ? (mi >> sh) | (hi << (64 - sh)) : mi;           // bytes 8..15
            // ---- websocketframe.c:124-147
            const u32 b0 = (u32)h0 & 0xFFu, b1 = (u32)(h0 >> 8) & 0xFFu;
            const u32 p7 = b1 & 0x7Fu;
            const u32 mask_len = (b1 >> 7) ? 4u : 0u;
            const u32 ext = p7 < 126 ? 0u : (p7 == 126 ? 2u : 8u);
            const u32 hdr = 2u + ext + mask_len;
            if (avail < hdr) break;                                         // :131,136,142
            u64 plen;
            if (ext == 0) plen = p7;
            else if (ext == 2) plen = ((h0 >> 16) & 0xFFu) << 8 | ((h0 >> 24) & 0xFFu);   // memReadBE16
            else plen = __builtin_bswap64((h0 >> 16) | (h1 << 48));                          // memReadBE64
            const u64 total = (u64)hdr + plen;                              // u64, may wrap (:149)
            if (avail < total) break;                                       // :149-150
            if (mask_len && total < plen) { status = WEBSOCKET_SEG_ERR_LEN_WRAP; break; }  // reference UB, fenced
            const int ret = (int)(u32)total;                                // :164
            // ---- prefetch the next frame's header words alongside this payload
            u32 hvn = 0;
            if (ret > 0 && off + (u32)ret < sl) hvn = load_header_dword(p + (u32)ret, end, lane);
            // ---- unmask (:152-158)
            if (mask_len) {
                const u32 K = ext == 0 ? (u32)(h0 >> 16) : (ext == 2 ? (u32)(h0 >> 32) : (u32)(h1 >> 16));
                unmask_payload<U, NT>(p + hdr, p + hdr + plen, K, lane);
            }
            if (ret == 0) break;                                            // (int) truncated to 0
            // ---- outputs (:160-163)
            if (lane == 0) {
                WebsocketFrameDesc_t* d = desc + dbase + nf;
                uint4 q0, q1;
                const u64 fo = so + off;
                const u64 dof = plen ? fo + hdr : WEBSOCKET_DATA_OFF_NULL;
                q0.x = (u32)fo; q0.y = (u32)(fo >> 32); q0.z = (u32)dof; q0.w = (u32)(dof >> 32);
                q1.x = (u32)plen; q1.y = (u32)(plen >> 32); q1.z = (u32)ret;
                q1.w = (b0 >> 7) | ((b0 & 0x0Fu) << 8) | ((b1 >> 7) << 16) | (hdr << 24);
                reinterpret_cast<uint4*>(d)[0] = q0;
                reinterpret_cast<uint4*>(d)[1] = q1;
            }
            ++nf;
            if (ret < 0) { status = WEBSOCKET_SEG_ERR_DECODE; break; }      // net_reactor.c:518-520
            off += (u32)ret;                                                // net_reactor.c:525
            hv = hvn;
        }
        if (lane == 0) {
            uint4 r;
            r.x = (u32)off; r.y = (u32)(off >> 32); r.z = nf; r.w = (u32)status;
            reinterpret_cast<uint4*>(res)[s] = r;
        }
    }
}

static int g_num_cus = 0;

static int num_cus() {
    if (!g_num_cus) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            g_num_cus = prop.multiProcessorCount;
        if (g_num_cus <= 0) g_num_cus = 256;
    }
    return g_num_cus;
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeBatchDecodeDevice(unsigned char* d_buf, const u64* d_seg_off,
                                                                  const u64* d_seg_len, unsigned int nseg,
                                                                  unsigned int max_frames, const u64* d_desc_base,
                                                                  WebsocketFrameDesc_t* d_desc,
                                                                  WebsocketSegResult_t* d_res, void* hip_stream) {
    if (nseg == 0) return 0;
    if (!d_buf || !d_seg_off || !d_seg_len || !d_desc || !d_res || max_frames == 0) {
        snprintf(g_last_error, sizeof(g_last_error), "websocketframeBatchDecodeDevice: invalid argument");
        return -1;
    }
    if ((reinterpret_cast<uintptr_t>(d_desc) | reinterpret_cast<uintptr_t>(d_res)) & 15) {
        snprintf(g_last_error, sizeof(g_last_error), "websocketframeBatchDecodeDevice: d_desc/d_res not 16-B aligned");
        return -1;
    }
    const u32 waves_wanted = nseg;
    u32 blocks = (waves_wanted + WS_WAVES_PER_BLOCK - 1) / WS_WAVES_PER_BLOCK;
    const u32 cap = (u32)num_cus() * 8u;  // 8 blocks x 4 waves = 32 waves per CU
    if (blocks > cap) blocks = cap;
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    hipLaunchKernelGGL((ws_decode_segments_kernel<4, 1>), dim3(blocks), dim3(WS_BLOCK), 0, st, d_buf, d_seg_off,
                       d_seg_len, (u32)nseg, (u32)max_frames, d_desc_base, d_desc, d_res);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err("ws_decode_segments_kernel launch", e);
    return 0;
}

// ---------------------------------------------------------------------------------------------
// host-buffer entry point: pinned staging + H2D + kernel + D2H (synchronous)

extern "C" WSFRAME_AMD_EXPORT int websocketframeBatchDecodeHost(unsigned char* h_buf, unsigned long long buflen,
                                                                const u64* h_seg_off, const u64* h_seg_len,
                                                                unsigned int nseg, unsigned int max_frames,
                                                                WebsocketFrameDesc_t* h_desc,
                                                                WebsocketSegResult_t* h_res, int device) {
    hipError_t e;
    unsigned char* d_buf = nullptr;
    u64 *d_off = nullptr, *d_len = nullptr;
    WebsocketFrameDesc_t* d_desc = nullptr;
    WebsocketSegResult_t* d_res = nullptr;
    hipStream_t st = nullptr;
    int rc = 0;
    const size_t ndesc = (size_t)nseg * max_frames;
    if (nseg == 0) return 0;
    if ((e = hipSetDevice(device)) != hipSuccess) return set_err("hipSetDevice", e);
#define WS_TRY(call, what) do { if ((e = (call)) != hipSuccess) { rc = set_err(what, e); goto out; } } while (0)
    WS_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
    WS_TRY(hipMalloc(&d_buf, buflen ? buflen : 1), "hipMalloc(buf)");
    WS_TRY(hipMalloc(&d_off, nseg * sizeof(u64)), "hipMalloc(seg_off)");
    WS_TRY(hipMalloc(&d_len, nseg * sizeof(u64)), "hipMalloc(seg_len)");
    WS_TRY(hipMalloc(&d_desc, (ndesc ? ndesc : 1) * sizeof(WebsocketFrameDesc_t)), "hipMalloc(desc)");
    WS_TRY(hipMalloc(&d_res, nseg * sizeof(WebsocketSegResult_t)), "hipMalloc(res)");
    WS_TRY(hipMemcpyAsync(d_buf, h_buf, buflen, hipMemcpyHostToDevice, st), "H2D buf");
    WS_TRY(hipMemcpyAsync(d_off, h_seg_off, nseg * sizeof(u64), hipMemcpyHostToDevice, st), "H2D seg_off");
    WS_TRY(hipMemcpyAsync(d_len, h_seg_len, nseg * sizeof(u64), hipMemcpyHostToDevice, st), "H2D seg_len");
    rc = websocketframeBatchDecodeDevice(d_buf, d_off, d_len, nseg, max_frames, nullptr, d_desc, d_res, st);
    if (rc) goto out;
    WS_TRY(hipMemcpyAsync(h_buf, d_buf, buflen, hipMemcpyDeviceToHost, st), "D2H buf");
    WS_TRY(hipMemcpyAsync(h_res, d_res, nseg * sizeof(WebsocketSegResult_t), hipMemcpyDeviceToHost, st), "D2H res");
    WS_TRY(hipStreamSynchronize(st), "hipStreamSynchronize");
    // descriptors: copy only the used prefix of every segment's slots
    for (u32 s = 0; s < nseg; ++s) {
        if (h_res[s].n_frames)
            WS_TRY(hipMemcpyAsync(h_desc + (size_t)s * max_frames, d_desc + (size_t)s * max_frames,
                                  h_res[s].n_frames * sizeof(WebsocketFrameDesc_t), hipMemcpyDeviceToHost, st),
                   "D2H desc");
    }
    WS_TRY(hipStreamSynchronize(st), "hipStreamSynchronize");
#undef WS_TRY
out:
    if (d_buf) (void)hipFree(d_buf);
    if (d_off) (void)hipFree(d_off);
    if (d_len) (void)hipFree(d_len);
    if (d_desc) (void)hipFree(d_desc);
    if (d_res) (void)hipFree(d_res);
    if (st) (void)hipStreamDestroy(st);
    return rc;
}

// ---------------------------------------------------------------------------------------------
// synthetic batches (bench/test input; ws_synth.h)

__global__ __launch_bounds__(256) void ws_synth_kernel(unsigned char* __restrict__ buf, const u64* __restrict__ frame_off,
                                                       u64 nframes, int plen_kind, u64 fixed_len, int b0_kind,
                                                       u64 seed) {
    for (u64 f = blockIdx.x; f < nframes; f += gridDim.x) {
        const u64 plen = ws_synth_plen(plen_kind, fixed_len, seed, f);
        const u32 key = ws_synth_key(seed, f);
        unsigned char* p = buf + frame_off[f];
        const u32 hl = ws_synth_headlen(plen) + 4u;
        if (threadIdx.x == 0) {
            unsigned char h[14];
            ws_synth_header(h, ws_synth_b0(b0_kind, f), plen, key);
            for (u32 i = 0; i < hl; ++i) p[i] = h[i];
        }
        unsigned char* pl = p + hl;
        const u64 km = (u64)key | ((u64)key << 32);
        const u64 nw = (plen + 7) >> 3;
        for (u64 j = threadIdx.x; j < nw; j += blockDim.x) {
            const u64 w = ws_synth_plain_word(seed, f, j) ^ km;
            const u64 nb = plen - 8 * j < 8 ? plen - 8 * j : 8;
            for (u64 b = 0; b < nb; ++b) pl[8 * j + b] = (unsigned char)(w >> (8 * b));
        }
    }
}

__global__ __launch_bounds__(256) void ws_verify_kernel(const unsigned char* __restrict__ buf,
                                                        const u64* __restrict__ frame_off, u64 nframes, int plen_kind,
                                                        u64 fixed_len, u64 seed, int expect_plain,
                                                        unsigned long long* __restrict__ mismatch) {
    u64 bad = 0;
    for (u64 f = blockIdx.x; f < nframes; f += gridDim.x) {
        const u64 plen = ws_synth_plen(plen_kind, fixed_len, seed, f);
        const u32 key = ws_synth_key(seed, f);
        const unsigned char* pl = buf + frame_off[f] + ws_synth_headlen(plen) + 4u;
        const u64 km = expect_plain ? 0ULL : ((u64)key | ((u64)key << 32));
        const u64 nw = (plen + 7) >> 3;
        for (u64 j = threadIdx.x; j < nw; j += blockDim.x) {
            const u64 w = ws_synth_plain_word(seed, f, j) ^ km;
            const u64 nb = plen - 8 * j < 8 ? plen - 8 * j : 8;
            for (u64 b = 0; b < nb; ++b) bad += pl[8 * j + b] != (unsigned char)(w >> (8 * b));
        }
    }
    for (int o = 32; o > 0; o >>= 1) bad += __shfl_down(bad, o);
    if ((threadIdx.x & 63) == 0 && bad) atomicAdd(mismatch, bad);
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeSynthDevice(unsigned char* d_buf, const u64* d_frame_off,
                                                            unsigned long long nframes, int plen_kind,
                                                            unsigned long long fixed_len, int b0_kind,
                                                            unsigned long long seed, void* hip_stream) {
    if (!nframes) return 0;
    const u32 blocks = nframes < 65536 ? (u32)nframes : 65536u;
    hipLaunchKernelGGL(ws_synth_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(hip_stream), d_buf,
                       d_frame_off, (u64)nframes, plen_kind, (u64)fixed_len, b0_kind, (u64)seed);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_err("ws_synth_kernel launch", e);
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeSynthVerifyDevice(const unsigned char* d_buf, const u64* d_frame_off,
                                                                  unsigned long long nframes, int plen_kind,
                                                                  unsigned long long fixed_len,
                                                                  unsigned long long seed, int expect_plain,
                                                                  unsigned long long* d_mismatch, void* hip_stream) {
    if (!nframes) return 0;
    const u32 blocks = nframes < 65536 ? (u32)nframes : 65536u;
    hipLaunchKernelGGL(ws_verify_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(hip_stream), d_buf,
                       d_frame_off, (u64)nframes, plen_kind, (u64)fixed_len, (u64)seed, expect_plain, d_mismatch);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_err("ws_verify_kernel launch", e);
}
