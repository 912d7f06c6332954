// ws_bench.hip — libwsframe_amd_bench.so, bench/test support kernels (NOT part of the
// drop-in libwsframe_amd.so; include/wsframe_amd_bench.h):
//   * synthetic frame batches generated in HBM (ws_synth.h), and their verification;
//   * streaming-bandwidth calibration kernels (the ceilings DESIGN.md §4 quotes).
#include <stdio.h>

#include "ws_common.h"
#include "ws_synth.h"
#include "../../include/wsframe_amd_bench.h"

static __thread char g_bench_error[256];
int ws_set_err(const char* what, hipError_t e) {
    snprintf(g_bench_error, sizeof(g_bench_error), "%s: %s", what, hipGetErrorString(e));
    return -(int)(e ? e : 1);
}
int ws_set_msg(const char* msg) {
    snprintf(g_bench_error, sizeof(g_bench_error), "%s", msg);
    return -1;
}
extern "C" WSFRAME_AMD_EXPORT const char* websocketframeBenchLastError(void) { return g_bench_error; }

extern "C" WSFRAME_AMD_EXPORT int websocketframeBenchAlloc(void** d_ptr, unsigned long long nbytes, unsigned int flags) {
    const hipError_t e = hipExtMallocWithFlags(d_ptr, nbytes, flags);
    return e == hipSuccess ? 0 : ws_set_err("hipExtMallocWithFlags", e);
}
extern "C" WSFRAME_AMD_EXPORT int websocketframeBenchFree(void* d_ptr) {
    const hipError_t e = hipFree(d_ptr);
    return e == hipSuccess ? 0 : ws_set_err("hipFree", e);
}
extern "C" WSFRAME_AMD_EXPORT void* websocketframeBenchTorchAlloc(long long nbytes, int device, void* hip_stream) {
    (void)hip_stream;
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, (size_t)nbytes, hipDeviceMallocContiguous) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
        if (hipMalloc(&p, (size_t)nbytes) != hipSuccess) p = nullptr;
    }
    if (cur != device) (void)hipSetDevice(cur);
    return p;
}
extern "C" WSFRAME_AMD_EXPORT void websocketframeBenchTorchFree(void* d_ptr, long long nbytes, int device,
                                                              void* hip_stream) {
    (void)nbytes; (void)device; (void)hip_stream;
    (void)hipFree(d_ptr);
}

// ---------------------------------------------------------------------------------------------
// synthetic batches (bench/test input; ws_synth.h)

// frames first + i (global generator indices) at buf + frame_off[i], i < nframes
__global__ __launch_bounds__(256) void ws_synth_kernel(unsigned char* __restrict__ buf, const u64* __restrict__ frame_off,
                                                       u64 first, u64 nframes, int plen_kind, u64 fixed_len, int b0_kind,
                                                       u64 seed) {
    for (u64 i = blockIdx.x; i < nframes; i += gridDim.x) {
        const u64 f = first + i;
        const u64 plen = ws_synth_plen(plen_kind, fixed_len, seed, f);
        const u32 key = ws_synth_key(seed, f);
        unsigned char* p = buf + frame_off[i];
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
                                                        const u64* __restrict__ frame_off, u64 first, u64 nframes,
                                                        int plen_kind, u64 fixed_len, u64 seed, int expect_plain,
                                                        unsigned long long* __restrict__ mismatch) {
    u64 bad = 0;
    for (u64 i = blockIdx.x; i < nframes; i += gridDim.x) {
        const u64 f = first + i;
        const u64 plen = ws_synth_plen(plen_kind, fixed_len, seed, f);
        const u32 key = ws_synth_key(seed, f);
        const unsigned char* pl = buf + frame_off[i] + ws_synth_headlen(plen) + 4u;
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

extern "C" WSFRAME_AMD_EXPORT int websocketframeSynthDeviceRange(unsigned char* d_buf, const u64* d_frame_off,
                                                                 unsigned long long first_frame,
                                                                 unsigned long long nframes, int plen_kind,
                                                                 unsigned long long fixed_len, int b0_kind,
                                                                 unsigned long long seed, void* hip_stream) {
    if (!nframes) return 0;
    const u32 blocks = nframes < 65536 ? (u32)nframes : 65536u;
    hipLaunchKernelGGL(ws_synth_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(hip_stream), d_buf,
                       d_frame_off, (u64)first_frame, (u64)nframes, plen_kind, (u64)fixed_len, b0_kind, (u64)seed);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_synth_kernel launch", e);
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeSynthDevice(unsigned char* d_buf, const u64* d_frame_off,
                                                            unsigned long long nframes, int plen_kind,
                                                            unsigned long long fixed_len, int b0_kind,
                                                            unsigned long long seed, void* hip_stream) {
    return websocketframeSynthDeviceRange(d_buf, d_frame_off, 0, nframes, plen_kind, fixed_len, b0_kind, seed,
                                          hip_stream);
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeSynthVerifyDeviceRange(const unsigned char* d_buf,
                                                                       const u64* d_frame_off,
                                                                       unsigned long long first_frame,
                                                                       unsigned long long nframes, int plen_kind,
                                                                       unsigned long long fixed_len,
                                                                       unsigned long long seed, int expect_plain,
                                                                       unsigned long long* d_mismatch,
                                                                       void* hip_stream) {
    if (!nframes) return 0;
    const u32 blocks = nframes < 65536 ? (u32)nframes : 65536u;
    hipLaunchKernelGGL(ws_verify_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(hip_stream), d_buf,
                       d_frame_off, (u64)first_frame, (u64)nframes, plen_kind, (u64)fixed_len, (u64)seed, expect_plain,
                       d_mismatch);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_verify_kernel launch", e);
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeSynthVerifyDevice(const unsigned char* d_buf, const u64* d_frame_off,
                                                                  unsigned long long nframes, int plen_kind,
                                                                  unsigned long long fixed_len,
                                                                  unsigned long long seed, int expect_plain,
                                                                  unsigned long long* d_mismatch, void* hip_stream) {
    return websocketframeSynthVerifyDeviceRange(d_buf, d_frame_off, 0, nframes, plen_kind, fixed_len, seed,
                                                expect_plain, d_mismatch, hip_stream);
}

// ---------------------------------------------------------------------------------------------
// output hash of a decoded batch (multi-GPU bit-exactness across shardings): for every
// descriptor of every segment, ws_frame_hash(datalen, is_fin, type, payload bytes); summed
// mod 2^64 (order-independent, so any split of the frames over ranks and rounds gives the same
// total). util_amd/dist.py:frame_hash is the numpy statement of the same function.
__device__ __forceinline__ u64 ws_frame_hash_word(u64 w, u64 j) { return ws_mix64(w + 0x9E3779B97F4A7C15ULL * (j + 1)); }

__global__ __launch_bounds__(256) void ws_hash_kernel(const unsigned char* __restrict__ buf,
                                                      const WebsocketFrameDesc_t* __restrict__ desc,
                                                      const WebsocketSegResult_t* __restrict__ res, u32 nseg,
                                                      u32 max_frames, unsigned long long* __restrict__ out) {
    const u32 lane = threadIdx.x & 63;
    const u64 w = (u64)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (u64)gridDim.x * 4;
    u64 acc = 0;
    for (u64 slot = w; slot < (u64)nseg * max_frames; slot += nw) {
        const u32 s = (u32)(slot / max_frames), k = (u32)(slot % max_frames);
        if (k >= res[s].n_frames) continue;
        const WebsocketFrameDesc_t d = desc[slot];
        const u64 n = d.datalen;
        const unsigned char* p = d.data_off == WEBSOCKET_DATA_OFF_NULL ? buf : buf + d.data_off;
        u64 sum = 0;
        for (u64 j = lane; j < (n + 7) / 8; j += 64) {
            u64 x = 0;
            const u64 nb = n - 8 * j < 8 ? n - 8 * j : 8;
            for (u64 b = 0; b < nb; ++b) x |= (u64)p[8 * j + b] << (8 * b);
            sum += ws_frame_hash_word(x, j);
        }
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_down(sum, o);
        if (lane == 0) acc += ws_mix64(sum ^ n ^ ((u64)d.is_fin << 56) ^ ((u64)d.type << 48));
    }
    if (lane == 0 && acc) atomicAdd(out, acc);
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeFrameHashDevice(const unsigned char* d_buf,
                                                                const WebsocketFrameDesc_t* d_desc,
                                                                const WebsocketSegResult_t* d_res, unsigned int nseg,
                                                                unsigned int max_frames, unsigned long long* d_hash,
                                                                void* hip_stream) {
    if (!nseg) return 0;
    const u64 waves = (u64)nseg * max_frames;
    const u32 blocks = (u32)(waves / 4 + 1 < 65536 ? waves / 4 + 1 : 65536);
    hipLaunchKernelGGL(ws_hash_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(hip_stream), d_buf,
                       d_desc, d_res, nseg, max_frames, d_hash);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_hash_kernel launch", e);
}

// ---------------------------------------------------------------------------------------------
// diagnostics: streaming ceilings on this device for the decode's access pattern
// (flat grid-stride, 16 B per lane, no frame structure). mode 0: in-place XOR
// (read+write the same bytes, like the unmask); mode 1: copy src -> dst; mode 2: read-only.

template <int NT, int MODE>
__global__ __launch_bounds__(256) void ws_calib_kernel(gu32x4* __restrict__ a, gu32x4* __restrict__ b, u64 n,
                                                       u32 key, unsigned long long* __restrict__ sink) {
    const u64 stride = (u64)gridDim.x * 256 * 4;
    u32 acc = 0;
    for (u64 i = (u64)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const u64 j = i + 256u * u;
            v[u] = j < n ? ld16<NT>(a + j) : (u32x4)0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const u64 j = i + 256u * u;
            if (MODE == 0 && j < n) st16<NT>(v[u] ^ key, a + j);
            if (MODE == 1 && j < n) st16<NT>(v[u], b + j);
            if (MODE == 2) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    }
    if (MODE == 2 && acc == 0x9E3779B9u) atomicAdd(sink, 1ull);
}

// mode 3: in-place XOR, software-pipelined: the next iteration's loads issue
// BEFORE this iteration's stores, so waiting for loads never waits for stores.
template <int NT>
__global__ __launch_bounds__(256) void ws_calib_pipe_kernel(gu32x4* __restrict__ a, u64 n, u32 key) {
    // branch-free body (clamped indices, benign duplicate stores of identical values) so
    // the waitcnt pass sees one path: wait for `cur` = vmcnt(4) with `nxt` still in flight
    const u64 stride = (u64)gridDim.x * 1024;
    u64 i = (u64)blockIdx.x * 1024 + threadIdx.x;
    const u64 last = n - 1;
    const u32 iters = (u32)((n + stride - 1) / stride);
    u32x4 cur[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = ld16<NT>(a + min(i + 256u * u, last));
    for (u32 it = 0; it < iters; ++it) {
        const u64 nx = i + stride;
        u32x4 nxt[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) nxt[u] = ld16<NT>(a + min(nx + 256u * u, last));
#pragma unroll
        for (int u = 0; u < 4; ++u) st16<NT>(cur[u] ^ key, a + min(i + 256u * u, last));
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
        i = nx;
    }
}

// mode 4: in-place XOR, one-shot blocks (no loop; 16 KiB per 256-thread block)
template <int NT>
__global__ __launch_bounds__(256) void ws_calib_oneshot_kernel(gu32x4* __restrict__ a, u64 n, u32 key) {
    const u64 i = (u64)blockIdx.x * 1024 + threadIdx.x;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld16<NT>(a + min(i + 256u * u, n - 1));
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (i + 256u * u < n) st16<NT>(v[u] ^ key, a + i + 256u * u);
}

// mode 5+K: in-place XOR, one-shot blocks that each do K rounds of (4 loads, 4 stores)
template <int NT, int K>
__global__ __launch_bounds__(256) void ws_calib_rounds_kernel(gu32x4* __restrict__ a, u64 n, u32 key) {
    const u64 last = n - 1;
#pragma unroll 1
    for (int k = 0; k < K; ++k) {
        const u64 i = ((u64)blockIdx.x * K + k) * 1024 + threadIdx.x;
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = ld16<NT>(a + min(i + 256u * u, last));
#pragma unroll
        for (int u = 0; u < 4; ++u) st16<NT>(v[u] ^ key, a + min(i + 256u * u, last));
    }
}

// mode 70/71: persistent in-place XOR over 16 KiB pieces (4 loads + 4 stores per lane).
// 70: work stealing — a block takes its next piece from a global ticket counter (drawn
// while its loads are in flight), so CUs/XCDs that run faster take more pieces and the
// grid drains together; 71: static, block b takes pieces b, b+G, ...
template <bool STEAL>
__global__ __launch_bounds__(256) void ws_calib_persist_kernel(gu32x4* __restrict__ a, u64 n, u32* __restrict__ ctr,
                                                              u32 key) {
    __shared__ u32 s_next[2];
    const u64 npieces = (n + 1023) / 1024, last = n - 1;
    u64 piece;
    if (STEAL) {
        if (threadIdx.x == 0) s_next[0] = atomicAdd(ctr, 1u);
        __syncthreads();
        piece = s_next[0];
    } else {
        piece = blockIdx.x;
    }
    u32 par = 1;
#pragma unroll 1
    while (piece < npieces) {
        const u64 i = piece * 1024 + threadIdx.x;
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = ld16<1>(a + min(i + 256u * u, last));
        if (STEAL && threadIdx.x == 0) s_next[par] = atomicAdd(ctr, 1u);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + 256u * u < n) st16<1>(v[u] ^ key, a + i + 256u * u);
        if (STEAL) {
            __syncthreads();
            piece = s_next[par];
            par ^= 1u;
        } else {
            piece += gridDim.x;
        }
    }
}

// mode 72: one-shot grid over 16 KiB pieces split into W windows streamed side by side
// (block b takes piece (b % W) * ceil(P / W) + b / W)
__global__ __launch_bounds__(256) void ws_calib_windows_kernel(gu32x4* __restrict__ a, u64 n, u32 W, u64 ppw,
                                                              u32 key) {
    const u64 npieces = (n + 1023) / 1024, last = n - 1;
    const u64 piece = (u64)(blockIdx.x % W) * ppw + blockIdx.x / W;
    if (piece >= npieces) return;
    const u64 i = piece * 1024 + threadIdx.x;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld16<1>(a + min(i + 256u * u, last));
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (i + 256u * u < n) st16<1>(v[u] ^ key, a + i + 256u * u);
}

// mode 76: as 72, but each wave's four loads cover 4 KiB of consecutive chunks (K2's
// layout: wave w of the block takes chunks [w*256, w*256 + 256) of its piece) instead of
// four 1 KiB rows 4 KiB apart
template <int WAIT>
__global__ __launch_bounds__(256) void ws_calib_windows_wc_kernel(gu32x4* __restrict__ a, u64 n, u32 W, u64 ppw,
                                                                  u32 key) {
    const u64 npieces = (n + 1023) / 1024, last = n - 1;
    const u64 piece = (u64)(blockIdx.x % W) * ppw + blockIdx.x / W;
    if (piece >= npieces) return;
    const u64 i = piece * 1024 + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld16<1>(a + min(i + 64u * u, last));
    if (WAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every load back before the first store
    if (WAIT == 2) __builtin_amdgcn_s_sleep(32);                    // then a pause (~2k clocks)
    if (WAIT == 3) { __builtin_amdgcn_s_sleep(127); __builtin_amdgcn_s_sleep(127); }   // (~16k clocks)
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (i + 64u * u < n) st16<1>(v[u] ^ key, a + i + 64u * u);
}

// mode 88: as 76 with U chunks per lane (wave w of a 256-thread block covers U KiB of
// consecutive chunks, a block 4U KiB), two windows, and `dyn` bytes of unused dynamic LDS
// per block (caps blocks per CU): the shape/occupancy grid for K2
template <int U>
__global__ __launch_bounds__(256) void ws_calib_wcu_kernel(gu32x4* __restrict__ a, u64 n, u32 W, u64 ppw, u32 key) {
    const u64 per = 256ull * U, npieces = (n + per - 1) / per, last = n - 1;
    const u64 piece = (u64)(blockIdx.x % W) * ppw + blockIdx.x / W;
    if (piece >= npieces) return;
    const u64 i = piece * per + (threadIdx.x >> 6) * (64 * U) + (threadIdx.x & 63);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16<1>(a + min(i + 64u * u, last));
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + 64u * u < n) st16<1>(v[u] ^ key, a + i + 64u * u);
}

// mode 900/901: K2's block shape (256 threads, each wave 4 KiB of consecutive chunks, two
// windows) with only half of a wave's bytes in flight at a time: 900 = load half A, store
// it, then load and store half B; 901 = load A, wait for it, load B, store A, store B (B's
// loads overlap A's stores). `dyn` bytes of unused LDS cap blocks per CU.
template <int PH>
__global__ __launch_bounds__(256) void ws_calib_2ph_kernel(gu32x4* __restrict__ a, u64 n, u32 W, u64 ppw, u32 key) {
    const u64 per = 1024, npieces = (n + per - 1) / per, last = n - 1;
    const u64 piece = (u64)(blockIdx.x % W) * ppw + blockIdx.x / W;
    if (piece >= npieces) return;
    const u64 i = piece * per + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
    u32x4 v[2], w[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) v[u] = ld16<1>(a + min(i + 64u * u, last));
    if (PH == 0) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
            if (i + 64u * u < n) st16<1>(v[u] ^ key, a + i + 64u * u);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < 2; ++u) w[u] = ld16<1>(a + min(i + 128u + 64u * u, last));
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < 2; ++u) w[u] = ld16<1>(a + min(i + 128u + 64u * u, last));
#pragma unroll
        for (int u = 0; u < 2; ++u)
            if (i + 64u * u < n) st16<1>(v[u] ^ key, a + i + 64u * u);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
        if (i + 128u + 64u * u < n) st16<1>(w[u] ^ key, a + i + 128u + 64u * u);
}

// mode 89x: blocks of T threads, U chunks per lane, wave-contiguous, two windows, and
// (SYNC) a block-level hand-off between the loads and the stores — wave 0 writes 64 words
// to LDS, barrier, every lane reads one before storing (a block that shares one lookup of
// its piece's frame records through LDS). `dyn` bytes of unused LDS cap blocks per CU.
template <int T, int U, bool SYNC>
__global__ __launch_bounds__(T) void ws_calib_blk_kernel(gu32x4* __restrict__ a, u64 n, u32 W, u64 ppw, u32 key) {
    __shared__ u32 sh[64];
    const u64 per = (u64)T * U, npieces = (n + per - 1) / per, last = n - 1;
    const u64 piece = (u64)(blockIdx.x % W) * ppw + blockIdx.x / W;
    if (piece >= npieces) return;
    const u64 i = piece * per + (threadIdx.x >> 6) * (64 * U) + (threadIdx.x & 63);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16<1>(a + min(i + 64u * u, last));
    u32 k = key;
    if (SYNC) {
        if (threadIdx.x < 64) sh[threadIdx.x] = (u32)piece + threadIdx.x;
        __syncthreads();
        k ^= sh[(threadIdx.x * 7) & 63] & 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + 64u * u < n) st16<1>(v[u] ^ k, a + i + 64u * u);
}

// mode 96/97/98: out-of-place copy a -> b in E3's shape (one-shot 256 x 4 blocks over 16 KiB
// output pieces, wave-contiguous), the source offset by 0 / 4 / 8 bytes (unaligned 16-B
// loads, as E3's payload loads behind a header of any length)
typedef u32x4 __attribute__((aligned(1))) cal_u32x4u;
template <int OFF>
__global__ __launch_bounds__(256) void ws_calib_copyoff_kernel(const unsigned char* __restrict__ a,
                                                               gu32x4* __restrict__ b, u64 n, u32 key) {
    const u64 npieces = (n + 1023) / 1024, last = n - 2;
    const u64 piece = blockIdx.x;
    if (piece >= npieces) return;
    const u64 i = piece * 1024 + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
        v[u] = *reinterpret_cast<const WS_GLOBAL cal_u32x4u*>(reinterpret_cast<uintptr_t>(a + 16 * min(i + 64u * u, last) + OFF));
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (i + 64u * u < n - 1) st16<1>(v[u] ^ key, b + i + 64u * u);
}

// mode 83: as 80, plus K2's lookups between the loads and the stores: a scalar load of a
// per-piece word from the table b, then 16 lanes load a 16-B entry it points at (entries
// spread over 16 MB like K2's items), consumed before the stores
__global__ __launch_bounds__(256) void ws_calib_windows_dep_kernel(gu32x4* __restrict__ a, u64 n, u32 W, u64 ppw,
                                                                   const u32* __restrict__ tab,
                                                                   const u32x4* __restrict__ items, u32 key) {
    const u64 npieces = (n + 1023) / 1024, last = n - 1;
    const u64 piece = (u64)(blockIdx.x % W) * ppw + blockIdx.x / W;
    if (piece >= npieces) return;
    const u32 lane = threadIdx.x & 63;
    const u64 i = piece * 1024 + (threadIdx.x >> 6) * 256 + lane;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld16<1>(a + min(i + 64u * u, last));
    const u32 k = *reinterpret_cast<const __attribute__((address_space(4))) u32*>(
        reinterpret_cast<uintptr_t>(tab + (piece & ((1u << 18) - 1))));
    u32x4 q = {0, 0, 0, 0};
    if (lane < 16) q = items[(k + lane) & ((1u << 20) - 1)];
    const u32 z = (q.x ^ q.y ^ q.z ^ q.w) & 0u;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (i + 64u * u < n) st16<1>(v[u] ^ (key ^ z), a + i + 64u * u);
}

// modes 73-75: the segment-kernel shape (segfuse / fused reassembly) without frame logic:
// one 256-thread block per "segment" of `segc` 16-B chunks (cfg5: 1032), segments taken in
// two windows (ws_winn), in-place XOR. 73: LDS-DMA of the segment (1 KiB slices by every
// wave), barrier, XOR from LDS, store (segfuse's data path); 74: the segment in registers
// (U chunks per lane), XOR, store (K2's data path at segment granularity); 75: as 74 plus a
// copy of the registers into LDS and a barrier before the stores (what a register-resident
// segment kernel needs for its walk).
typedef __attribute__((address_space(3))) void ws_lds_void;
template <int MODE, int U>
__global__ __launch_bounds__(256) void ws_calib_seg_kernel(gu32x4* __restrict__ a, u64 nseg, u32 segc, u32 half,
                                                           u32 key) {
    __shared__ __attribute__((aligned(16))) u32x4 win[U * 256];
    const u32 b = half ? (blockIdx.x & 1u) * half + (blockIdx.x >> 1) : blockIdx.x;
    if (b >= nseg) return;
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    gu32x4* const g = a + (u64)b * segc;
    if (MODE == 73) {
        const u32 nsl = (segc + 63) / 64;
        for (u32 i = wv; i < nsl; i += 4) {
            const u32 c = i * 64 + lane < segc ? i * 64 + lane : segc - 1;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const WS_GLOBAL void*>(g + c), (ws_lds_void*)(&win[i * 64]),
                                             16, 0, 2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 c = u * 256 + tid;
            if (c < segc) st16<1>(win[c] ^ key, g + c);
        }
    } else {
        // MODE 84/85: 74/75 with each wave's U loads over consecutive chunks (wave w: chunks
        // [w*U*64, (w+1)*U*64)), K2's layout
        auto ci = [&](int u) -> u32 { return (MODE == 84 || MODE == 85) ? wv * (U * 64) + u * 64 + lane : u * 256 + tid; };
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 c = ci(u);
            v[u] = ld16<1>(g + (c < segc ? c : segc - 1));
        }
        if (MODE == 75 || MODE == 85) {
#pragma unroll
            for (int u = 0; u < U; ++u) win[ci(u)] = v[u];
            __syncthreads();
            key ^= win[(tid * 7) & (U * 256 - 1)].x & 0u;   // a dependent LDS read (value unused)
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 c = ci(u);
            if (c < segc) st16<1>(v[u] ^ key, g + c);
        }
    }
}

// modes 86/87: the segment-kernel shape with every wave owning whole ABSOLUTE 4 KiB pages
// (the layout of mode 76, which streams 3.3 % faster than 1 KiB rows, kept when blocks are
// segments at any offset): the segment's chunks [c0, c1) touch pages c0>>8 .. (c1-1)>>8;
// wave w takes pages w, w+4 of that list. 86: in registers (4 loads per page); 87: LDS-DMA
// of the page's four 1 KiB rows into a window laid out on the absolute 1 KiB grid, barrier,
// XOR from LDS and store (segfuse's data path).
template <int MODE>
__global__ __launch_bounds__(256) void ws_calib_seg_pages_kernel(gu32x4* __restrict__ a, u64 nseg, u32 segc, u32 half,
                                                                 u32 key) {
    __shared__ __attribute__((aligned(16))) u32x4 win[MODE == 87 ? 6 * 256 : 1];
    const u32 b = half ? (blockIdx.x & 1u) * half + (blockIdx.x >> 1) : blockIdx.x;
    if (b >= nseg) return;
    const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const u64 c0 = (u64)b * segc, c1 = c0 + segc;
    const u64 pg0 = c0 >> 8, npg = ((c1 - 1) >> 8) - pg0 + 1;                 // <= 6 pages
    if (MODE == 86) {
        for (u64 p = wv; p < npg; p += 4) {
            u32x4 v[4];
            const u64 cb = (pg0 + p) << 8;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u64 c = cb + u * 64 + lane;
                v[u] = ld16<1>(a + (c < c0 ? c0 : (c < c1 ? c : c1 - 1)));
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u64 c = cb + u * 64 + lane;
                if (c >= c0 && c < c1) st16<1>(v[u] ^ key, a + c);
            }
        }
    } else {
        const u64 wbase = pg0 << 8;                                            // window chunk 0
        for (u64 p = wv; p < npg; p += 4)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u64 c = ((pg0 + p) << 8) + u * 64 + lane;
                __builtin_amdgcn_global_load_lds(
                    reinterpret_cast<const WS_GLOBAL void*>(a + (c < c0 ? c0 : (c < c1 ? c : c1 - 1))),
                    (ws_lds_void*)(&win[(p << 8) + u * 64]), 16, 0, 2);
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (u64 p = wv; p < npg; p += 4)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u64 c = ((pg0 + p) << 8) + u * 64 + lane;
                if (c >= c0 && c < c1) st16<1>(win[c - wbase] ^ key, a + c);
            }
    }
}

// mode 16+: one-shot in-place XOR through buffer instructions with explicit cache
// bits (aux: bit0 sc0, bit1 nt, bit4 sc1), T threads x U chunks per block.
template <int T, int U, int LAUX, int SAUX>
__global__ __launch_bounds__(T) void ws_calib_buf_kernel(unsigned char* __restrict__ a, u64 nbytes, u32 key) {
    const u64 blk = (u64)blockIdx.x * (T * U * 16);
    const u64 left = nbytes - blk;
    const u32 nrec = left < (u64)(T * U * 16) ? (u32)left : (u32)(T * U * 16);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a + blk, (short)0, (int)nrec, 0x00020000);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (threadIdx.x + u * T) * 16, 0, LAUX));
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v[u] ^ key), rs,
                                               (threadIdx.x + u * T) * 16, 0, SAUX);
}

// mode 40+: in-place XOR through an LDS pipeline. Wave 0 only issues LDS-DMA loads
// (global_load_lds, D stages of S chunks in flight, never a store, never an LDS read,
// so its vmcnt waits cover only its own loads); waves 1..NC only read LDS and store
// (never a global load, so no store ever delays a load). One barrier per stage.
template <int S, int D, int NC, bool IL>
__global__ __launch_bounds__(64 * (NC + 1)) void ws_calib_ldspipe_kernel(gu32x4* __restrict__ a, u64 nstages,
                                                                        u32 key) {
    constexpr int R = D + 1, NI = S / 64;
    static_assert(S % 64 == 0 && (D - 1) * NI <= 63, "vmcnt immediate");
    __shared__ __attribute__((aligned(16))) u32x4 lbuf[R * S];
    const u32 wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // IL: block b takes stages b, b+G, ... (all blocks stream one compact window);
    // otherwise one contiguous range per block
    const u64 per = (nstages + gridDim.x - 1) / gridDim.x;
    const u64 q0 = IL ? 0 : (u64)blockIdx.x * per;
    const u64 q1 = IL ? 0 : (q0 + per < nstages ? q0 + per : nstages);
    const u64 Q = IL ? (blockIdx.x < nstages ? (nstages - 1 - blockIdx.x) / gridDim.x + 1 : 0) : (q1 > q0 ? q1 - q0 : 0);
    if (Q == 0) return;
    auto stage = [&](u64 t) -> u64 { return IL ? t * gridDim.x + blockIdx.x : q0 + t; };
    auto issue = [&](u64 t) {
        gu32x4* g = a + stage(t) * S;
        u32x4* l = &lbuf[(t % R) * S];
#pragma unroll
        for (int i = 0; i < NI; ++i)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const WS_GLOBAL void*>(g + i * 64 + lane),
                                             (ws_lds_void*)(l + i * 64), 16, 0, 2);
    };
    if (wv == 0) {
        for (u64 t = 0; t < (u64)D && t < Q; ++t) issue(t);
        if (Q >= (u64)D) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * NI) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (u64 t = 0; t < Q; ++t) {
        if (wv == 0) {
            if (t + D < Q) {
                issue(t + D);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * NI) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        } else {
            const u32x4* l = &lbuf[(t % R) * S];
            gu32x4* g = a + stage(t) * S;
            for (u32 c = (wv - 1) * 64 + lane; c < (u32)S; c += NC * 64) st16<1>(l[c] ^ key, g + c);
        }
        __syncthreads();
    }
}

// mode 60+: one-shot in-place XOR blocks that also resolve a dependent lookup chain of
// depth DEP (each link a 16-B load whose address depends on the previous one; the
// last gives the XOR key) while their payload loads are in flight: what a one-shot
// unmask block pays to find its frame's key from a precomputed table. The table is
// the other buffer (d_b), read-only.
template <int T, int U, int DEP>
__global__ __launch_bounds__(T) void ws_calib_dep_kernel(gu32x4* __restrict__ a, const gu32x4* __restrict__ tbl,
                                                         u64 n, u64 ntbl) {
    const u64 i = (u64)blockIdx.x * (T * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16<1>(a + min(i + (u64)T * u, n - 1));
    u32 idx = blockIdx.x;
#pragma unroll
    for (int d = 0; d < DEP; ++d) {
        const u32x4 t = tbl[(idx * 2654435761u + d) % ntbl];
        idx = t.x ^ t.y;
    }
    const u32 key = idx | 1u;
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + (u64)T * u < n) st16<1>(v[u] ^ key, a + i + (u64)T * u);
}

template <int T, int U, int DEP>
static void cal_dep(gu32x4* a, gu32x4* b, u64 n, hipStream_t st) {
    const u64 per = (u64)T * U;
    hipLaunchKernelGGL((ws_calib_dep_kernel<T, U, DEP>), dim3((u32)((n + per - 1) / per)), dim3(T), 0, st, a, b, n,
                       (u64)(1u << 20));
}

template <int S, int D, int NC, bool IL = false>
static void cal_ldspipe(gu32x4* a, u64 n, int blocks, hipStream_t st) {
    hipLaunchKernelGGL((ws_calib_ldspipe_kernel<S, D, NC, IL>), dim3(blocks), dim3(64 * (NC + 1)), 0, st, a, n / S,
                       0x5A5A5A5Au);
}

template <int T, int U, int LAUX, int SAUX>
static void cal_buf(unsigned char* a, u64 n, hipStream_t st) {
    const u64 per = (u64)T * U * 16;
    hipLaunchKernelGGL((ws_calib_buf_kernel<T, U, LAUX, SAUX>), dim3((u32)((n + per - 1) / per)), dim3(T), 0, st, a, n,
                       0x5A5A5A5Au);
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeGpuCalibrate(void* d_a, void* d_b, unsigned long long nbytes, int mode,
                                                             int nt, int blocks, void* hip_stream) {
    const u64 n = nbytes / 16;
    if (blocks <= 0) blocks = 2048;
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    gu32x4* a = reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(d_a));
    gu32x4* b = reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(d_b));
    unsigned long long* sink = reinterpret_cast<unsigned long long*>(d_b);
    if (mode == 3) {
        if (nt) hipLaunchKernelGGL((ws_calib_pipe_kernel<1>), dim3(blocks), dim3(256), 0, st, a, n, 0x5A5A5A5Au);
        else hipLaunchKernelGGL((ws_calib_pipe_kernel<0>), dim3(blocks), dim3(256), 0, st, a, n, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_pipe_kernel launch", e);
    }
    if (mode == 4) {
        const u64 nb = (n + 1023) / 1024;
        if (nt) hipLaunchKernelGGL((ws_calib_oneshot_kernel<1>), dim3((u32)nb), dim3(256), 0, st, a, n, 0x5A5A5A5Au);
        else hipLaunchKernelGGL((ws_calib_oneshot_kernel<0>), dim3((u32)nb), dim3(256), 0, st, a, n, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_oneshot_kernel launch", e);
    }
    if (mode == 72) {  // `blocks` = number of windows
        const u32 W = blocks > 0 ? (u32)blocks : 2u;
        const u64 np = (n + 1023) / 1024, ppw = (np + W - 1) / W;
        hipLaunchKernelGGL(ws_calib_windows_kernel, dim3((u32)(ppw * W)), dim3(256), 0, st, a, n, W, ppw, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_windows_kernel launch", e);
    }
    if (mode >= 76 && mode <= 82) {  // `blocks` = number of windows; 77/78/79: unused dynamic LDS so that
                                     // at most 7 / 6 / 5 blocks fit a CU; 80: stores after every load is back;
                                     // 81 / 82: and after a pause of ~2k / ~16k clocks
        const u32 W = blocks > 0 ? (u32)blocks : 2u;
        const u64 np = (n + 1023) / 1024, ppw = (np + W - 1) / W;
        const u32 dyn = mode == 77 ? 21u << 10 : (mode == 78 ? 24u << 10 : (mode == 79 ? 30u << 10 : 0u));
        if (mode == 80)
            hipLaunchKernelGGL(ws_calib_windows_wc_kernel<1>, dim3((u32)(ppw * W)), dim3(256), 0, st, a, n, W, ppw,
                               0x5A5A5A5Au);
        else if (mode == 81)
            hipLaunchKernelGGL(ws_calib_windows_wc_kernel<2>, dim3((u32)(ppw * W)), dim3(256), 0, st, a, n, W, ppw,
                               0x5A5A5A5Au);
        else if (mode == 82)
            hipLaunchKernelGGL(ws_calib_windows_wc_kernel<3>, dim3((u32)(ppw * W)), dim3(256), 0, st, a, n, W, ppw,
                               0x5A5A5A5Au);
        else
            hipLaunchKernelGGL(ws_calib_windows_wc_kernel<0>, dim3((u32)(ppw * W)), dim3(256), dyn, st, a, n, W, ppw,
                               0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_windows_wc_kernel launch", e);
    }
    if (mode >= 96 && mode <= 98) {  // d_b: >= nbytes
        const u64 np = (n + 1023) / 1024;
        const unsigned char* a8 = reinterpret_cast<const unsigned char*>(d_a);
        if (mode == 96) hipLaunchKernelGGL(ws_calib_copyoff_kernel<0>, dim3((u32)np), dim3(256), 0, st, a8, b, n, 0x5A5A5A5Au);
        else if (mode == 97) hipLaunchKernelGGL(ws_calib_copyoff_kernel<4>, dim3((u32)np), dim3(256), 0, st, a8, b, n, 0x5A5A5A5Au);
        else hipLaunchKernelGGL(ws_calib_copyoff_kernel<8>, dim3((u32)np), dim3(256), 0, st, a8, b, n, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_copyoff_kernel launch", e);
    }
    if (mode == 900 || mode == 901) {  // `blocks` = unused LDS bytes per block
        const u32 W = 2u;
        const u64 np = (n + 1023) / 1024, ppw = (np + W - 1) / W;
        const u32 dyn = blocks > 0 && blocks <= 65536 ? (u32)blocks : 0u;
        if (mode == 900) hipLaunchKernelGGL(ws_calib_2ph_kernel<0>, dim3((u32)(ppw * W)), dim3(256), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
        else hipLaunchKernelGGL(ws_calib_2ph_kernel<1>, dim3((u32)(ppw * W)), dim3(256), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_2ph_kernel launch", e);
    }
    if (mode >= 890 && mode <= 895) {  // 890/891: 512 x 2 (no sync / sync); 892/893: 256 x 4; 894/895: 1024 x 1
        const u32 W = 2u;
        const int T = mode < 892 ? 512 : (mode < 894 ? 256 : 1024), U = 16384 / (T * 16);
        const bool sy = mode & 1;
        const u64 per = (u64)T * U, np = (n + per - 1) / per, ppw = (np + W - 1) / W;
        const u32 dyn = blocks > 0 && blocks <= 65536 ? (u32)blocks : 0u;
        const dim3 g((u32)(ppw * W));
        if (T == 512) { if (sy) hipLaunchKernelGGL((ws_calib_blk_kernel<512, 2, true>), g, dim3(512), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
                        else hipLaunchKernelGGL((ws_calib_blk_kernel<512, 2, false>), g, dim3(512), dyn, st, a, n, W, ppw, 0x5A5A5A5Au); }
        else if (T == 256) { if (sy) hipLaunchKernelGGL((ws_calib_blk_kernel<256, 4, true>), g, dim3(256), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
                             else hipLaunchKernelGGL((ws_calib_blk_kernel<256, 4, false>), g, dim3(256), dyn, st, a, n, W, ppw, 0x5A5A5A5Au); }
        else { if (sy) hipLaunchKernelGGL((ws_calib_blk_kernel<1024, 1, true>), g, dim3(1024), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
               else hipLaunchKernelGGL((ws_calib_blk_kernel<1024, 1, false>), g, dim3(1024), dyn, st, a, n, W, ppw, 0x5A5A5A5Au); }
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_blk_kernel launch", e);
    }
    if (mode >= 880 && mode < 900) {  // 88U: U chunks per lane (1, 2, 4, 6, 8); `blocks` = unused LDS bytes per block
        const int U = mode - 880;
        const u32 W = 2u;
        const u64 per = 256ull * (U > 0 ? U : 4), np = (n + per - 1) / per, ppw = (np + W - 1) / W;
        const u32 dyn = blocks > 0 && blocks <= 65536 ? (u32)blocks : 0u;
        if (U == 1) hipLaunchKernelGGL(ws_calib_wcu_kernel<1>, dim3((u32)(ppw * W)), dim3(256), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
        else if (U == 2) hipLaunchKernelGGL(ws_calib_wcu_kernel<2>, dim3((u32)(ppw * W)), dim3(256), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
        else if (U == 8) hipLaunchKernelGGL(ws_calib_wcu_kernel<8>, dim3((u32)(ppw * W)), dim3(256), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
        else if (U == 6) hipLaunchKernelGGL(ws_calib_wcu_kernel<6>, dim3((u32)(ppw * W)), dim3(256), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
        else hipLaunchKernelGGL(ws_calib_wcu_kernel<4>, dim3((u32)(ppw * W)), dim3(256), dyn, st, a, n, W, ppw, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_wcu_kernel launch", e);
    }
    if (mode == 83) {  // `blocks` = number of windows; d_b: >= 18 MB (a zeroed table + items)
        const u32 W = blocks > 0 ? (u32)blocks : 2u;
        const u64 np = (n + 1023) / 1024, ppw = (np + W - 1) / W;
        const u32* tab = reinterpret_cast<const u32*>(d_b);
        const u32x4* items = reinterpret_cast<const u32x4*>(reinterpret_cast<unsigned char*>(d_b) + (2u << 20));
        hipLaunchKernelGGL(ws_calib_windows_dep_kernel, dim3((u32)(ppw * W)), dim3(256), 0, st, a, n, W, ppw, tab,
                           items, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_windows_dep_kernel launch", e);
    }
    if ((mode >= 73 && mode <= 75) || mode == 84 || mode == 85) {  // `blocks` = chunks per segment (<= 1280)
        const u32 segc = blocks > 0 && blocks <= 1280 ? (u32)blocks : 1032u;
        const u64 nseg = n / segc;
        const u32 half = nseg >= 512 ? (u32)((nseg + 1) / 2) : 0u;
        const u32 grid = half ? 2 * half : (u32)nseg;
        if (mode == 73) hipLaunchKernelGGL((ws_calib_seg_kernel<73, 5>), dim3(grid), dim3(256), 0, st, a, nseg, segc, half, 0x5A5A5A5Au);
        if (mode == 74) hipLaunchKernelGGL((ws_calib_seg_kernel<74, 5>), dim3(grid), dim3(256), 0, st, a, nseg, segc, half, 0x5A5A5A5Au);
        if (mode == 75) hipLaunchKernelGGL((ws_calib_seg_kernel<75, 5>), dim3(grid), dim3(256), 0, st, a, nseg, segc, half, 0x5A5A5A5Au);
        if (mode == 84) hipLaunchKernelGGL((ws_calib_seg_kernel<84, 5>), dim3(grid), dim3(256), 0, st, a, nseg, segc, half, 0x5A5A5A5Au);
        if (mode == 85) hipLaunchKernelGGL((ws_calib_seg_kernel<85, 5>), dim3(grid), dim3(256), 0, st, a, nseg, segc, half, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_seg_kernel launch", e);
    }
    if (mode == 86 || mode == 87) {  // `blocks` = chunks per segment (<= 1280: <= 6 pages)
        const u32 segc = blocks > 0 && blocks <= 1280 ? (u32)blocks : 1032u;
        const u64 nseg = n / segc;
        const u32 half = nseg >= 512 ? (u32)((nseg + 1) / 2) : 0u;
        const u32 grid = half ? 2 * half : (u32)nseg;
        if (mode == 86) hipLaunchKernelGGL(ws_calib_seg_pages_kernel<86>, dim3(grid), dim3(256), 0, st, a, nseg, segc, half, 0x5A5A5A5Au);
        else hipLaunchKernelGGL(ws_calib_seg_pages_kernel<87>, dim3(grid), dim3(256), 0, st, a, nseg, segc, half, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_seg_pages_kernel launch", e);
    }
    if (mode == 70 || mode == 71) {  // persistent; d_b's first 4 bytes are the ticket counter
        const u32 nb = blocks > 0 ? (u32)blocks : 2048u;
        u32* ctr = reinterpret_cast<u32*>(d_b);
        hipError_t e = hipMemsetAsync(ctr, 0, 4, st);
        if (e != hipSuccess) return ws_set_err("hipMemsetAsync(calib counter)", e);
        if (mode == 70) hipLaunchKernelGGL((ws_calib_persist_kernel<true>), dim3(nb), dim3(256), 0, st, a, n, ctr, 0x5A5A5A5Au);
        else hipLaunchKernelGGL((ws_calib_persist_kernel<false>), dim3(nb), dim3(256), 0, st, a, n, ctr, 0x5A5A5A5Au);
        e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_persist_kernel launch", e);
    }
    if (mode >= 60) {  // one-shot + dependent lookups (d_b must hold >= 16 MiB)
        switch (mode) {
        case 60: cal_dep<256, 4, 0>(a, b, n, st); break;
        case 61: cal_dep<256, 4, 1>(a, b, n, st); break;
        case 62: cal_dep<256, 4, 2>(a, b, n, st); break;
        case 63: cal_dep<256, 4, 4>(a, b, n, st); break;
        case 64: cal_dep<256, 8, 2>(a, b, n, st); break;
        case 65: cal_dep<512, 8, 2>(a, b, n, st); break;
        default: return ws_set_msg("websocketframeGpuCalibrate: unknown mode");
        }
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_dep_kernel launch", e);
    }
    if (mode >= 40) {  // LDS pipeline; n must be a multiple of the stage size (1024 chunks covers all)
        switch (mode) {
        case 40: cal_ldspipe<512, 6, 3>(a, n, blocks, st); break;
        case 41: cal_ldspipe<512, 8, 3>(a, n, blocks, st); break;
        case 42: cal_ldspipe<256, 12, 3>(a, n, blocks, st); break;
        case 43: cal_ldspipe<1024, 3, 3>(a, n, blocks, st); break;
        case 44: cal_ldspipe<512, 6, 1>(a, n, blocks, st); break;
        case 45: cal_ldspipe<512, 6, 7>(a, n, blocks, st); break;
        case 46: cal_ldspipe<256, 8, 3>(a, n, blocks, st); break;
        case 47: cal_ldspipe<512, 6, 3, true>(a, n, blocks, st); break;
        case 48: cal_ldspipe<256, 8, 3, true>(a, n, blocks, st); break;
        case 49: cal_ldspipe<1024, 3, 3, true>(a, n, blocks, st); break;
        default: return ws_set_msg("websocketframeGpuCalibrate: unknown mode");
        }
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_ldspipe_kernel launch", e);
    }
    if (mode >= 16) {
        unsigned char* a8 = reinterpret_cast<unsigned char*>(d_a);
        const u64 nb = n * 16;
        switch (mode) {
        case 16: cal_buf<256, 4, 2, 2>(a8, nb, st); break;
        case 17: cal_buf<256, 4, 0, 0>(a8, nb, st); break;
        case 18: cal_buf<256, 4, 2, 16>(a8, nb, st); break;
        case 19: cal_buf<256, 4, 2, 0>(a8, nb, st); break;
        case 20: cal_buf<256, 4, 0, 2>(a8, nb, st); break;
        case 21: cal_buf<256, 8, 2, 2>(a8, nb, st); break;
        case 22: cal_buf<512, 4, 2, 2>(a8, nb, st); break;
        case 23: cal_buf<1024, 4, 2, 2>(a8, nb, st); break;
        case 24: cal_buf<256, 2, 2, 2>(a8, nb, st); break;
        case 25: cal_buf<256, 16, 2, 2>(a8, nb, st); break;
        case 26: cal_buf<256, 4, 3, 3>(a8, nb, st); break;
        case 27: cal_buf<256, 4, 2, 18>(a8, nb, st); break;
        case 28: cal_buf<128, 4, 2, 2>(a8, nb, st); break;
        case 29: cal_buf<64, 4, 2, 2>(a8, nb, st); break;
        case 30: cal_buf<256, 4, 18, 18>(a8, nb, st); break;   // sc1|nt loads, sc1|nt stores
        case 31: cal_buf<256, 4, 3, 18>(a8, nb, st); break;    // sc0|nt loads, sc1|nt stores
        case 32: cal_buf<256, 4, 19, 18>(a8, nb, st); break;   // sc0|sc1|nt loads, sc1|nt stores
        case 33: cal_buf<256, 4, 16, 18>(a8, nb, st); break;   // sc1 loads, sc1|nt stores
        case 34: cal_buf<256, 4, 2, 19>(a8, nb, st); break;    // nt loads, sc0|sc1|nt stores
        default: return ws_set_msg("websocketframeGpuCalibrate: unknown mode");
        }
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_buf_kernel launch", e);
    }
    if (mode >= 5 && mode <= 8) {
        const int K = mode == 5 ? 1 : (mode == 6 ? 2 : (mode == 7 ? 4 : 16));
        const u32 nb = (u32)((n + 1024ull * K - 1) / (1024ull * K));
        if (K == 1) hipLaunchKernelGGL((ws_calib_rounds_kernel<1, 1>), dim3(nb), dim3(256), 0, st, a, n, 0x5A5A5A5Au);
        if (K == 2) hipLaunchKernelGGL((ws_calib_rounds_kernel<1, 2>), dim3(nb), dim3(256), 0, st, a, n, 0x5A5A5A5Au);
        if (K == 4) hipLaunchKernelGGL((ws_calib_rounds_kernel<1, 4>), dim3(nb), dim3(256), 0, st, a, n, 0x5A5A5A5Au);
        if (K == 16) hipLaunchKernelGGL((ws_calib_rounds_kernel<1, 16>), dim3(nb), dim3(256), 0, st, a, n, 0x5A5A5A5Au);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : ws_set_err("ws_calib_rounds_kernel launch", e);
    }
#define WS_CAL(NTV, M) hipLaunchKernelGGL((ws_calib_kernel<NTV, M>), dim3(blocks), dim3(256), 0, st, a, b, n, 0x5A5A5A5Au, sink)
    if (nt) { if (mode == 0) WS_CAL(1, 0); else if (mode == 1) WS_CAL(1, 1); else WS_CAL(1, 2); }
    else { if (mode == 0) WS_CAL(0, 0); else if (mode == 1) WS_CAL(0, 1); else WS_CAL(0, 2); }
#undef WS_CAL
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ws_set_err("ws_calib_kernel launch", e);
}
