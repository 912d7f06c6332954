// tools/exp_k1k2.hip — experiment only (not part of the drop-in): why does K2 stream faster
// right behind K1 than alone or than any plain in-place XOR of its shape? Linked against
// the product's objects (internal launchers), built by tools/exp_k1k2.sh into
// tools/libexp_k1k2.so. Sequences, each `iters` times on `stream` (after one K1 that leaves
// the workspace in place):
//   0  K1 + K2 (the product's classic step)
//   1  K2 alone (the same items again)
//   2  spin kernel (`arg` us, one block, no memory traffic) + K2
//   3  header-line touch (32 B at every frame start, like K1's loads, no stores) + K2
//   4  mid-frame touch (32 B at every frame start + arg bytes: lines K2 reads too) + K2
//   5  touch of lines in another buffer (same count, not read by K2) + K2
//   6  header-line touch alone      7  K1 alone      8  spin alone
//   9  K1 with the first-step stride guess `arg` + K2      10  that K1 alone
//   13 K1 + plain XOR of `arg` MiB of another buffer + K2   14 read the workspace (items, pointers) + K2
//   15 K1 twice + K2
//   11 latency-bound chase kernel (arg % 1000 x 10 us; 256 blocks if arg > 1000, else 1) + K2   12 it alone
//   20-23 a pass of arg MiB over another buffer + K2 (20 nt XOR, 21 plain write-only, 22 nt
//   write-only, 23 plain read-only); 30-33 the same pass alone
//   40 K1 variant `arg` alone, 41 it + K2 (round 5 breakdown; the library must be built with
//   tools/exp_k1k2.sh, which compiles ws_piece.hip with WS_K1_VARIANTS): arg = store bitmask
//   (1 descriptors, 2 items, 4 piece pointers, 8 segment records; 16 = all stores at 8 waves/SIMD),
//   first step guessing the stride `stride` (the product's hinted call)
#include "../util_amd/csrc/ws_common.h"
int ws_launch_piece_scan_variant(const WsLaunch& L, u64 lo, u64 hi, unsigned char* ws, u32 gen, u32 g0, int st,
                                 PieceWs* out);

__global__ void exp_spin_kernel(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

// one block of 256 threads: dependent random loads over the buffer until `ticks` (100 MHz)
// have passed (a latency-bound, low-activity kernel like the raw stream's walks)
__global__ __launch_bounds__(256) void exp_chase_kernel(const u32* __restrict__ a, unsigned long long n4,
                                                       unsigned long long ticks, u32* sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    u32 x = threadIdx.x * 2654435761u;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        const unsigned long long i = ((unsigned long long)(x * 2654435761u) * 64ull) % n4;
        x += a[i] | 1u;
    }
    if (x == 0x12345678u) *gptr<u32>(sink) = x;
}

// in-place XOR of n16 16-B chunks (a plain stream that evicts the caches)
__global__ __launch_bounds__(256) void exp_xor_kernel(gu32x4* __restrict__ a, unsigned long long n16) {
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n16;
         i += (unsigned long long)gridDim.x * 256) {
        u32x4 v = a[i];
        v.x ^= 0x5A5A5A5Au; v.y ^= 0x5A5A5A5Au; v.z ^= 0x5A5A5A5Au; v.w ^= 0x5A5A5A5Au;
        a[i] = v;
    }
}

// passes over n16 16-B chunks of another buffer, by cache policy (round 4: what in a pass in
// front of K2 makes it fast): 0 nt XOR (nt loads + nt stores), 1 plain write-only, 2 nt
// write-only, 3 plain read-only
template <int KIND>
__global__ __launch_bounds__(256) void exp_pass_kernel(gu32x4* __restrict__ a, unsigned long long n16, u32* sink) {
    u32 h = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n16;
         i += (unsigned long long)gridDim.x * 256) {
        if (KIND == 0) {
            u32x4 v = __builtin_nontemporal_load(a + i);
            v.x ^= 0x5A5A5A5Au; v.y ^= 0x5A5A5A5Au; v.z ^= 0x5A5A5A5Au; v.w ^= 0x5A5A5A5Au;
            __builtin_nontemporal_store(v, a + i);
        } else if (KIND == 1) {
            const u32x4 v = {(u32)i, 1u, 2u, 3u};
            a[i] = v;
        } else if (KIND == 2) {
            const u32x4 v = {(u32)i, 1u, 2u, 3u};
            __builtin_nontemporal_store(v, a + i);
        } else {
            const u32x4 v = a[i];
            h ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (KIND == 3 && h == 0xA5A5F00Du) *gptr<u32>(sink) = h;
}

// read every 16-B entry of [p, p + n16) (the items / piece pointers K2 will read)
__global__ __launch_bounds__(256) void exp_read_kernel(const gu32x4* __restrict__ a, unsigned long long n16, u32* sink) {
    u32 h = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n16;
         i += (unsigned long long)gridDim.x * 256) {
        const u32x4 v = a[i];
        h ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (h == 0xA5A5F00Du) *gptr<u32>(sink) = h;
}

// every CU busy with ALU work (FMA chains) until `ticks` (100 MHz) have passed: no memory traffic
__global__ __launch_bounds__(256) void exp_alu_kernel(unsigned long long ticks, u32* sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
#pragma unroll
        for (int i = 0; i < 64; ++i) a = __builtin_fmaf(a, b, 1e-7f);
    }
    if (a == 12345.f) *gptr<u32>(sink) = 1;
}

// thread i loads 32 B at base + i*stride + off (clamped to n); the sum never matches the
// run-time key, so nothing is stored, but the loads cannot be removed
__global__ __launch_bounds__(256) void exp_touch_kernel(const unsigned char* __restrict__ base, unsigned long long n,
                                                       unsigned long long count, unsigned long long stride,
                                                       unsigned long long off, u32 key, u32* sink) {
    const unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    unsigned long long a = i * stride + off;
    if (a + 32 > n) a = n - 32;
    const gu32x4* q = reinterpret_cast<const gu32x4*>(reinterpret_cast<uintptr_t>(base + a) & ~(uintptr_t)15);
    const u32x4 x0 = q[0], x1 = q[1];
    const u32 h = x0.x ^ x0.y ^ x0.z ^ x0.w ^ x1.x ^ x1.y ^ x1.z ^ x1.w;
    if (h == key) *gptr<u32>(sink) = h;
}

extern "C" __attribute__((visibility("default"))) int exp_k1k2_run(
    unsigned char* buf, unsigned long long buflen, const u64* seg_off, const u64* seg_len, unsigned int nseg,
    unsigned int max_frames, WebsocketFrameDesc_t* desc, WebsocketSegResult_t* res, unsigned char* other,
    unsigned long long other_len, unsigned long long nframes, unsigned long long stride, int mode, int iters,
    long long arg, void* hip_stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    static unsigned char* ws = nullptr;
    static size_t ws_bytes = 0;
    static u32* sink = nullptr;
    const size_t need = ws_piece_workspace_bytes(buflen, nseg, max_frames);
    if (ws_bytes < need) {
        if (ws) (void)hipFree(ws);
        if (hipMalloc(&ws, need) != hipSuccess) return -2;
        (void)hipMemset(ws, 0, need);
        ws_bytes = need;
    }
    if (!sink && hipMalloc(&sink, 64) != hipSuccess) return -2;
    int cus = 256, lds = 160 * 1024;
    WsLaunch L;
    L.buf = buf; L.seg_off = seg_off; L.seg_len = seg_len; L.nseg = nseg; L.max_frames = max_frames;
    L.desc_base = nullptr; L.desc = desc; L.res = res; L.stream = st; L.cus = cus; L.lds_per_cu = lds;
    static u32 gen = 100;
    PieceWs P;
    int rc = ws_launch_piece_scan(L, 0, buflen, ws, ++gen, &P);
    if (rc) return rc;
    const u32 tb = (u32)((nframes + 255) / 256);
    const unsigned long long spin = (unsigned long long)(arg > 0 ? arg : 40) * 100;   // 100 MHz counter
    for (int it = 0; it < iters; ++it) {
        switch (mode) {
        case 0: if ((rc = ws_launch_piece_scan(L, 0, buflen, ws, gen, &P))) return rc; break;
        case 2: case 8: hipLaunchKernelGGL(exp_spin_kernel, dim3(1), dim3(64), 0, st, spin); break;
        case 3: case 6:
            hipLaunchKernelGGL(exp_touch_kernel, dim3(tb), dim3(256), 0, st, buf, buflen, nframes, stride, 0ull,
                               0xA5A5F00Du, sink);
            break;
        case 4:
            hipLaunchKernelGGL(exp_touch_kernel, dim3(tb), dim3(256), 0, st, buf, buflen, nframes, stride,
                               (unsigned long long)arg, 0xA5A5F00Du, sink);
            break;
        case 5:
            hipLaunchKernelGGL(exp_touch_kernel, dim3(tb), dim3(256), 0, st, other, other_len, nframes, stride, 0ull,
                               0xA5A5F00Du, sink);
            break;
        case 7: if ((rc = ws_launch_piece_scan(L, 0, buflen, ws, gen, &P))) return rc; break;
        case 11: case 12:
            hipLaunchKernelGGL(exp_chase_kernel, dim3(arg > 1000 ? 256 : 1), dim3(256), 0, st,
                               reinterpret_cast<const u32*>(buf), buflen / 4, (unsigned long long)(arg % 1000) * 100 * 10,
                               sink);
            break;
        case 16: case 17:                       // the whole GPU ALU-busy for arg us (+ K2 for 16)
            hipLaunchKernelGGL(exp_alu_kernel, dim3(2048), dim3(256), 0, st, (unsigned long long)arg * 100, sink);
            break;
        case 18: case 19:                       // a plain XOR of arg MiB of `other` (+ K2 for 18)
            hipLaunchKernelGGL(exp_xor_kernel, dim3(4096), dim3(256), 0, st,
                               reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(other)),
                               (unsigned long long)arg << 16);
            break;
        case 13:                                // K1, then a plain XOR of arg MiB of `other`, then K2
            if ((rc = ws_launch_piece_scan(L, 0, buflen, ws, gen, &P))) return rc;
            hipLaunchKernelGGL(exp_xor_kernel, dim3(4096), dim3(256), 0, st,
                               reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(other)),
                               (unsigned long long)arg << 16);
            break;
        case 14:                                // read the items + piece pointers, then K2
            hipLaunchKernelGGL(exp_read_kernel, dim3(2048), dim3(256), 0, st,
                               reinterpret_cast<const gu32x4*>(reinterpret_cast<uintptr_t>(ws)),
                               (unsigned long long)(need / 16), sink);
            break;
        case 15:                                // K1 twice, then K2
            if ((rc = ws_launch_piece_scan(L, 0, buflen, ws, gen, &P))) return rc;
            if ((rc = ws_launch_piece_scan(L, 0, buflen, ws, gen, &P))) return rc;
            break;
        case 9: case 10: if ((rc = ws_launch_piece_scan(L, 0, buflen, ws, gen, &P, false, (u32)arg))) return rc; break;
        case 40: case 41:
            if ((rc = ws_launch_piece_scan_variant(L, 0, buflen, ws, gen, (u32)stride, (int)arg, &P))) return rc;
            break;
        case 20: case 30: case 21: case 31: case 22: case 32: case 23: case 33: {   // pass of arg MiB (+ K2 for 2x)
            gu32x4* o = reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(other));
            const unsigned long long n16 = (unsigned long long)arg << 16;
            const int kind = mode % 10;
            if (kind == 0) hipLaunchKernelGGL(exp_pass_kernel<0>, dim3(4096), dim3(256), 0, st, o, n16, sink);
            if (kind == 1) hipLaunchKernelGGL(exp_pass_kernel<1>, dim3(4096), dim3(256), 0, st, o, n16, sink);
            if (kind == 2) hipLaunchKernelGGL(exp_pass_kernel<2>, dim3(4096), dim3(256), 0, st, o, n16, sink);
            if (kind == 3) hipLaunchKernelGGL(exp_pass_kernel<3>, dim3(4096), dim3(256), 0, st, o, n16, sink);
            break;
        }
        default: break;
        }
        if ((mode <= 5 || mode == 9 || mode == 11 || (mode >= 13 && mode <= 16) || mode == 18 || (mode >= 20 && mode <= 23) || mode == 41) &&
            (rc = ws_launch_piece_unmask(L, P, gen)))
            return rc;
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// The raw-stream path's K2 again on the workspace the stream call just left (same items,
// pointers and segment pair): `iters` K2 launches after one websocketframeStreamDecodeDevice
// call (mode 0), or that call alone `iters` times (mode 1). Isolates the stream K2's
// +6 % over the batch K2 on cfg3: context (what runs before it) or inputs (what it reads).
// thread i loads 32 B at base + offs[i] (the frame starts: what K1's header loads touch)
__global__ __launch_bounds__(256) void exp_touch_idx_kernel(const unsigned char* __restrict__ base,
                                                           const unsigned long long* __restrict__ offs,
                                                           unsigned long long count, u32 key, u32* sink) {
    const unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const gu32x4* q = reinterpret_cast<const gu32x4*>(reinterpret_cast<uintptr_t>(base + offs[i]) & ~(uintptr_t)15);
    const u32x4 x0 = q[0], x1 = q[1];
    const u32 h = x0.x ^ x0.y ^ x0.z ^ x0.w ^ x1.x ^ x1.y ^ x1.z ^ x1.w;
    if (h == key) *gptr<u32>(sink) = h;
}

extern "C" int websocketframeStreamDecodeDevice(unsigned char* d_buf, unsigned long long len, unsigned int max_frames,
                                                WebsocketFrameDesc_t* d_desc, WebsocketSegResult_t* d_res,
                                                void* hip_stream);
extern "C" __attribute__((visibility("default"))) int exp_stream_k2(unsigned char* buf, unsigned long long len,
                                                                   unsigned int max_frames, WebsocketFrameDesc_t* desc,
                                                                   WebsocketSegResult_t* res, int mode, int iters,
                                                                   const unsigned long long* frame_off,
                                                                   unsigned long long nframes, void* hip_stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    if (mode == 1) {
        for (int i = 0; i < iters; ++i) {
            const int rc = websocketframeStreamDecodeDevice(buf, len, max_frames, desc, res, hip_stream);
            if (rc) return rc;
        }
        return 0;
    }
    int rc = websocketframeStreamDecodeDevice(buf, len, max_frames, desc, res, hip_stream);
    if (rc) return rc;
    const size_t pws = ws_piece_workspace_bytes(len, 1, max_frames);
    void* ws = nullptr;
    WsSlot slot;
    if ((rc = slot.acquire(st)) || (rc = slot.workspace(pws + 64, 16, &ws))) return rc;
    unsigned char* w8 = reinterpret_cast<unsigned char*>(ws);
    u64* d_seg = reinterpret_cast<u64*>(w8 + ((pws + 15) & ~(size_t)15));
    WsLaunch L;
    L.buf = buf; L.seg_off = d_seg; L.seg_len = d_seg + 1; L.nseg = 1; L.max_frames = max_frames;
    L.desc_base = nullptr; L.desc = desc; L.res = res; L.stream = st;
    L.cus = slot.cus; L.lds_per_cu = slot.lds;
    PieceWs Pw;
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    Pw.npieces = len + lead0 ? ((len + lead0 - 1) >> WS_PIECE_SHIFT) + 1 : 0;
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
    static u32* sink = nullptr;
    if (!sink && hipMalloc(&sink, 64) != hipSuccess) return -2;
    for (int i = 0; i < iters; ++i) {
        if (mode == 2)                          // the frame starts touched first (K1's header lines)
            hipLaunchKernelGGL(exp_touch_idx_kernel, dim3((u32)((nframes + 255) / 256)), dim3(256), 0, st, buf,
                               frame_off, nframes, 0xA5A5F00Du, sink);
        if ((rc = ws_launch_piece_unmask(L, Pw, 0x7FFFFFF1u))) return rc;
    }
    return 0;
}

// batch: K1 once, then (frame-start touch + K2) x iters
extern "C" __attribute__((visibility("default"))) int exp_batch_touch_k2(
    unsigned char* buf, unsigned long long buflen, const u64* seg_off, const u64* seg_len, unsigned int nseg,
    unsigned int max_frames, WebsocketFrameDesc_t* desc, WebsocketSegResult_t* res,
    const unsigned long long* frame_off, unsigned long long nframes, int iters, void* hip_stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    static unsigned char* ws = nullptr;
    static size_t ws_bytes = 0;
    static u32* sink = nullptr;
    const size_t need = ws_piece_workspace_bytes(buflen, nseg, max_frames);
    if (ws_bytes < need) {
        if (ws) (void)hipFree(ws);
        if (hipMalloc(&ws, need) != hipSuccess) return -2;
        (void)hipMemset(ws, 0, need);
        ws_bytes = need;
    }
    if (!sink && hipMalloc(&sink, 64) != hipSuccess) return -2;
    WsLaunch L;
    L.buf = buf; L.seg_off = seg_off; L.seg_len = seg_len; L.nseg = nseg; L.max_frames = max_frames;
    L.desc_base = nullptr; L.desc = desc; L.res = res; L.stream = st; L.cus = 256; L.lds_per_cu = 160 * 1024;
    PieceWs P;
    int rc = ws_launch_piece_scan(L, 0, buflen, ws, 77, &P);
    if (rc) return rc;
    for (int i = 0; i < iters; ++i) {
        hipLaunchKernelGGL(exp_touch_idx_kernel, dim3((u32)((nframes + 255) / 256)), dim3(256), 0, st, buf, frame_off,
                           nframes, 0xA5A5F00Du, sink);
        if ((rc = ws_launch_piece_unmask(L, P, 77))) return rc;
    }
    return 0;
}

// the raw-stream call once, then `iters` x (the BATCH K1 over the same wire with the batch's
// own segments and workspace + the stream's K2 on the stream's workspace): does any K1 in
// front speed up the stream's K2, or only the K1 whose items it reads?
extern "C" __attribute__((visibility("default"))) int exp_stream_batchk1_k2(
    unsigned char* buf, unsigned long long len, unsigned int max_frames, WebsocketFrameDesc_t* desc,
    WebsocketSegResult_t* res, const u64* seg_off, const u64* seg_len, unsigned int nseg, unsigned int fps,
    WebsocketFrameDesc_t* bdesc, WebsocketSegResult_t* bres, int iters, int with_k1, void* hip_stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    int rc = websocketframeStreamDecodeDevice(buf, len, max_frames, desc, res, hip_stream);
    if (rc) return rc;
    const size_t pws = ws_piece_workspace_bytes(len, 1, max_frames);
    void* ws = nullptr;
    WsSlot slot;
    if ((rc = slot.acquire(st)) || (rc = slot.workspace(pws + 64, 16, &ws))) return rc;
    unsigned char* w8 = reinterpret_cast<unsigned char*>(ws);
    u64* d_seg = reinterpret_cast<u64*>(w8 + ((pws + 15) & ~(size_t)15));
    WsLaunch L;
    L.buf = buf; L.seg_off = d_seg; L.seg_len = d_seg + 1; L.nseg = 1; L.max_frames = max_frames;
    L.desc_base = nullptr; L.desc = desc; L.res = res; L.stream = st;
    L.cus = slot.cus; L.lds_per_cu = slot.lds;
    PieceWs Pw;
    const u64 lead0 = reinterpret_cast<uintptr_t>(buf) & 15;
    Pw.npieces = len + lead0 ? ((len + lead0 - 1) >> WS_PIECE_SHIFT) + 1 : 0;
    Pw.pbase = 0; Pw.c_lo = 0; Pw.c_hi = (len + lead0 + 15) >> 4;
    Pw.disorder = reinterpret_cast<u32*>(w8);
    Pw.nonuni = reinterpret_cast<u32*>(w8) + 1;
    Pw.ptr = reinterpret_cast<u64*>(w8 + 16);
    size_t b = (16 + Pw.npieces * 8 + 15) & ~(size_t)15;
    Pw.nwork = reinterpret_cast<u32*>(w8 + b);
    b = (b + 4 + 15) & ~(size_t)15;
    Pw.items = reinterpret_cast<u32x4*>(w8 + b);
    static unsigned char* bws = nullptr;
    static size_t bws_bytes = 0;
    const size_t need = ws_piece_workspace_bytes(len, nseg, fps);
    if (bws_bytes < need) {
        if (bws) (void)hipFree(bws);
        if (hipMalloc(&bws, need) != hipSuccess) return -2;
        (void)hipMemset(bws, 0, need);
        bws_bytes = need;
    }
    WsLaunch LB = L;
    LB.seg_off = seg_off; LB.seg_len = seg_len; LB.nseg = nseg; LB.max_frames = fps; LB.desc = bdesc; LB.res = bres;
    PieceWs PB;
    for (int i = 0; i < iters; ++i) {
        if (with_k1 && (rc = ws_launch_piece_scan(LB, 0, len, bws, 99, &PB))) return rc;
        if ((rc = ws_launch_piece_unmask(L, Pw, 0x7FFFFFF1u))) return rc;
    }
    return 0;
}
