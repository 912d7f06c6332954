// ws_api.hip — C ABI of the batch decode (include/wsframe_amd.h Part 2):
// argument checks, per-device workspace, variant dispatch (host-buffer path:
// ws_hostpath.hip).
//
// Default path 3 = ws_piece.hip (walk kernel + one-shot unmask over 16 KiB pieces;
// fastest measured); path 4 = ws_segfuse.hip (one workgroup per segment,
// auto for many small segments); path 1 "walker" = ws_walker.hip (one wave walks and
// unmasks one segment; also the gated fallback of path 3 for unordered segments).
//
// Options (websocketframeGpuSetOption) are std::atomic: a call reads each knob once
// (WsTuning snapshot below) and concurrent SetOption calls never race with a launch.
// Every option value yields bit-identical results; only the speed differs.
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <deque>
#include <mutex>

#include "ws_common.h"

static __thread char g_last_error[256];
extern std::atomic<size_t> ws_host_chunk_bytes;
extern WsOpt ws_piece_scan;
extern WsOpt ws_reasm_path;
extern WsOpt ws_reasm_cfg;
extern WsOpt ws_segfuse_cfg;
extern WsOpt ws_enc_lds;
extern WsOpt ws_encode_side;
extern WsOpt ws_encode_fused;
extern WsOpt ws_piece_whole;
extern WsOpt ws_piece_occ;
extern WsOpt ws_piece_lds;
extern WsOpt ws_piece_win;
extern WsOpt ws_piece_wbit;
extern WsOpt ws_k2_timing;
void ws_k2_timing_reset();
int ws_k2_stat(unsigned long long* ns, unsigned long long* calls);
extern WsOpt ws_scan_win;
extern WsOpt ws_piece_wn;
extern WsOpt ws_enc_win;
extern WsOpt ws_enc_front;
extern WsOpt ws_seg_lds;
WsOpt ws_seg_win{1};      // "seg_win": segfuse and fused reassembly take segments in two windows (ws_win2)
extern WsOpt ws_reasm_merge;
extern WsOpt ws_stream_rw, ws_stream_rw_cmax, ws_stream_rounds;
extern std::atomic<unsigned long long> ws_stat_rw_chunks, ws_stat_rw_chunk_walks;

int ws_set_err(const char* what, hipError_t e) {
    snprintf(g_last_error, sizeof(g_last_error), "%s: %s", what, hipGetErrorString(e));
    return -(int)(e ? e : 1);
}

int ws_set_msg(const char* msg) {
    snprintf(g_last_error, sizeof(g_last_error), "%s", msg);
    return -1;
}

extern "C" WSFRAME_AMD_EXPORT const char* websocketframeGpuLastError(void) { return g_last_error; }

// ---------------------------------------------------------------------------------------------
// launch configuration (tunable for in-process A/B by bench/profiling tools)

struct WsTuning {
    int path = -1;          // -1 auto (4 for many small segments, else 3), 1: walker (one wave per segment),
                            // 3: walk + one-shot 16 KiB pieces (ws_piece), 4: one workgroup per segment,
                            // walk + unmask fused (ws_segfuse)
    int nt = 1;             // 0 plain, 1 nontemporal loads+stores, 2 nontemporal stores only
    int dyn = 0;            // walker: 1 dynamic segment dequeue, 0 static grid-stride
    int unroll = 4;         // walker: 16-B chunks per lane per batch
    int blocks_per_cu = 64; // walker: grid cap in blocks per CU (64: one segment per wave)
};
static WsOpt g_path{-1}, g_nt{1}, g_dyn{0}, g_unroll{4}, g_bpc{64};
static WsTuning tuning() {                        // one consistent read per call
    WsTuning t;
    t.path = g_path; t.nt = g_nt; t.dyn = g_dyn; t.unroll = g_unroll; t.blocks_per_cu = g_bpc;
    return t;
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeGpuSetOption(const char* name, long long value) {
    if (!strcmp(name, "path")) {
        if (value != -1 && value != 1 && value != 3 && value != 4) return -1;
        g_path = (int)value;
    }
    else if (!strcmp(name, "nt")) g_nt = (int)value;
    else if (!strcmp(name, "dyn")) g_dyn = (int)value;
    else if (!strcmp(name, "unroll")) {
        if (value != 2 && value != 4 && value != 8) return -1;
        g_unroll = (int)value;
    }
    else if (!strcmp(name, "blocks_per_cu")) g_bpc = (int)value;
    else if (!strcmp(name, "host_chunk_mb") && value > 0) ws_host_chunk_bytes = (size_t)value << 20;
    else if (!strcmp(name, "piece_scan")) ws_piece_scan = (int)value;
    else if (!strcmp(name, "reasm_path")) ws_reasm_path = (int)value;
    else if (!strcmp(name, "reasm_cfg")) ws_reasm_cfg = (int)value;
    else if (!strcmp(name, "segfuse_cfg")) ws_segfuse_cfg = (int)value;
    else if (!strcmp(name, "encode_side")) ws_encode_side = (int)value;
    else if (!strcmp(name, "encode_fused")) ws_encode_fused = (int)value;
    else if (!strcmp(name, "piece_whole")) ws_piece_whole = (int)value;
    else if (!strcmp(name, "piece_occ")) ws_piece_occ = (int)value;
    else if (!strcmp(name, "piece_lds")) ws_piece_lds = (int)value;
    else if (!strcmp(name, "piece_win")) ws_piece_win = (int)value;
    else if (!strcmp(name, "seg_win")) ws_seg_win = (int)value;
    else if (!strcmp(name, "seg_lds")) ws_seg_lds = (int)value;
    else if (!strcmp(name, "piece_wbit")) ws_piece_wbit = (int)value;
    else if (!strcmp(name, "scan_win")) ws_scan_win = (int)value;
    else if (!strcmp(name, "piece_wn")) ws_piece_wn = (int)value;
    else if (!strcmp(name, "enc_win")) ws_enc_win = (int)value;
    else if (!strcmp(name, "enc_lds")) ws_enc_lds = (int)value;
    else if (!strcmp(name, "enc_front")) ws_enc_front = (int)value;
    else if (!strcmp(name, "k2_timing")) {
        ws_k2_timing = (int)value;
        ws_k2_timing_reset();
    }
    else if (!strcmp(name, "reasm_merge")) ws_reasm_merge = (int)value;
    else if (!strcmp(name, "stream_rw")) ws_stream_rw = (int)value;
    else if (!strcmp(name, "stream_rw_cmax")) ws_stream_rw_cmax = (int)value;
    else if (!strcmp(name, "stream_rounds")) ws_stream_rounds = (int)value;
    else return -1;
    return 0;
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeGpuGetStat(const char* name, unsigned long long* value) {
    if (!value) return -1;
    unsigned long long ns = 0, calls = 0;
    if (!strcmp(name, "k2_ns") || !strcmp(name, "k2_calls")) {
        if (ws_k2_stat(&ns, &calls)) return -1;
        *value = name[3] == 'n' ? ns : calls;
        return 0;
    }
    if (!strcmp(name, "stream_rw_chunks")) *value = ws_stat_rw_chunks.load();
    else if (!strcmp(name, "stream_rw_chunk_walks")) *value = ws_stat_rw_chunk_walks.load();
    else return -1;
    return 0;
}

// ---------------------------------------------------------------------------------------------
// Per-device state: CU count, the walker's dequeue-counter ring, and one workspace set
// (decode + encode) per HIP stream, grown on demand. Calls on different streams of one
// device may overlap in time (a reactor with several rx batches in flight, one stream
// each); calls on one stream are ordered by the stream (slot rules: stream_slot).
#define WS_MAX_DEV 64
#define WS_CTR_RING 64
#define WS_STREAM_SLOTS 16
struct WsStreamWs {
    hipStream_t stream = nullptr;
    unsigned long long capture = 0; // capture id of the graph this slot belongs to (0: eager calls)
    bool captured = false;         // belongs to a graph capture: never reassigned, never given to eager calls
    unsigned long long last = 0;   // LRU tick
    u32* ws = nullptr;             // decode / reassembly / stream workspace
    size_t ws_bytes = 0;
    void* ews = nullptr;           // encode workspace (scan temp + piece pointers)
    size_t ews_bytes = 0;
    void* aws = nullptr;           // auxiliary device scratch (the stream path's chunk-parallel walk)
    size_t aws_bytes = 0;
    void* hws = nullptr;           // ... and its pinned host copy
    void* hws_dev = nullptr;       // (its device address)
    size_t hws_bytes = 0;
    bool aux_state_ok = false;     // the stream path's state (aux head) rests at zero
};
struct WsDevState {
    int init = 0;
    int cus = 0;
    u32* ctr = nullptr;
    std::atomic<unsigned> slot{0};
    std::deque<WsStreamWs> sw;     // grows; stable addresses
    unsigned long long tick = 0;
};
static WsDevState g_dev[WS_MAX_DEV];
static std::mutex g_dev_mu;        // device init and the stream-slot table

static int dev_state(WsDevState** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return ws_set_err("hipGetDevice", e);
    if (dev < 0 || dev >= WS_MAX_DEV) return ws_set_err("device index", hipErrorInvalidDevice);
    WsDevState& st = g_dev[dev];
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (!st.init) {
        hipDeviceProp_t prop;
        if ((e = hipGetDeviceProperties(&prop, dev)) != hipSuccess) return ws_set_err("hipGetDeviceProperties", e);
        st.cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
        // the first call may come while the thread's stream captures a graph: allocate in
        // relaxed mode and clear on a private non-blocking stream (neither is part of the graph)
        hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
        (void)hipThreadExchangeStreamCaptureMode(&mode);
        hipStream_t ps = nullptr;
        e = hipMalloc(&st.ctr, WS_CTR_RING * 128);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipMemsetAsync(st.ctr, 0, WS_CTR_RING * 128, ps);
        if (e == hipSuccess) e = hipStreamSynchronize(ps);
        if (ps) (void)hipStreamDestroy(ps);
        (void)hipThreadExchangeStreamCaptureMode(&mode);
        if (e != hipSuccess) return ws_set_err("counters", e);
        st.init = 1;
    }
    *out = &st;
    return 0;
}

static bool capturing(hipStream_t stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(stream, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
}

// the id of the capture the stream is in (0: not capturing)
static unsigned long long capture_id(hipStream_t stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    if (hipStreamGetCaptureInfo(stream, &st, &id) != hipSuccess || st != hipStreamCaptureStatusActive) return 0;
    return id ? id : ~0ull;
}

// the workspace slot of (stream, capture) (caller holds g_dev_mu). Eager calls keep at most
// WS_STREAM_SLOTS slots: a further stream takes the least recently used one after a device
// synchronize. Every graph capture gets slots of its own, keyed by its capture id (torch
// captures every graph on one shared stream, so the stream alone does not tell graphs apart):
// its graph uses that workspace on every replay, so it is never handed to another capture or
// to an eager call, and graphs captured separately may be replayed concurrently.
static int stream_slot(WsDevState* ds, hipStream_t stream, WsStreamWs** out) {
    const unsigned long long cap = capture_id(stream);
    WsStreamWs* lru = nullptr;
    for (WsStreamWs& w : ds->sw) {
        if (w.stream == stream && w.capture == cap) {
            w.last = ++ds->tick;
            *out = &w;
            return 0;
        }
        if (!w.captured && (!lru || w.last < lru->last)) lru = &w;
    }
    if (cap || ds->sw.size() < WS_STREAM_SLOTS || !lru) {
        ds->sw.emplace_back();
        lru = &ds->sw.back();
        lru->captured = cap != 0;
    } else {                       // every slot taken by another stream: drain the device, then reuse
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) return ws_set_err("hipDeviceSynchronize", e);
    }
    lru->stream = stream;
    lru->capture = cap;
    lru->last = ++ds->tick;
    *out = lru;
    return 0;
}

// grow *p to at least `bytes` (the stream's previous work may still read it: drain first).
// A stream capturing a graph (e.g. torch's private capture stream) may get its first
// allocation (hipMalloc in relaxed capture mode, the head zeroed by a captured memset)
// but cannot drain and free an existing one.
static int grow(void** p, size_t* have, size_t bytes, hipStream_t stream, size_t zero_bytes, const char* what) {
    if (*have >= bytes) return 0;
    hipError_t e;
    const bool cap = capturing(stream);
    if (*p) {
        if (cap) return ws_set_msg("workspace must grow while the stream captures a graph: "
                                   "make one call of this size on the stream before capturing");
        if ((e = hipStreamSynchronize(stream)) != hipSuccess) return ws_set_err("hipStreamSynchronize", e);
        (void)hipFree(*p);
        *p = nullptr;
        *have = 0;
    }
    const size_t sz = bytes + bytes / 4 + 4096;
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    if (cap) (void)hipThreadExchangeStreamCaptureMode(&mode);
    e = hipMalloc(p, sz);
    if (cap) (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (e != hipSuccess) return ws_set_err(what, e);
    if (zero_bytes && cap) {
        // not part of the graph: cleared once, on a private stream, in relaxed mode
        hipStream_t ps = nullptr;
        hipStreamCaptureMode m2 = hipStreamCaptureModeRelaxed;
        (void)hipThreadExchangeStreamCaptureMode(&m2);
        e = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipMemsetAsync(*p, 0, zero_bytes < sz ? zero_bytes : sz, ps);
        if (e == hipSuccess) e = hipStreamSynchronize(ps);
        if (ps) (void)hipStreamDestroy(ps);
        (void)hipThreadExchangeStreamCaptureMode(&m2);
        if (e != hipSuccess) return ws_set_err(what, e);
    } else if (zero_bytes && (e = hipMemsetAsync(*p, 0, zero_bytes < sz ? zero_bytes : sz, stream)) != hipSuccess) {
        return ws_set_err(what, e);
    }
    *have = sz;
    return 0;
}

static int workspace(WsDevState* ds, size_t bytes, hipStream_t stream, void** out) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    WsStreamWs* w = nullptr;
    int rc = stream_slot(ds, stream, &w);
    if (rc) return rc;
    void* p = w->ws;
    if ((rc = grow(&p, &w->ws_bytes, bytes, stream, 16, "hipMalloc(workspace)"))) return rc;
    w->ws = reinterpret_cast<u32*>(p);
    *out = p;
    return 0;
}

// encode workspace (ws_encode.hip), same growth rules as the decode workspace
int ws_encode_workspace(size_t bytes, hipStream_t stream, void** out) {
    WsDevState* ds = nullptr;
    int rc = dev_state(&ds);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    WsStreamWs* w = nullptr;
    if ((rc = stream_slot(ds, stream, &w))) return rc;
    if ((rc = grow(&w->ews, &w->ews_bytes, bytes, stream, 0, "hipMalloc(encode workspace)"))) return rc;
    *out = w->ews;
    return 0;
}

// auxiliary scratch (ws_stream.hip): device part grown like the workspaces, its first
// WS_AUX_HEAD bytes zeroed at every (re)allocation (the stream path's state rests at zero);
// a pinned, device-visible host part grown after draining the stream (never while capturing)
int ws_aux_workspace(size_t dbytes, size_t hbytes, hipStream_t stream, WsAux* out) {
    WsDevState* ds = nullptr;
    int rc = dev_state(&ds);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    WsStreamWs* w = nullptr;
    if ((rc = stream_slot(ds, stream, &w))) return rc;
    const void* before = w->aws;
    const size_t have = w->aws_bytes;
    if ((rc = grow(&w->aws, &w->aws_bytes, dbytes < WS_AUX_HEAD ? WS_AUX_HEAD : dbytes, stream, WS_AUX_HEAD,
                   "hipMalloc(aux workspace)")))
        return rc;
    if (w->aws != before || w->aws_bytes != have) w->aux_state_ok = true;   // freshly zeroed
    if (w->hws_bytes < hbytes) {
        if (capturing(stream)) return ws_set_msg("aux host scratch cannot grow while the stream captures a graph");
        hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return ws_set_err("hipStreamSynchronize", e);
        if (w->hws) (void)hipHostFree(w->hws);
        w->hws = nullptr;
        w->hws_dev = nullptr;
        w->hws_bytes = 0;
        const size_t sz = hbytes + hbytes / 4 + 4096;
        if ((e = hipHostMalloc(&w->hws, sz, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
            return ws_set_err("hipHostMalloc(aux scratch)", e);
        memset(w->hws, 0, sz);
        if ((e = hipHostGetDevicePointer(&w->hws_dev, w->hws, 0)) != hipSuccess)
            return ws_set_err("hipHostGetDevicePointer(aux scratch)", e);
        w->hws_bytes = sz;
    }
    out->d = w->aws;
    out->h = w->hws;
    out->h_dev = w->hws_dev;
    out->state_ok = &w->aux_state_ok;
    return 0;
}

bool ws_capturing(hipStream_t stream) { return capturing(stream); }

// per-call generation number for the piece path's disorder word (never 0)
u32 ws_next_gen() {
    static std::atomic<u32> s_gen{0};
    u32 gen = ++s_gen;
    if (gen == 0) gen = ++s_gen;                                       // 0 = a fresh workspace's value
    return gen;
}

// the calling stream's decode workspace (first 16 bytes zeroed at allocation)
int ws_device_workspace(size_t bytes, hipStream_t stream, void** out) {
    WsDevState* ds = nullptr;
    int rc = dev_state(&ds);
    if (rc) return rc;
    return workspace(ds, bytes, stream, out);
}

// the decode variant a call takes
static int decode_path(const WsTuning& t, u64 span, u32 nseg, u32 max_frames) {
    if (t.path == 4) return max_frames <= 64 ? 4 : 3;                 // segfuse holds <= 64 frames per segment
    if (t.path >= 0) return t.path;
    return ws_segfuse_fits(span, nseg, max_frames) ? 4 : 3;
}

size_t ws_decode_workspace_bytes(u64 span, u32 nseg, u32 max_frames) {
    const int path = decode_path(tuning(), span, nseg, max_frames);
    return path == 3 ? ws_piece_workspace_bytes(span, nseg, max_frames) : 0;
}

int ws_decode_range(unsigned char* d_buf, u64 lo, u64 hi, const u64* d_seg_off, const u64* d_seg_len, u32 nseg,
                    u32 max_frames, const u64* d_desc_base, WebsocketFrameDesc_t* d_desc, WebsocketSegResult_t* d_res,
                    hipStream_t stream, void* ws, size_t ws_bytes) {
    if (nseg == 0) return 0;
    if (!d_buf || !d_seg_off || !d_seg_len || !d_desc || !d_res || max_frames == 0 || hi < lo)
        return ws_set_msg("websocketframeBatchDecodeDevice: invalid argument");
    if ((reinterpret_cast<uintptr_t>(d_desc) | reinterpret_cast<uintptr_t>(d_res)) & 15)
        return ws_set_msg("websocketframeBatchDecodeDevice: d_desc/d_res not 16-B aligned");
    WsDevState* ds = nullptr;
    int rc = dev_state(&ds);
    if (rc) return rc;
    const WsTuning t = tuning();
    WsLaunch L;
    L.buf = d_buf; L.seg_off = d_seg_off; L.seg_len = d_seg_len; L.nseg = nseg; L.max_frames = max_frames;
    L.desc_base = d_desc_base; L.desc = d_desc; L.res = d_res;
    L.stream = stream;
    L.cus = ds->cus;
    u32* ctr = ds->ctr + (size_t)(ds->slot++ % WS_CTR_RING) * 32;
    const int path = decode_path(t, hi - lo, nseg, max_frames);
    if (path == 1) return ws_launch_walker(L, t.unroll, t.nt, t.dyn, t.blocks_per_cu, ctr);
    if (path == 4) return ws_launch_segfuse(L, t.nt);
    const size_t need = ws_decode_workspace_bytes(hi - lo, nseg, max_frames);
    if (ws && ws_bytes < need) return ws_set_msg("websocketframe batch decode: workspace too small");
    if (!ws && need) {
        if ((rc = workspace(ds, need, L.stream, &ws))) return rc;
    }
    const u32 gen = ws_next_gen();
    const u32* disorder = nullptr;
    bool fallback = false;
    if ((rc = ws_launch_piece(L, lo, hi, t.nt, reinterpret_cast<unsigned char*>(ws), gen, &disorder, &fallback)))
        return rc;
    // segments out of buffer order are decoded by K2's fallback; with no pieces to launch K2
    // on, a small gated walker grid does it (exits at once for ordered batches)
    return fallback ? ws_launch_walker(L, t.unroll, t.nt, 0, 1, ctr, disorder, gen) : 0;
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeBatchDecodeDevice(unsigned char* d_buf, unsigned long long buflen,
                                                                  const u64* d_seg_off, const u64* d_seg_len,
                                                                  unsigned int nseg, unsigned int max_frames,
                                                                  const u64* d_desc_base, WebsocketFrameDesc_t* d_desc,
                                                                  WebsocketSegResult_t* d_res, void* hip_stream) {
    return ws_decode_range(d_buf, 0, buflen, d_seg_off, d_seg_len, nseg, max_frames, d_desc_base, d_desc, d_res,
                           reinterpret_cast<hipStream_t>(hip_stream));
}
