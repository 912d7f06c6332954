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
#include <vector>

#include "ws_common.h"

static __thread char g_last_error[256];
extern std::atomic<size_t> ws_host_chunk_bytes;
extern WsOpt ws_reasm_path;
extern WsOpt ws_reasm_cfg;
extern WsOpt ws_piece_lds;
extern WsOpt ws_piece_win;
extern WsOpt ws_k2_timing;
void ws_k2_timing_reset();
int ws_k2_stat(unsigned long long* ns, unsigned long long* calls);
extern WsOpt ws_enc_front;
extern WsOpt ws_scan_alpha;
WsOpt ws_seg_win{-1};     // "seg_win": segfuse and fused reassembly take segments in 2^seg_win windows (ws_winn);
                          // -1: 4 windows for segfuse, 8 for the fused reassembly (profiles/r06_seg_win_ab.log)
extern WsOpt ws_stream_rw, ws_stream_rw_cmax, ws_stream_rounds, ws_stream_plink;
extern WsOpt ws_stream_win, ws_stream_split_capture, ws_stream_split, ws_stream_split_wait, ws_stream_c0, ws_stream_side_prio, ws_stream_split2,
    ws_stream_c1;
size_t ws_workspace_bytes_total();
extern std::atomic<unsigned long long> ws_stat_rw_chunks, ws_stat_rw_chunk_walks, ws_stat_stream_skips,
    ws_stat_stream_splits;
extern std::atomic<unsigned long long> ws_stat_adoptions;
extern std::atomic<unsigned long long> ws_stat_k2_windows;
extern std::atomic<unsigned long long> ws_stat_adoption_refusals;

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
// launch configuration (tunable for in-process A/B by bench/profiling tools; every value is
// parity-tested, tests/test_gpu_options.py)

static WsOpt g_path{-1};   // "path": -1 auto (4 for many small segments, else 3), 1 walker (one wave per
                           // segment), 3 piece (K1 + K2), 4 segfuse

extern "C" WSFRAME_AMD_EXPORT int websocketframeGpuSetOption(const char* name, long long value) {
    if (!strcmp(name, "path")) {
        if (value != -1 && value != 1 && value != 3 && value != 4) return -1;
        g_path = (int)value;
    }
    else if (!strcmp(name, "host_chunk_mb")) {
        if (value <= 0 || value > 65536) return -1;
        ws_host_chunk_bytes = (size_t)value << 20;
    }
    else if (!strcmp(name, "piece_lds")) {
        if (value < 0 || value > 65536) return -1;
        ws_piece_lds = (int)value;
    }
    else if (!strcmp(name, "piece_win")) {
        if (value < -1 || value > 6) return -1;
        ws_piece_win = (int)value;
    }
    else if (!strcmp(name, "seg_win")) {
        if (value < -1 || value > 3) return -1;
        ws_seg_win = (int)value;
    }
    else if (!strcmp(name, "reasm_path")) {
        if (value < 0 || value > 2) return -1;
        ws_reasm_path = (int)value;
    }
    else if (!strcmp(name, "reasm_cfg")) {
        if (value < 0 || value > 2) return -1;
        ws_reasm_cfg = (int)value;
    }
    else if (!strcmp(name, "enc_front")) {
        if (value < 0 || value > 1) return -1;
        ws_enc_front = (int)value;
    }
    else if (!strcmp(name, "stream_rw")) {
        if (value < 0 || value > 2) return -1;
        ws_stream_rw = (int)value;
    }
    else if (!strcmp(name, "stream_rw_cmax")) {
        if (value < 16 || value > 26) return -1;
        ws_stream_rw_cmax = (int)value;
    }
    else if (!strcmp(name, "stream_plink")) {
        if (value < 0 || value > 1) return -1;
        ws_stream_plink = (int)value;
    }
    else if (!strcmp(name, "stream_split")) {
        if (value < 0 || value > 255) return -1;
        ws_stream_split = (int)value;
    }
    else if (!strcmp(name, "stream_split_wait")) {
        if (value < 0 || value > 2) return -1;
        ws_stream_split_wait = (int)value;
    }
    else if (!strcmp(name, "stream_split2")) {
        if (value < 0 || value > 255) return -1;
        ws_stream_split2 = (int)value;
    }
    else if (!strcmp(name, "stream_win")) {
        if (value < -1 || value > 6) return -1;
        ws_stream_win = (int)value;
    }
    else if (!strcmp(name, "stream_split_capture")) {
        if (value < 0 || value > 1) return -1;
        ws_stream_split_capture = (int)value;
    }
    else if (!strcmp(name, "stream_c1")) {
        if (value < 0 || value > 6) return -1;
        ws_stream_c1 = (int)value;
    }
    else if (!strcmp(name, "stream_side_prio")) {
        if (value < 0 || value > 2) return -1;
        ws_stream_side_prio = (int)value;
    }
    else if (!strcmp(name, "stream_c0")) {
        if (value < 0 || value > 6) return -1;
        ws_stream_c0 = (int)value;
    }
    else if (!strcmp(name, "stream_rounds")) {
        if (value < 1 || value > 64) return -1;
        ws_stream_rounds = (int)value;
    }
    else if (!strcmp(name, "scan_alpha")) {
        if (value < 0 || value > 1) return -1;
        ws_scan_alpha = (int)value;
    }
    else if (!strcmp(name, "k2_timing")) {
        ws_k2_timing = value ? 1 : 0;
        ws_k2_timing_reset();
    }
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
    else if (!strcmp(name, "stream_skips")) *value = ws_stat_stream_skips.load();
    else if (!strcmp(name, "stream_splits")) *value = ws_stat_stream_splits.load();
    else if (!strcmp(name, "workspace_bytes")) *value = ws_workspace_bytes_total();
    else if (!strcmp(name, "capture_adoptions")) *value = ws_stat_adoptions.load();
    else if (!strcmp(name, "k2_windows")) *value = ws_stat_k2_windows.load();
    else if (!strcmp(name, "capture_adoption_refusals")) *value = ws_stat_adoption_refusals.load();

    else return -1;
    return 0;
}

// ---------------------------------------------------------------------------------------------
// Per-device state: CU count, LDS per CU, and one workspace slot per (HIP stream, graph
// capture), grown on demand. Calls on different streams of one device may overlap in time (a
// reactor with several rx batches in flight, one stream each); calls on one stream are ordered
// by the stream. A call pins its slot for its whole duration (WsSlot): LRU eviction never
// takes a pinned slot. A graph capture's slot belongs to that graph: a HIP user object on the
// graph marks it dead when the graph (and every executable made from it) is destroyed, and the
// next eager library call frees its buffers (or the next capture adopts them, slot_rezero).
#define WS_MAX_DEV 64
#define WS_STREAM_SLOTS 16
struct WsStreamWs {
    hipStream_t stream = nullptr;
    unsigned long long capture = 0; // capture id of the graph this slot belongs to (0: eager calls)
    bool used = false;             // assigned to a stream (eager) or a capture
    bool captured = false;         // belongs to a graph capture: never reassigned while its graph lives
    std::atomic<int> dead{0};      // its graph was destroyed (set by the user object's destructor)
    int busy = 0;                  // calls holding the slot (WsSlot)
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
    int* adv_h = nullptr;          // pinned host words: the device's stride hint for the next call
    int* adv_d = nullptr;
    std::vector<std::pair<void*, size_t>> retired;   // buffers replaced while capturing (the graph still uses them)
    hipEvent_t done = nullptr;     // captured slots: recorded at the end of every captured call (an event
                                   // record node), so a destroyed graph's replays are known to be finished
    hipStream_t side = nullptr;    // the raw stream's split walk: part 1 runs here (ws_stream.hip RwSplit)
    int side_prio = 0;             // ... created with this priority choice (0 default, 1 least, 2 greatest)
    hipEvent_t sev[WS_SIDE_EVENTS] = {};   // ... and its fork / join events
};
struct WsDevState {
    int init = 0;
    int cus = 0;
    int lds = 0;
    std::deque<WsStreamWs> sw;     // grows; stable addresses
    unsigned long long tick = 0;
    std::vector<std::pair<void*, size_t>> deferred;   // adopted slots' retired buffers: freed by the next eager call
};
static WsDevState g_dev[WS_MAX_DEV];
static std::mutex g_dev_mu;        // device init and the stream-slot table
size_t ws_workspace_bytes_total() {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    size_t t = 0;
    for (auto& d : g_dev) {
        for (auto& w : d.sw) {
            t += w.ws_bytes + w.ews_bytes + w.aws_bytes;
            for (auto& r : w.retired) t += r.second;
        }
        for (auto& r : d.deferred) t += r.second;
    }
    return t;
}

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
        st.lds = prop.maxSharedMemoryPerMultiProcessor > 0 ? (int)prop.maxSharedMemoryPerMultiProcessor : 65536;
        st.init = 1;
    }
    *out = &st;
    return 0;
}

int ws_device_info(int* cus, int* lds_per_cu) {
    WsDevState* ds = nullptr;
    const int rc = dev_state(&ds);
    if (rc) return rc;
    *cus = ds->cus;
    *lds_per_cu = ds->lds;
    return 0;
}

static bool capturing(hipStream_t stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(stream, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
}

// free a slot's buffers (its stream's work, or its graph, is done)
static void slot_free(WsStreamWs& w) {
    (void)hipFree(w.ws);
    (void)hipFree(w.ews);
    (void)hipFree(w.aws);
    if (w.hws) (void)hipHostFree(w.hws);
    if (w.adv_h) (void)hipHostFree(w.adv_h);
    for (auto& r : w.retired) (void)hipFree(r.first);
    w.retired.clear();
    w.ws = nullptr; w.ews = nullptr; w.aws = nullptr; w.hws = nullptr; w.hws_dev = nullptr;
    w.adv_h = nullptr; w.adv_d = nullptr;
    w.ws_bytes = w.ews_bytes = w.aws_bytes = w.hws_bytes = 0;
    w.aux_state_ok = false;
    w.stream = nullptr;
    w.capture = 0;
    w.used = false;
    w.captured = false;
    w.dead = 0;
}

std::atomic<unsigned long long> ws_stat_adoptions{0};
std::atomic<unsigned long long> ws_stat_adoption_refusals{0};   // dead slots not adopted: a replay still queued
static void capture_slot_destroyed(void* p) { reinterpret_cast<WsStreamWs*>(p)->dead.store(1); }

// a destroyed graph's slot may be adopted only once every replay that was launched has finished:
// its calls end with an event record node, so the event is complete (or was never recorded) then.
// The user object's release alone does not say that (hipUserObjectNoDestructorSync).
static bool replays_done(WsStreamWs& w) {
    if (!w.done) return true;
    hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&m);
    const hipError_t e = hipEventQuery(w.done);
    (void)hipThreadExchangeStreamCaptureMode(&m);
    return e == hipSuccess;
}

// zero the resting heads of a slot's buffers (decode/reassembly/stream workspace: 16 B; the
// auxiliary scratch: WS_AUX_HEAD) outside any capture: private stream, relaxed capture mode
static int slot_rezero(WsStreamWs& w) {
    if (!w.ws && !w.aws) return 0;
    hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&m);
    hipStream_t ps = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
    if (e == hipSuccess && w.ws) e = hipMemsetAsync(w.ws, 0, 16, ps);
    if (e == hipSuccess && w.aws) e = hipMemsetAsync(w.aws, 0, w.aws_bytes < WS_AUX_ZERO ? w.aws_bytes : WS_AUX_ZERO, ps);
    if (e == hipSuccess) e = hipStreamSynchronize(ps);
    if (ps) (void)hipStreamDestroy(ps);
    (void)hipThreadExchangeStreamCaptureMode(&m);
    if (e != hipSuccess) return ws_set_err("workspace re-zero (adopted capture slot)", e);
    if (w.aws) w.aux_state_ok = true;
    return 0;
}

// the slot of (stream, capture) (caller holds g_dev_mu), pinned. Eager calls keep at most
// WS_STREAM_SLOTS slots: a further stream takes the least recently used idle one after a
// device synchronize (a new slot if every one is pinned). Every graph capture gets a slot of its
// own, keyed by its capture id (torch captures every graph on one shared stream, so the stream
// alone does not tell graphs apart): the graph uses that workspace on every replay, so it is
// never handed to another capture or to an eager call while the graph lives.
static int stream_slot(WsDevState* ds, hipStream_t stream, WsStreamWs** out) {
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    unsigned long long cap = 0;
    hipGraph_t graph = nullptr;
    if (hipStreamGetCaptureInfo_v2(stream, &cst, &cap, &graph, nullptr, nullptr) != hipSuccess ||
        cst != hipStreamCaptureStatusActive)
        cap = 0;
    else if (!cap)
        cap = ~0ull;
    // release the slots of destroyed graphs, from eager calls only: a hipFree while this stream
    // captures would invalidate the capture (relaxed mode for captures on other threads)
    if (!cap) {
        hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
        (void)hipThreadExchangeStreamCaptureMode(&mode);
        for (WsStreamWs& w : ds->sw)
            if (w.used && w.captured && w.dead.load() && !w.busy) slot_free(w);
        for (auto& r : ds->deferred) (void)hipFree(r.first);
        ds->deferred.clear();
        (void)hipThreadExchangeStreamCaptureMode(&mode);
    }
    WsStreamWs* lru = nullptr;
    WsStreamWs* freeslot = nullptr;
    WsStreamWs* adopt = nullptr;   // a destroyed graph's idle slot: a new capture takes its buffers
    size_t eager = 0;
    for (WsStreamWs& w : ds->sw) {
        if (w.used && w.stream == stream && w.capture == cap && !w.dead.load()) {
            w.last = ++ds->tick;
            ++w.busy;
            *out = &w;
            return 0;
        }
        if (!w.used && !w.busy) {
            if (!freeslot) freeslot = &w;
            continue;
        }
        if (w.captured && w.dead.load() && !w.busy) {
            if (!adopt && cap) {
                if (replays_done(w)) adopt = &w;
                else ++ws_stat_adoption_refusals;
            }
            continue;
        }
        if (!w.captured) {
            ++eager;
            if (!w.busy && (!lru || w.last < lru->last)) lru = &w;
        }
    }
    WsStreamWs* w = nullptr;
    if (cap && adopt) {
        // a process that only captures, replays and destroys graphs never makes the eager call that
        // frees dead slots: the new capture reuses one as it is (no hipFree inside a capture), with
        // the workspace heads zeroed once on a private stream, as a fresh allocation would be
        int rc = slot_rezero(*adopt);
        if (rc) return rc;
        w = adopt;
        w->dead = 0;
        ++ws_stat_adoptions;
        // the buffers its dead graph's capture replaced: free at the next eager call (not inside a capture)
        ds->deferred.insert(ds->deferred.end(), w->retired.begin(), w->retired.end());
        w->retired.clear();
    } else if (freeslot) {
        w = freeslot;
    } else if (cap || eager < WS_STREAM_SLOTS || !lru) {
        ds->sw.emplace_back();
        w = &ds->sw.back();
    } else {                       // every eager slot taken by another stream: drain the device, then reuse
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) return ws_set_err("hipDeviceSynchronize", e);
        w = lru;
    }
    w->used = true;
    w->stream = stream;
    w->capture = cap;
    w->captured = cap != 0;
    w->last = ++ds->tick;
    ++w->busy;
    if (cap && graph) {
        // tie the slot's lifetime to the graph being captured
        hipUserObject_t uo = nullptr;
        hipError_t e = w->done ? hipSuccess : hipEventCreateWithFlags(&w->done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipUserObjectCreate(&uo, w, capture_slot_destroyed, 1, hipUserObjectNoDestructorSync);
        if (e == hipSuccess) e = hipGraphRetainUserObject(graph, uo, 1, hipGraphUserObjectMove);
        if (e != hipSuccess) {
            // the slot is not tied to any graph: hand it back (its buffers stay for the next user)
            --w->busy;
            w->used = false;
            w->captured = false;
            w->capture = 0;
            w->stream = nullptr;
            return ws_set_err("hipUserObjectCreate (capture workspace)", e);
        }
    }
    *out = w;
    return 0;
}

// grow *p to at least `bytes`. Eagerly: the stream's previous work may still read it, so drain
// first. While capturing a graph (relaxed-mode allocation), the buffer being replaced stays
// alive until the slot is released (kernels captured earlier in this graph use it).
static int grow(WsStreamWs* w, void** p, size_t* have, size_t bytes, hipStream_t stream, size_t zero_bytes,
                const char* what) {
    if (*have >= bytes) return 0;
    hipError_t e;
    const bool cap = capturing(stream);
    if (*p) {
        if (cap) {
            w->retired.emplace_back(*p, *have);
        } else {
            if ((e = hipStreamSynchronize(stream)) != hipSuccess) return ws_set_err("hipStreamSynchronize", e);
            (void)hipFree(*p);
        }
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

// ---- WsSlot: a (stream, capture) slot pinned for one call
WsSlot::~WsSlot() { release(); }

void WsSlot::release() {
    if (!w) return;
    // a captured call ends with an event record node (replays_done). Assumption: once
    // hipGraphLaunch has queued a replay, w->done reads as not ready until that replay's record
    // node has run — HIP's host-side launch resets the event's status at enqueue. If the record
    // only changed the status when the node ran, a query between launch and node would report the
    // previous replay's completed record and the slot could be adopted too early; the capture test
    // (tests/test_gpu_graph.py, refusal stat) checks the refusal whenever the runtime leaves a
    // destroyed graph's replay queued.
    if (w->captured && w->done && capturing(st)) (void)hipEventRecord(w->done, st);
    std::lock_guard<std::mutex> lk(g_dev_mu);
    --w->busy;
    w = nullptr;
}

int WsSlot::acquire(hipStream_t stream) {
    release();
    WsDevState* ds = nullptr;
    int rc = dev_state(&ds);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    st = stream;
    cus = ds->cus;
    lds = ds->lds;
    return stream_slot(ds, stream, &w);
}

int WsSlot::workspace(size_t bytes, size_t zero_bytes, void** out) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    void* p = w->ws;
    const int rc = grow(w, &p, &w->ws_bytes, bytes, st, zero_bytes < 16 ? 16 : zero_bytes, "hipMalloc(workspace)");
    w->ws = reinterpret_cast<u32*>(p);
    if (rc) return rc;
    *out = p;
    return 0;
}

int WsSlot::encode_workspace(size_t bytes, void** out) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    const int rc = grow(w, &w->ews, &w->ews_bytes, bytes, st, 0, "hipMalloc(encode workspace)");
    if (rc) return rc;
    *out = w->ews;
    return 0;
}

// auxiliary scratch (ws_stream.hip): device part grown like the workspaces, its first
// WS_AUX_HEAD bytes zeroed at every (re)allocation (the stream path's state rests at zero);
// a pinned, device-visible host part grown after draining the stream (never while capturing)
int WsSlot::aux(size_t dbytes, size_t hbytes, WsAux* out) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    const void* before = w->aws;
    const size_t have = w->aws_bytes;
    int rc = grow(w, &w->aws, &w->aws_bytes, dbytes < WS_AUX_HEAD ? WS_AUX_HEAD : dbytes, st, WS_AUX_ZERO,
                  "hipMalloc(aux workspace)");
    if (rc) return rc;
    if (w->aws != before || w->aws_bytes != have) w->aux_state_ok = true;   // freshly zeroed
    if (w->hws_bytes < hbytes) {
        if (capturing(st)) return ws_set_msg("aux host scratch cannot grow while the stream captures a graph");
        hipError_t e = hipStreamSynchronize(st);
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

// the side stream and events of the raw stream's split walk (created once per slot, outside any
// capture's rules: relaxed mode; a capture forks into the side stream through its events)
int WsSlot::side(hipStream_t* side_out, hipEvent_t* ev, int prio) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (w->side && w->side_prio != prio && !capturing(st)) {      // another priority asked for (eager calls only)
        hipError_t e = hipStreamSynchronize(w->side);
        if (e == hipSuccess) e = hipStreamDestroy(w->side);
        if (e != hipSuccess) return ws_set_err("side stream (raw stream split)", e);
        w->side = nullptr;
    }
    if (!w->side || !w->sev[WS_SIDE_EVENTS - 1]) {
        hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
        (void)hipThreadExchangeStreamCaptureMode(&m);
        int least = 0, greatest = 0;
        hipError_t e = hipSuccess;
        if (!w->side) {
            if (prio) e = hipDeviceGetStreamPriorityRange(&least, &greatest);
            if (e == hipSuccess)
                e = prio ? hipStreamCreateWithPriority(&w->side, hipStreamNonBlocking, prio == 1 ? least : greatest)
                         : hipStreamCreateWithFlags(&w->side, hipStreamNonBlocking);
            w->side_prio = prio;
        }
        for (int k = 0; k < WS_SIDE_EVENTS && e == hipSuccess; ++k)
            if (!w->sev[k]) e = hipEventCreateWithFlags(&w->sev[k], hipEventDisableTiming);
        (void)hipThreadExchangeStreamCaptureMode(&m);
        if (e != hipSuccess) return ws_set_err("side stream (raw stream split)", e);
    }
    *side_out = w->side;
    for (int k = 0; k < WS_SIDE_EVENTS; ++k) ev[k] = w->sev[k];
    return 0;
}

// the pinned advice words (eager calls only): [0] 1 = nearly every segment of the last call held frames of
// one length, [1] the length of its first frame (K1's first-step stride guess for the next call)
int WsSlot::advice(int** host, int** dev) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (!w->adv_h) {
        if (capturing(st)) return ws_set_msg("advice word cannot be allocated while capturing");
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&w->adv_h), 64, hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) return ws_set_err("hipHostMalloc(advice)", e);
        memset(w->adv_h, 0, 64);
        if ((e = hipHostGetDevicePointer(reinterpret_cast<void**>(&w->adv_d), w->adv_h, 0)) != hipSuccess)
            return ws_set_err("hipHostGetDevicePointer(advice)", e);
    }
    *host = w->adv_h;
    *dev = w->adv_d;
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

// the decode variant a call takes
static int decode_path(int path, u64 span, u32 nseg, u32 max_frames) {
    if (path == 4) return max_frames <= 64 ? 4 : 3;                   // segfuse holds <= 64 frames per segment
    if (path >= 0) return path;
    return ws_segfuse_fits(span, nseg, max_frames) ? 4 : 3;
}

size_t ws_decode_workspace_bytes(u64 span, u32 nseg, u32 max_frames) {
    const int path = decode_path(g_path, span, nseg, max_frames);
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
    WsLaunch L;
    L.buf = d_buf; L.seg_off = d_seg_off; L.seg_len = d_seg_len; L.nseg = nseg; L.max_frames = max_frames;
    L.desc_base = d_desc_base; L.desc = d_desc; L.res = d_res;
    L.stream = stream;
    L.cus = ds->cus;
    L.lds_per_cu = ds->lds;
    const int path = decode_path(g_path, hi - lo, nseg, max_frames);
    if (path == 1) return ws_launch_walker(L);
    if (path == 4) return ws_launch_segfuse(L);
    const size_t need = ws_decode_workspace_bytes(hi - lo, nseg, max_frames);
    if (ws && ws_bytes < need) return ws_set_msg("websocketframe batch decode: workspace too small");
    WsSlot slot;
    int* adv_h = nullptr;
    int* adv_d = nullptr;
    if (!ws) {
        if ((rc = slot.acquire(stream))) return rc;
        // captured calls have no advice word: their K1 starts with no stride guess
        if (!capturing(stream) && (rc = slot.advice(&adv_h, &adv_d))) return rc;
    }
    const u32 gen = ws_next_gen();
    // K1's first-step stride guess: the previous call's first frame length, while the device
    // advised that nearly every segment held frames of one length (eager calls only)
    const u32 g0 = adv_h && __atomic_load_n(adv_h, __ATOMIC_RELAXED) == 1 ? (u32)__atomic_load_n(adv_h + 1, __ATOMIC_RELAXED)
                                                                         : 0u;
    if (!ws && need && (rc = slot.workspace(need, 16, &ws))) return rc;
    const u32* disorder = nullptr;
    bool fallback = false;
    if ((rc = ws_launch_piece(L, lo, hi, reinterpret_cast<unsigned char*>(ws), gen, adv_d, &disorder, &fallback,
                              g0 >= 2 ? g0 : 0u)))
        return rc;
    // segments out of buffer order are decoded by K2's fallback; with no pieces to launch K2
    // on, a small gated walker grid does it (exits at once for ordered batches)
    return fallback ? ws_launch_walker(L, disorder, gen) : 0;
}

extern "C" WSFRAME_AMD_EXPORT int websocketframeBatchDecodeDevice(unsigned char* d_buf, unsigned long long buflen,
                                                                  const u64* d_seg_off, const u64* d_seg_len,
                                                                  unsigned int nseg, unsigned int max_frames,
                                                                  const u64* d_desc_base, WebsocketFrameDesc_t* d_desc,
                                                                  WebsocketSegResult_t* d_res, void* hip_stream) {
    return ws_decode_range(d_buf, 0, buflen, d_seg_off, d_seg_len, nseg, max_frames, d_desc_base, d_desc, d_res,
                           reinterpret_cast<hipStream_t>(hip_stream));
}
