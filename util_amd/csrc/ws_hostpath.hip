// ws_hostpath.hip — websocketframeBatchDecodeHost: the batch lives in host memory
// (the reactor's inbufs, net_reactor.c:484-498). Pipelined over groups of
// consecutive segments on WS_HOST_SLOTS streams, each with its own device slot:
//   H2D(group g+2) | decode(group g+1) | D2H(group g)
// so the PCIe copies in both directions and the kernel overlap. With pinned host
// memory (hipHostMalloc / hipHostRegister) the copies are asynchronous DMA; pageable
// memory works but goes through the runtime's staging copies.
//
// The device slot is addressed as d_slot - lo, so the kernel sees the caller's own
// segment offsets and writes descriptors with buffer-relative offsets directly.
// Only segment bytes are copied back (adjacent segments merged into one copy): host bytes
// between segments are read by the H2D copy of a group's span but never written, so a
// neighbouring inbuf that another thread is filling meanwhile is left alone. The calling
// thread's current HIP device is restored before returning.
#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include <string>

#include "ws_common.h"

#define WS_HOST_DEV 64
#define WS_HOST_SLOTS 3

struct WsHostSlot {
    hipStream_t st = nullptr;
    unsigned char* buf = nullptr;
    size_t buf_bytes = 0;
    u64* segs = nullptr;  // seg_off[cap] then seg_len[cap]
    size_t seg_cap = 0;
    WebsocketFrameDesc_t* desc = nullptr;
    size_t desc_cap = 0;
    WebsocketSegResult_t* res = nullptr;
    size_t res_cap = 0;
    unsigned char* ws = nullptr;   // decode workspace of this slot's stream
    size_t ws_cap = 0;
};

struct WsHostPipe {
    std::mutex mu;
    WsHostSlot slot[WS_HOST_SLOTS];
};
static WsHostPipe g_pipe[WS_HOST_DEV];

std::atomic<size_t> ws_host_chunk_bytes{64ull << 20};  // group size target ("host_chunk_mb")

template <typename T>
static int grow(T** p, size_t* cap, size_t need, const char* what) {
    if (*cap >= need) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), need * sizeof(T));
    if (e != hipSuccess) return ws_set_err(what, e);
    *cap = need;
    return 0;
}

struct Group {
    u32 s0, s1;   // segments [s0, s1)
    u64 lo, hi;   // host byte span [lo, hi)
};

struct DeviceGuard {          // restores the calling thread's current device on every return
    int dev = -1;
    DeviceGuard() { if (hipGetDevice(&dev) != hipSuccess) dev = -1; }
    ~DeviceGuard() { if (dev >= 0) (void)hipSetDevice(dev); }
};

extern "C" WSFRAME_AMD_EXPORT int websocketframeBatchDecodeHost(unsigned char* h_buf, unsigned long long buflen,
                                                                const u64* h_seg_off, const u64* h_seg_len,
                                                                unsigned int nseg, unsigned int max_frames,
                                                                WebsocketFrameDesc_t* h_desc,
                                                                WebsocketSegResult_t* h_res, int device) {
    if (nseg == 0) return 0;
    if (!h_buf || !h_seg_off || !h_seg_len || !h_desc || !h_res || max_frames == 0)
        return ws_set_msg("websocketframeBatchDecodeHost: invalid argument");
    if (device < 0 || device >= WS_HOST_DEV) return ws_set_err("device index", hipErrorInvalidDevice);
    DeviceGuard guard;
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return ws_set_err("hipSetDevice", e);

    // groups of consecutive, ascending, non-overlapping segments of about one chunk;
    // any other layout is decoded as one group spanning all segments
    bool ordered = true;
    u64 prev_end = 0, lo_all = ~0ull, hi_all = 0;
    for (u32 s = 0; s < nseg; ++s) {
        const u64 o = h_seg_off[s], l = h_seg_len[s];
        if (o > buflen || l > buflen - o) return ws_set_msg("websocketframeBatchDecodeHost: segment outside buffer");
        if (o < prev_end) ordered = false;
        prev_end = o + l;
        lo_all = o < lo_all ? o : lo_all;
        hi_all = o + l > hi_all ? o + l : hi_all;
    }
    const size_t desc_cap_bytes = 64ull << 20;
    std::vector<Group> groups;
    if (!ordered) {
        groups.push_back(Group{0, nseg, lo_all, hi_all});
    } else {
        for (u32 s = 0; s < nseg;) {
            Group g{s, s + 1, h_seg_off[s], h_seg_off[s] + h_seg_len[s]};
            while (g.s1 < nseg) {
                const u64 end = h_seg_off[g.s1] + h_seg_len[g.s1];
                if (end - g.lo > ws_host_chunk_bytes) break;
                if ((size_t)(g.s1 + 1 - g.s0) * max_frames * sizeof(WebsocketFrameDesc_t) > desc_cap_bytes) break;
                g.hi = end;
                ++g.s1;
            }
            groups.push_back(g);
            s = g.s1;
        }
    }
    // the host ranges written back per group: its segments' bytes, in buffer order, adjacent
    // segments merged
    std::vector<std::vector<std::pair<u64, u64>>> back(groups.size());
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        const Group& g = groups[gi];
        std::vector<std::pair<u64, u64>> r;
        r.reserve(g.s1 - g.s0);
        for (u32 s = g.s0; s < g.s1; ++s)
            if (h_seg_len[s]) r.emplace_back(h_seg_off[s], h_seg_off[s] + h_seg_len[s]);
        if (!ordered) std::sort(r.begin(), r.end());
        for (const auto& x : r) {
            if (!back[gi].empty() && x.first <= back[gi].back().second)
                back[gi].back().second = std::max(back[gi].back().second, x.second);
            else
                back[gi].push_back(x);
        }
    }
    size_t max_span = 0, max_nseg = 0;
    for (const Group& g : groups) {
        max_span = g.hi - g.lo > max_span ? g.hi - g.lo : max_span;
        max_nseg = g.s1 - g.s0 > max_nseg ? g.s1 - g.s0 : max_nseg;
    }

    WsHostPipe& P = g_pipe[device];
    std::lock_guard<std::mutex> lock(P.mu);
    int rc = 0;
    const int nslots = groups.size() < WS_HOST_SLOTS ? (int)groups.size() : WS_HOST_SLOTS;
    for (int k = 0; k < nslots; ++k) {
        WsHostSlot& S = P.slot[k];
        if (!S.st && (e = hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking)) != hipSuccess)
            return ws_set_err("hipStreamCreate", e);
        if ((e = hipStreamSynchronize(S.st)) != hipSuccess) return ws_set_err("hipStreamSynchronize", e);
        if ((rc = grow(&S.buf, &S.buf_bytes, max_span + WEBSOCKET_BATCH_PAD, "hipMalloc(host slot)"))) return rc;
        if ((rc = grow(&S.segs, &S.seg_cap, 2 * max_nseg, "hipMalloc(host slot segs)"))) return rc;
        if ((rc = grow(&S.desc, &S.desc_cap, max_nseg * max_frames, "hipMalloc(host slot desc)"))) return rc;
        if ((rc = grow(&S.res, &S.res_cap, max_nseg, "hipMalloc(host slot res)"))) return rc;
        const size_t wsb = ws_decode_workspace_bytes(max_span, (u32)max_nseg, max_frames);
        if (wsb && S.ws_cap < wsb) {
            if ((rc = grow(&S.ws, &S.ws_cap, wsb, "hipMalloc(host slot workspace)"))) return rc;
            if ((e = hipMemset(S.ws, 0, 16)) != hipSuccess) return ws_set_err("hipMemset(host slot workspace)", e);
        }
    }
#define WS_TRY(call, what) do { if ((e = (call)) != hipSuccess) { rc = ws_set_err(what, e); goto drain; } } while (0)
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        const Group& g = groups[gi];
        WsHostSlot& S = P.slot[gi % nslots];
        const u32 n = g.s1 - g.s0;
        const size_t span = g.hi - g.lo;
        const size_t nd = (size_t)n * max_frames;
        WS_TRY(hipMemcpyAsync(S.buf, h_buf + g.lo, span, hipMemcpyHostToDevice, S.st), "H2D batch");
        WS_TRY(hipMemsetAsync(S.buf + span, 0, WEBSOCKET_BATCH_PAD, S.st), "hipMemset(pad)");
        WS_TRY(hipMemcpyAsync(S.segs, h_seg_off + g.s0, n * sizeof(u64), hipMemcpyHostToDevice, S.st), "H2D seg_off");
        WS_TRY(hipMemcpyAsync(S.segs + S.seg_cap / 2, h_seg_len + g.s0, n * sizeof(u64), hipMemcpyHostToDevice, S.st),
               "H2D seg_len");
        WS_TRY(hipMemsetAsync(S.desc, 0, nd * sizeof(WebsocketFrameDesc_t), S.st), "hipMemset(desc)");
        rc = ws_decode_range(S.buf - g.lo, g.lo, g.hi, S.segs, S.segs + S.seg_cap / 2, n, max_frames, nullptr, S.desc,
                             S.res, S.st, S.ws, S.ws_cap);
        if (rc) goto drain;
        for (const auto& x : back[gi])
            WS_TRY(hipMemcpyAsync(h_buf + x.first, S.buf + (x.first - g.lo), x.second - x.first, hipMemcpyDeviceToHost,
                                  S.st), "D2H batch");
        WS_TRY(hipMemcpyAsync(h_desc + (size_t)g.s0 * max_frames, S.desc, nd * sizeof(WebsocketFrameDesc_t),
                              hipMemcpyDeviceToHost, S.st), "D2H desc");
        WS_TRY(hipMemcpyAsync(h_res + g.s0, S.res, n * sizeof(WebsocketSegResult_t), hipMemcpyDeviceToHost, S.st),
               "D2H res");
    }
#undef WS_TRY
drain:
    for (int k = 0; k < nslots; ++k) {
        hipError_t e2 = hipStreamSynchronize(P.slot[k].st);
        if (e2 != hipSuccess && !rc) rc = ws_set_err("hipStreamSynchronize", e2);
    }
    return rc;
}

// ---------------------------------------------------------------------------------------------
// Several devices on one host rx arena (net_reactor.c:484-500): the
// ascending segments are cut into `ndev` contiguous ranges of about equal bytes (the segment
// boundary nearest to each equal share), and each range runs websocketframeBatchDecodeHost's
// pipeline on its own device from its own host thread, so every device's PCIe link carries its
// share (one pinned arena served by up to ndev links). A device listed twice runs its ranges one
// after the other (its pipeline is locked per device). Any other segment layout is decoded on
// devices[0] alone. Returns the first range's error (every range is drained first).
extern "C" WSFRAME_AMD_EXPORT int websocketframeBatchDecodeHostMulti(unsigned char* h_buf, unsigned long long buflen,
                                                                     const u64* h_seg_off, const u64* h_seg_len,
                                                                     unsigned int nseg, unsigned int max_frames,
                                                                     WebsocketFrameDesc_t* h_desc,
                                                                     WebsocketSegResult_t* h_res, const int* devices,
                                                                     int ndev) {
    if (nseg == 0) return 0;
    if (!devices || ndev <= 0 || !h_seg_off || !h_seg_len)
        return ws_set_msg("websocketframeBatchDecodeHostMulti: invalid argument");
    bool ordered = true;
    u64 prev_end = 0, total = 0;
    for (u32 s = 0; s < nseg; ++s) {
        if (h_seg_off[s] < prev_end) ordered = false;
        prev_end = h_seg_off[s] + h_seg_len[s];
        total += h_seg_len[s];
    }
    if (!ordered || ndev == 1 || nseg < 2)
        return websocketframeBatchDecodeHost(h_buf, buflen, h_seg_off, h_seg_len, nseg, max_frames, h_desc, h_res,
                                             devices[0]);
    // cuts: the segment boundary nearest to each equal share of the bytes
    const u32 nd = (u32)std::min<u64>((u64)ndev, nseg);
    std::vector<u32> cut(nd + 1, 0);
    cut[nd] = nseg;
    {
        u64 acc = 0;
        u32 s = 0;
        for (u32 r = 1; r < nd; ++r) {
            const long double t = (long double)total * r / nd;
            while (s < nseg && (long double)(acc + h_seg_len[s]) <= t) acc += h_seg_len[s++];
            // acc <= t < acc + len[s]: the nearer boundary
            if (s < nseg && (long double)(acc + h_seg_len[s]) - t < t - (long double)acc) acc += h_seg_len[s++];
            cut[r] = std::max(s, cut[r - 1]);
        }
    }
    std::vector<int> rc(nd, 0);
    std::vector<std::string> err(nd);
    auto part = [&](u32 r) {
        const u32 a = cut[r], b = cut[r + 1];
        if (a < b) {
            rc[r] = websocketframeBatchDecodeHost(h_buf, buflen, h_seg_off + a, h_seg_len + a, b - a, max_frames,
                                                  h_desc + (size_t)a * max_frames, h_res + a, devices[r]);
            if (rc[r]) err[r] = websocketframeGpuLastError();            // (the error text is per thread)
        }
    };
    std::vector<std::thread> th;
    th.reserve(nd);
    for (u32 r = 1; r < nd; ++r) th.emplace_back(part, r);
    part(0);
    for (auto& t : th) t.join();
    for (u32 r = 0; r < nd; ++r)
        if (rc[r]) {
            char msg[320];
            snprintf(msg, sizeof(msg), "websocketframeBatchDecodeHostMulti (device %d): %s", devices[r], err[r].c_str());
            ws_set_msg(msg);
            return rc[r];
        }
    return 0;
}
