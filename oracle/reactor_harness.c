/*
 * reactor_harness.c — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Runs the REFERENCE's own rx stack on a byte stream: NetReactor_handle
 * (src/component/net_reactor.c:1073-1169) → reactor_stream_readev (:465-545, the
 * per-frame loop :515-526) → the stream hook on_read_stream
 * (src/component/net_channel_ex.c:110-157: fragment cache, check_cache_overflow :45-53,
 * streamtransportctxCacheRecvPacket/MergeRecvPacket src/datastruct/transport_ctx.c
 * :179-201, channel_merge_packet_handler/merge_packet :55-108) → on_recv.
 * The reactor, channel, transport and sysapi code are compiled from the reference
 * sources where they lie (oracle/Makefile `ref`, outputs only into oracle/_ref/).
 *
 * The stream is written into one end of an AF_UNIX socketpair in `chunk`-byte writes
 * (so frames are split across recv() calls at arbitrary points) and the other end is a
 * NET_CHANNEL_SIDE_SERVER channel opened with NetChannel_open_with_fd (:1206-1248),
 * wired with NetChannelEx_get_hook(side, SOCK_STREAM) (:616-619) + NetChannelEx_init
 * (:631-654) the way a user of the library does it.
 *
 * on_decode is either the websocket glue below (pktype NETPACKET_FRAGMENT,
 * fragment_eof = is_fin, bodylen = (unsigned int)datalen) around a websocketframeDecode
 * passed in by pointer (the reference's, from oracle/_ref/libwsref.so), or any other
 * on_decode passed in by pointer (libwsframe_amd.so's websocketframeOnDecode: the
 * drop-in check). Every on_recv message is recorded.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>
#include <fcntl.h>

#include "component/net_channel_ex.h"
#include "component/net_reactor.h"

typedef int (*decode_fn)(unsigned char* buf, unsigned long long len, unsigned char** data,
                         unsigned long long* datalen, int* is_fin, int* type);
typedef void (*on_decode_fn)(NetChannel_t* channel, unsigned char* buf, size_t len,
                             NetChannelInbufDecodeResult_t* result);

typedef struct Run {
    decode_fn decode;
    unsigned char* out;
    unsigned long long out_cap, out_len;
    unsigned long long* msg_len;
    unsigned int max_msgs, n_msgs;
    unsigned long long consumed, frames;
    int detached, detach_error, overrun;
    const NetChannelExHookProc_t* hook;
} Run;

static Run* g_run;   /* one run at a time (the reference callbacks carry no user pointer we own) */

/* the websocket glue a user of the reference writes */
static void ws_glue(NetChannel_t* channel, unsigned char* buf, size_t len, NetChannelInbufDecodeResult_t* r) {
    unsigned char* data = 0;
    unsigned long long datalen = 0;
    int is_fin = 0, type = 0;
    int ret = g_run->decode(buf, len, &data, &datalen, &is_fin, &type);
    (void)channel;
    if (ret < 0) { r->err = 1; return; }
    if (ret == 0) { r->incomplete = 1; return; }
    r->decodelen = (unsigned int)ret;
    r->bodyptr = data;
    r->bodylen = (unsigned int)datalen;
    r->fragment_eof = (char)is_fin;
    r->pktype = NETPACKET_FRAGMENT;
}

static void rec_recv(NetChannel_t* channel, unsigned char* bodyptr, size_t bodylen, const struct sockaddr* a,
                     socklen_t al) {
    Run* R = g_run;
    (void)channel; (void)a; (void)al;
    if (R->n_msgs >= R->max_msgs || R->out_len + bodylen > R->out_cap) { R->overrun = 1; return; }
    if (bodylen) memcpy(R->out + R->out_len, bodyptr, bodylen);
    R->out_len += bodylen;
    R->msg_len[R->n_msgs++] = bodylen;
}

/* on_read = the stream hook, counting what the reactor loop consumes (net_reactor.c:516-525) */
static int counted_read(NetChannel_t* ch, unsigned char* buf, unsigned int len, long long ts,
                        const struct sockaddr* a, socklen_t al) {
    int r = g_run->hook->on_read(ch, buf, len, ts, a, al);
    if (r > 0) { g_run->consumed += (unsigned int)r; g_run->frames++; }
    return r;
}

static void on_detach(NetChannel_t* ch) {
    g_run->detached = 1;
    g_run->detach_error = ch->detach_error;
    NetChannel_close_ref(ch);
}

/*
 * Returns 0 on success (results in the out-params), < 0 on a harness failure.
 *   wire/len        the byte stream a peer sends on one connection
 *   chunk           bytes per write() (>= 1)
 *   readcache_max   NetChannel_t.readcache_max_size (0 = unlimited, net_reactor.h:100)
 *   decode / glue   glue == NULL: ws_glue around decode; else glue is on_decode
 *   out, msg_len    message bodies back to back, their lengths (max_msgs)
 *   consumed/frames bytes/frames the reactor loop consumed (Σ on_read returns > 0)
 *   detach_error    NetChannel_t.detach_error at detach (0 = still attached at the end)
 *   pending/cached  at the end: fragments still cached (stream_ctx.recvlist non-empty) and
 *                   stream_ctx.cache_recv_bytes (transport_ctx.c:179-201)
 */
__attribute__((visibility("default")))
int ref_reactor_deliver(const unsigned char* wire, unsigned long long len, unsigned int chunk,
                        unsigned int readcache_max, decode_fn decode, on_decode_fn glue,
                        unsigned char* out, unsigned long long out_cap, unsigned long long* msg_len,
                        unsigned int max_msgs, unsigned int* n_msgs, unsigned long long* consumed,
                        unsigned long long* frames, int* detach_error, int* pending, unsigned int* cached) {
    Run R;
    NetChannelProc_t proc;
    NetChannelExProc_t exproc;
    NetChannelExData_t exdata;
    struct NetReactor_t* reactor;
    NetChannel_t* ch;
    NioEv_t ev[16];
    int sp[2], idle = 0, rounds = 0;
    unsigned long long sent = 0;

    memset(&R, 0, sizeof(R));
    R.decode = decode;
    R.out = out; R.out_cap = out_cap; R.msg_len = msg_len; R.max_msgs = max_msgs;
    R.hook = NetChannelEx_get_hook(NET_CHANNEL_SIDE_SERVER, SOCK_STREAM);
    g_run = &R;
    if (chunk == 0) return -1;
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sp)) return -2;
    fcntl(sp[1], F_SETFL, fcntl(sp[1], F_GETFL) | O_NONBLOCK);
    reactor = NetReactor_create();
    if (!reactor) return -3;
    memset(&proc, 0, sizeof(proc));
    proc.on_read = counted_read;
    proc.on_pre_send = R.hook->on_pre_send;
    proc.on_detach = on_detach;
    memset(&exproc, 0, sizeof(exproc));
    exproc.on_decode = glue ? glue : ws_glue;
    exproc.on_recv = rec_recv;
    ch = NetChannel_open_with_fd(NET_CHANNEL_SIDE_SERVER, &proc, sp[0], AF_UNIX, 0);
    if (!ch) return -4;
    NetChannelEx_init(ch, &exdata, &exproc);
    ch->readcache_max_size = readcache_max;
    NetChannel_reg(reactor, ch);

    /* feed the stream; then run the reactor until it has been idle for a few rounds */
    while (!R.detached && (sent < len || idle < 3)) {
        if (sent < len) {
            unsigned long long n = len - sent < chunk ? len - sent : chunk;
            ssize_t w = write(sp[1], wire + sent, (size_t)n);
            if (w > 0) sent += (unsigned long long)w;
            else if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK) break;
        }
        int n = NetReactor_handle(reactor, ev, 16, sent < len ? 0 : 1);
        idle = (n == 0 && sent >= len) ? idle + 1 : 0;
        if (++rounds > 100000000) break;
    }
    *n_msgs = R.n_msgs;
    *consumed = R.consumed;
    *frames = R.frames;
    *detach_error = R.detached ? R.detach_error : 0;
    *pending = ch->stream_ctx.recvlist.head != 0;
    *cached = ch->stream_ctx.cache_recv_bytes;
    if (!R.detached) NetChannel_close_ref(ch);
    close(sp[1]);
    {   /* let the reactor run the channel's free command, then drop it */
        int i;
        for (i = 0; i < 4; ++i) NetReactor_handle(reactor, ev, 16, 0);
    }
    NetReactor_destroy(reactor);
    g_run = 0;
    return R.overrun ? -5 : 0;
}

/* ------------------------------------------------------------------------------------------
 * The GPU batch binding at the reactor, driven over the reference's own
 * reactor and stream hook. The reactor change §2 describes — recv for every readable channel
 * first, then ONE batch decode over every such channel's whole m_inbuf (its undecoded tail from
 * the previous read + the new bytes), then each channel's on_read loop — is emulated around the
 * unmodified reference reactor:
 *   1. NetReactor_handle runs with a capture glue: the first on_decode of a read records the
 *      channel and answers "incomplete", so reactor_stream_readev (net_reactor.c:465-545) has
 *      done its recv and left m_inbuf[0, m_inbuflen) untouched (inbuf_off == 0);
 *   2. one batch over every recorded channel's m_inbuf: `gpu` (websocketframeBatchDecodeHost,
 *      libwsframe_amd.so) or `oracle` (ws_oracle_decode_segments), gathered into one host arena
 *      and scattered back;
 *   3. per channel, the reactor's loop :515-539 restated (on_read = the reference hook, whose
 *      on_decode now replays the batch through `replay` = websocketframeOnDecodeBatch) and its
 *      tail handling (:528-539: memmove of the undecoded tail to the front).
 * Streams are written in `chunk`-byte writes, so frames and headers split across reads and
 * every read's segment starts with the previous read's tail.
 */
#include "../include/wsframe_amd_channel.h"

typedef int (*batch_host_fn)(unsigned char* h_buf, unsigned long long buflen, const unsigned long long* so,
                             const unsigned long long* sl, unsigned int nseg, unsigned int max_frames,
                             WebsocketFrameDesc_t* desc, WebsocketSegResult_t* res, int device);
typedef int (*oracle_batch_fn)(unsigned char* buf, const unsigned long long* so, const unsigned long long* sl,
                               unsigned int nseg, unsigned int max_frames, const unsigned long long* desc_base,
                               WebsocketFrameDesc_t* desc, WebsocketSegResult_t* res);
typedef void (*replay_fn)(WebsocketBatchCursor_t* cur, unsigned char* buf, size_t len,
                          struct NetChannelInbufDecodeResult_t* result);

typedef struct HChan {
    NetChannel_t* ch;
    int sp[2];
    const unsigned char* wire;
    unsigned long long len, sent;
    int replaying, pending_read, detached, detach_error;
    WebsocketBatchCursor_t cur;
    unsigned char* out;
    unsigned long long out_cap, out_len;
    unsigned long long* msg_len;
    unsigned int max_msgs, n_msgs, overrun;
    unsigned long long consumed, frames;
} HChan;

static replay_fn g_replay;

static void bh_glue(NetChannel_t* channel, unsigned char* buf, size_t len, NetChannelInbufDecodeResult_t* r) {
    HChan* h = (HChan*)channel->userdata;
    if (!h->replaying) {             /* 1. capture: the read's bytes stay in m_inbuf for the batch */
        h->pending_read = 1;
        r->incomplete = 1;
        return;
    }
    g_replay(&h->cur, buf, len, (struct NetChannelInbufDecodeResult_t*)r);
}

static void bh_recv(NetChannel_t* channel, unsigned char* bodyptr, size_t bodylen, const struct sockaddr* a,
                    socklen_t al) {
    HChan* h = (HChan*)channel->userdata;
    (void)a; (void)al;
    if (h->n_msgs >= h->max_msgs || h->out_len + bodylen > h->out_cap) { h->overrun = 1; return; }
    if (bodylen) memcpy(h->out + h->out_len, bodyptr, bodylen);
    h->out_len += bodylen;
    h->msg_len[h->n_msgs++] = bodylen;
}

static int bh_read(NetChannel_t* ch, unsigned char* buf, unsigned int len, long long ts, const struct sockaddr* a,
                   socklen_t al) {
    HChan* h = (HChan*)ch->userdata;
    int r = g_run->hook->on_read(ch, buf, len, ts, a, al);
    if (r > 0) { h->consumed += (unsigned int)r; h->frames++; }
    return r;
}

static void bh_detach(NetChannel_t* ch) {
    HChan* h = (HChan*)ch->userdata;
    h->detached = 1;
    h->detach_error = ch->detach_error;
}

/* 3. the reactor loop (net_reactor.c:514-539) over the channel's decoded inbuf */
static void bh_loop(HChan* h) {
    NetReactorObject_t* o = h->ch->o;
    int inbuf_off = 0, res;
    h->replaying = 1;
    while (inbuf_off < o->m_inbuflen) {
        res = h->ch->proc->on_read(h->ch, o->m_inbuf + inbuf_off, o->m_inbuflen - inbuf_off, 0, NULL, 0);
        if (res < 0 || !h->ch->valid) {        /* :518-520: the channel is invalid -> detached */
            h->detached = 1;
            h->detach_error = h->ch->detach_error;
            h->replaying = 0;
            return;
        }
        if (0 == res) break;
        inbuf_off += res;
    }
    if (inbuf_off >= o->m_inbuflen) {
        o->m_inbuflen = 0;
    } else if (inbuf_off > 0) {                /* :536-539 the undecoded tail leads the next read */
        memmove(o->m_inbuf, o->m_inbuf + inbuf_off, o->m_inbuflen - inbuf_off);
        o->m_inbuflen -= inbuf_off;
    }
    h->replaying = 0;
}

/*
 * nch connections, stream c = wires[c][0, lens[c]); per-channel outputs at [c * (cap / nch)],
 * [c * (max_msgs / nch)] and [c]. *batches = batch decodes run. Returns 0, < 0 on a harness
 * failure, > 0 = a batch decode's error code.
 */
__attribute__((visibility("default")))
int ref_reactor_deliver_batched(unsigned int nch, const unsigned char* const* wires, const unsigned long long* lens,
                                unsigned int chunk, unsigned int readcache_max, unsigned int max_frames,
                                batch_host_fn gpu, oracle_batch_fn oracle, replay_fn replay, unsigned char* out,
                                unsigned long long out_cap, unsigned long long* msg_len, unsigned int max_msgs,
                                unsigned int* n_msgs, unsigned long long* consumed, unsigned long long* frames,
                                int* detach_error, int* pending, unsigned int* cached, unsigned int* batches) {
    Run R;
    NetChannelProc_t proc;
    NetChannelExProc_t exproc;
    NetChannelExData_t* exdata;
    struct NetReactor_t* reactor;
    HChan* hc;
    NioEv_t ev[64];
    unsigned int c, nb = 0;
    int idle = 0, rounds = 0, rc = 0;
    if (!nch || !chunk || !replay || (!gpu && !oracle)) return -1;
    memset(&R, 0, sizeof(R));
    R.hook = NetChannelEx_get_hook(NET_CHANNEL_SIDE_SERVER, SOCK_STREAM);
    g_run = &R;
    g_replay = replay;
    hc = (HChan*)calloc(nch, sizeof(HChan));
    exdata = (NetChannelExData_t*)calloc(nch, sizeof(NetChannelExData_t));
    reactor = NetReactor_create();
    if (!hc || !exdata || !reactor) return -3;
    memset(&proc, 0, sizeof(proc));
    proc.on_read = bh_read;
    proc.on_pre_send = R.hook->on_pre_send;
    proc.on_detach = bh_detach;
    memset(&exproc, 0, sizeof(exproc));
    exproc.on_decode = bh_glue;
    exproc.on_recv = bh_recv;
    for (c = 0; c < nch; ++c) {
        HChan* h = &hc[c];
        h->wire = wires[c];
        h->len = lens[c];
        h->out = out + (unsigned long long)c * (out_cap / nch);
        h->out_cap = out_cap / nch;
        h->msg_len = msg_len + (unsigned long long)c * (max_msgs / nch);
        h->max_msgs = max_msgs / nch;
        if (socketpair(AF_UNIX, SOCK_STREAM, 0, h->sp)) return -2;
        fcntl(h->sp[1], F_SETFL, fcntl(h->sp[1], F_GETFL) | O_NONBLOCK);
        h->ch = NetChannel_open_with_fd(NET_CHANNEL_SIDE_SERVER, &proc, h->sp[0], AF_UNIX, 0);
        if (!h->ch) return -4;
        h->ch->userdata = h;
        NetChannelEx_init(h->ch, &exdata[c], &exproc);
        h->ch->readcache_max_size = readcache_max;
        NetChannel_reg(reactor, h->ch);
    }
    for (;;) {
        int feeding = 0, npend = 0;
        for (c = 0; c < nch; ++c) {            /* every peer writes one chunk */
            HChan* h = &hc[c];
            if (h->detached || h->sent >= h->len) continue;
            feeding = 1;
            {
                unsigned long long n = h->len - h->sent < chunk ? h->len - h->sent : chunk;
                ssize_t w = write(h->sp[1], h->wire + h->sent, (size_t)n);
                if (w > 0) h->sent += (unsigned long long)w;
            }
        }
        int n = NetReactor_handle(reactor, ev, 64, feeding ? 0 : 1);   /* 1. recv (+ capture) */
        for (c = 0; c < nch; ++c) npend += hc[c].pending_read && !hc[c].detached && hc[c].ch->o;
        if (npend) {                                                    /* 2. one batch */
            unsigned long long total = 0, *so = (unsigned long long*)calloc(npend, 8),
                               *sl = (unsigned long long*)calloc(npend, 8);
            WebsocketFrameDesc_t* desc = (WebsocketFrameDesc_t*)calloc((size_t)npend * max_frames, sizeof(*desc));
            WebsocketSegResult_t* res = (WebsocketSegResult_t*)calloc(npend, sizeof(*res));
            unsigned char* arena;
            unsigned int k = 0;
            for (c = 0; c < nch; ++c)
                if (hc[c].pending_read && !hc[c].detached && hc[c].ch->o) total += hc[c].ch->o->m_inbuflen;
            arena = (unsigned char*)malloc(total + 64);
            total = 0;
            for (c = 0; c < nch; ++c) {
                HChan* h = &hc[c];
                if (!(h->pending_read && !h->detached && h->ch->o)) continue;
                so[k] = total;
                sl[k] = (unsigned long long)h->ch->o->m_inbuflen;
                memcpy(arena + total, h->ch->o->m_inbuf, sl[k]);
                total += sl[k++];
            }
            memset(arena + total, 0, 64);
            rc = gpu ? gpu(arena, total, so, sl, npend, max_frames, desc, res, 0)
                     : oracle(arena, so, sl, npend, max_frames, NULL, desc, res);
            ++nb;
            k = 0;
            for (c = 0; c < nch && !rc; ++c) {                          /* 3. each channel's loop */
                HChan* h = &hc[c];
                if (!(h->pending_read && !h->detached && h->ch->o)) continue;
                memcpy(h->ch->o->m_inbuf, arena + so[k], sl[k]);
                h->cur.desc = desc + (size_t)k * max_frames;
                h->cur.res = res[k];
                h->cur.seg_off = so[k];
                h->cur.inbuf = h->ch->o->m_inbuf;
                h->cur.next = 0;
                h->pending_read = 0;
                ++k;
                bh_loop(h);
            }
            free(arena); free(so); free(sl); free(desc); free(res);
            if (rc) break;
        }
        {
            int more = 0;
            for (c = 0; c < nch; ++c) more |= !hc[c].detached && hc[c].sent < hc[c].len;
            idle = (!more && n == 0 && !npend) ? idle + 1 : 0;
            if (!more && idle >= 3) break;
        }
        if (++rounds > 10000000) { rc = -6; break; }
    }
    for (c = 0; c < nch; ++c) {
        HChan* h = &hc[c];
        n_msgs[c] = h->n_msgs;
        consumed[c] = h->consumed;
        frames[c] = h->frames;
        detach_error[c] = h->detached ? h->detach_error : 0;
        pending[c] = h->ch->stream_ctx.recvlist.head != 0;
        cached[c] = h->ch->stream_ctx.cache_recv_bytes;
        if (h->overrun && !rc) rc = -5;
        NetChannel_close_ref(h->ch);
        close(h->sp[1]);
    }
    for (c = 0; c < 4; ++c) NetReactor_handle(reactor, ev, 64, 0);
    NetReactor_destroy(reactor);
    *batches = nb;
    free(hc);
    free(exdata);
    g_run = 0;
    return rc;
}
